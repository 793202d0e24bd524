"""Host runtime for the EfficientDet hot path: buffers, lazy activations, parameters, tape.

Design:
  * Every activation is an ``Act``: a raw NHWC buffer ``[rows][ld]`` plus an optional
    *pending* per-channel transform ``v = act(bn(raw)) * gate`` that consumers apply while
    loading.  Training-mode BatchNorm therefore never runs as its own forward pass: the
    producing kernel emits per-channel sums, the consuming kernel normalises.
  * ``Pyr`` is the row layout of an activation: one segment for a plain tensor, five for the
    P3..P7 feature pyramid the heads run over in single launches.
  * ``ParamStore`` keeps every trainable variable in one flat fp32 buffer (master weights),
    a flat gradient buffer (one all-reduce for data parallelism), momentum / EMA slots and a
    compute-dtype copy for the kernels; BN moving statistics and per-step batch statistics
    live in their own flat arenas so each is zeroed / updated by one launch.
  * ``Tape`` records one backward closure per forward op (explicit reverse-mode AD on the
    static EfficientDet graph; no torch.autograd).  Gradients of an activation accumulate in
    place through the kernels' ``accumulate`` flag.

PyTorch is used only for device memory (caching allocator) and streams.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L

ROW_ALIGN = 128  # segment starts of a pyramid buffer (GEMM row tiles never straddle levels)
PARAM_ALIGN = 64  # elements; keeps every weight view 256-B aligned


def _vp(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


# --------------------------------------------------------------------------- layout
class Pyr:
    """Row layout: segment s holds batch*H*W rows starting at a 128-aligned offset."""

    def __init__(self, batch: int, sizes: Sequence[Tuple[int, int]]):
        assert 1 <= len(sizes) <= L.MAX_SEG
        self.batch = int(batch)
        self.sizes = [(int(h), int(w)) for h, w in sizes]
        self.nseg = len(self.sizes)
        self.row_off: List[int] = []
        off = 0
        for h, w in self.sizes:
            self.row_off.append(off)
            off = round_up(off + self.batch * h * w, ROW_ALIGN)
        self.rows = self.row_off[-1] + self.seg_rows(self.nseg - 1)
        c = L.Pyramid()
        c.nseg, c.batch = self.nseg, self.batch
        for i, (h, w) in enumerate(self.sizes):
            c.row_off[i], c.H[i], c.W[i] = self.row_off[i], h, w
        self.c = c

    def seg_rows(self, s: int) -> int:
        h, w = self.sizes[s]
        return self.batch * h * w

    def seg_slice(self, s: int) -> slice:
        return slice(self.row_off[s], self.row_off[s] + self.seg_rows(s))

    def strided(self, s: int) -> "Pyr":
        return Pyr(self.batch, [((h + s - 1) // s, (w + s - 1) // s) for h, w in self.sizes])

    @property
    def H(self):
        assert self.nseg == 1
        return self.sizes[0][0]

    @property
    def W(self):
        assert self.nseg == 1
        return self.sizes[0][1]

    def __repr__(self):
        return f"Pyr(batch={self.batch}, sizes={self.sizes})"


# --------------------------------------------------------------------------- BN
class BNParam:
    """One Keras BatchNormalization (momentum 0.99, eps 1e-3 by default)."""

    def __init__(self, name: str, C: int, momentum: float, eps: float):
        self.name, self.C, self.momentum, self.eps = name, C, momentum, eps
        self.gamma = self.beta = self.dgamma = self.dbeta = None
        self.mmean = self.mvar = self.count = None
        self.tsum = self.tsq = None    # batch statistics (training), replicated (L.stat_len(C))
        self.isum = self.isq = None    # moving statistics as sums (inference), replicated
        self.coff = -1                 # channel offset in the BN arenas (a multiple of 16)

    def stats(self, training: bool):
        return (self.tsum, self.tsq) if training else (self.isum, self.isq)


# --------------------------------------------------------------------------- activations
class SERec:
    """Saved state of one squeeze-excitation (layers/se.py) for its backward."""

    def __init__(self, s, z1, gate, w1, b1, w2, b2, dw1, db1, dw2, db2, R):
        self.s, self.z1, self.gate = s, z1, gate
        self.w1, self.b1, self.w2, self.b2 = w1, b1, w2, b2
        self.dw1, self.db1, self.dw2, self.db2 = dw1, db1, dw2, db2
        self.R = R


class Act:
    """Raw activation buffer + pending transform v = act(bn(raw)) * gate."""

    __slots__ = ("raw", "pyr", "C", "ld", "bns", "act", "gate", "se", "training", "name", "_lz", "uses", "se_source")

    def __init__(self, raw: torch.Tensor, pyr: Pyr, C: int, bns: Optional[List[BNParam]] = None,
                 act: int = L.ACT_NONE, ld: Optional[int] = None, training: bool = False,
                 name: str = ""):
        self.raw, self.pyr, self.C = raw, pyr, C
        self.ld = C if ld is None else ld
        assert raw.dim() == 2 and raw.shape[0] >= pyr.rows and raw.shape[1] == self.ld, (raw.shape, pyr.rows, self.ld)
        self.bns = bns
        if bns is not None:
            assert len(bns) == pyr.nseg
        self.act, self.gate, self.se = act, None, None
        self.training, self.name = training, name
        self._lz = None
        self.uses = 0  # forward ops that will send a gradient into this value (consume())
        # a plain copy of an SE-gated value (ops.materialize): that value's Act, whose backward
        # sums the consumer's dgrad may take in its epilogue (edet_conv1x1_dgrad_sesum)
        self.se_source = None

    def consume(self) -> "Act":
        """Count a training-mode consumer: a backward that owns the whole gradient of the
        value (uses == 1) may fold the value's BN-backward sums into its own pass."""
        if self.training:
            self.uses += 1
        return self

    @property
    def has_transform(self) -> bool:
        return self.bns is not None or self.act != L.ACT_NONE or self.gate is not None

    def set_gate(self, gate: torch.Tensor, se: SERec):
        self.gate, self.se, self._lz = gate, se, None

    def lazy(self) -> L.Lazy:
        if self._lz is None:
            lz = L.Lazy()
            lz.x = self.raw.data_ptr()
            lz.gate = self.gate.data_ptr() if self.gate is not None else None
            lz.ld = self.ld
            lz.act = self.act
            if self.bns is not None:
                lz.bn.enabled = 1
                lz.bn.eps = self.bns[0].eps
                for s, bn in enumerate(self.bns):
                    ssum, ssq = bn.stats(self.training)
                    lz.bn.sum[s] = ssum.data_ptr()
                    lz.bn.sq[s] = ssq.data_ptr()
                    lz.bn.gamma[s] = bn.gamma.data_ptr()
                    lz.bn.beta[s] = bn.beta.data_ptr()
            self._lz = lz
        return self._lz

    def seg_view(self, s: int) -> torch.Tensor:
        return self.raw[self.pyr.seg_slice(s), : self.C]

    def __repr__(self):
        return f"Act({self.name}, C={self.C}, {self.pyr})"


def seg_out(pairs: Sequence[Tuple[torch.Tensor, torch.Tensor]]) -> L.SegOut:
    so = L.SegOut()
    for i, (a, b) in enumerate(pairs):
        so.a[i] = a.data_ptr()
        so.b[i] = b.data_ptr()
    return so


def stat_out(pairs: Sequence[Tuple[torch.Tensor, torch.Tensor]]) -> L.StatOut:
    """Per-segment fp64 (sum, sum of squares) BN statistics destinations of a producer."""
    so = L.StatOut()
    for i, (a, b) in enumerate(pairs):
        assert a.dtype == torch.float64 and b.dtype == torch.float64
        so.sum[i], so.sq[i] = a.data_ptr(), b.data_ptr()
    return so


# --------------------------------------------------------------------------- parameters
class ParamSpec:
    __slots__ = ("name", "shape", "init", "l2", "offset", "size", "pw", "toff")

    def __init__(self, name, shape, init, l2, pw=False):
        self.name, self.shape, self.init, self.l2 = name, tuple(shape), init, l2
        self.size = int(np.prod(self.shape))
        self.offset = -1
        self.pw = pw      # 1x1 conv kernel [N][K]: also kept transposed for the dgrad GEMM
        self.toff = -1


class ParamStore:
    """Flat fp32 master weights / grads / momentum / EMA + compute-dtype copy + BN arenas.

    Variables matching the reference's L2 regex (``.*(kernel|weight):0$``,
    efficientdet_net_train.py:21) are laid out first so the fused optimizer applies the
    4e-5 * w gradient term to one prefix.
    """

    def __init__(self):
        self.specs: Dict[str, ParamSpec] = {}
        self.order: List[str] = []
        self.bns: List[BNParam] = []
        self.finalized = False

    # ---- registration
    def add(self, name: str, shape, init, l2: bool, pw: bool = False) -> str:
        assert not self.finalized and name not in self.specs, name
        self.specs[name] = ParamSpec(name, shape, init, l2, pw)
        self.order.append(name)
        return name

    def add_bn(self, name: str, C: int, momentum: float, eps: float) -> BNParam:
        bn = BNParam(name, C, momentum, eps)
        self.add(name + "/gamma", (C,), ("const", 1.0), False)
        self.add(name + "/beta", (C,), ("const", 0.0), False)
        self.bns.append(bn)
        return bn

    # ---- allocation
    def finalize(self, device, compute_dtype: torch.dtype, seed: int = 0):
        assert not self.finalized
        names = [n for n in self.order if self.specs[n].l2] + [n for n in self.order if not self.specs[n].l2]
        off = 0
        self.n_l2 = 0
        for n in names:
            sp = self.specs[n]
            sp.offset = off
            off = round_up(off + sp.size, PARAM_ALIGN)
            if sp.l2:
                self.n_l2 = off
        self.numel = off
        self.n_trainable = sum(sp.size for sp in self.specs.values())
        host = np.zeros(self.numel, np.float32)
        rng = np.random.default_rng(seed)
        for n in self.order:  # init in registration order (deterministic per model)
            sp = self.specs[n]
            host[sp.offset: sp.offset + sp.size] = _init_values(sp, rng).reshape(-1)
        self.device = device
        self.w = torch.from_numpy(host).to(device)
        self.g = torch.zeros_like(self.w)
        self.v = torch.zeros_like(self.w)
        self.ema = self.w.clone()
        self.compute_dtype = compute_dtype
        if compute_dtype == torch.float32:
            self.wc = self.w
        else:
            self.wc = torch.empty(self.numel, dtype=compute_dtype, device=device)
        # transposed compute copies of the 1x1 kernels ([K][roundup(N,8)]) for dgrad
        toff, table, max_tiles = 0, [], 0
        for n in names:
            sp = self.specs[n]
            if sp.pw:
                N, K = sp.shape
                sp.toff = toff
                ldn = round_up(N, 8)
                toff = round_up(toff + K * ldn, PARAM_ALIGN)
                table.append([sp.offset, sp.toff, N, K])
                max_tiles = max(max_tiles, ((N + 31) // 32) * ((K + 31) // 32))
        self.wct = torch.empty(max(toff, 1), dtype=compute_dtype, device=device)
        self.t_table = torch.tensor(np.asarray(table, np.int64).reshape(-1, 4), device=device)
        self.t_entries, self.t_max_tiles = len(table), max_tiles
        # BN arenas: every BN's channels start on a multiple of 16, so one channel index space
        # (padding channels: count 1, statistics 0) serves the per-channel arrays and the
        # replicated fp64 statistics (include/edet.h "Statistics vectors": channel c of the
        # arena at L.stat_idx(c, r), each BN's vector a contiguous L.stat_len(C) slice)
        o = 0
        for bn in self.bns:
            bn.coff = o
            o += round_up(bn.C, 16)
        nch = max(o, 16)
        self.n_bn = nch
        self.bn_mm = torch.zeros(nch, device=device)
        self.bn_mv = torch.ones(nch, device=device)
        self.bn_count = torch.ones(nch, device=device)
        self.bn_tstats = torch.zeros(2, L.stat_len(nch), dtype=torch.float64, device=device)
        self.bn_istats = torch.zeros(2, L.stat_len(nch), dtype=torch.float64, device=device)
        for bn in self.bns:
            sl = slice(bn.coff, bn.coff + bn.C)
            ssl = slice(bn.coff * L.STAT_REPLICAS, bn.coff * L.STAT_REPLICAS + L.stat_len(bn.C))
            bn.gamma, bn.beta = self.view(bn.name + "/gamma"), self.view(bn.name + "/beta")
            bn.dgamma, bn.dbeta = self.grad(bn.name + "/gamma"), self.grad(bn.name + "/beta")
            bn.mmean, bn.mvar, bn.count = self.bn_mm[sl], self.bn_mv[sl], self.bn_count[sl]
            bn.tsum, bn.tsq = self.bn_tstats[0, ssl], self.bn_tstats[1, ssl]
            bn.isum, bn.isq = self.bn_istats[0, ssl], self.bn_istats[1, ssl]
        self.finalized = True
        if torch.device(device).type == "cuda":
            ensure_workspace(device)
            self.refresh_compute_copy()
        # else: host-only store (model structure + initial parameters for CPU tools/tests);
        # the model refuses to run its compute path on it.

    def refresh_compute_copy(self, cast: bool = True):
        dt = L.F32 if self.compute_dtype == torch.float32 else L.BF16
        if cast and self.wc is not self.w:
            L.call("edet_cast_f32", dt, _vp(self.w), _vp(self.wc), self.numel, stream())
        L.call("edet_transpose_cast", dt, _vp(self.w), _vp(self.wct), _vp(self.t_table), self.t_entries,
               self.t_max_tiles, stream())

    # ---- views
    def _sl(self, name):
        sp = self.specs[name]
        return slice(sp.offset, sp.offset + sp.size), sp.shape

    def view(self, name) -> torch.Tensor:
        sl, shape = self._sl(name)
        return self.w[sl].view(shape)

    def grad(self, name) -> torch.Tensor:
        sl, shape = self._sl(name)
        return self.g[sl].view(shape)

    def wcv(self, name) -> torch.Tensor:
        sl, shape = self._sl(name)
        return self.wc[sl].view(shape)

    def wtv(self, name) -> torch.Tensor:
        """Transposed compute copy [K][roundup(N,8)] of a 1x1 kernel."""
        sp = self.specs[name]
        N, K = sp.shape
        ldn = round_up(N, 8)
        return self.wct[sp.toff: sp.toff + K * ldn].view(K, ldn)

    # ---- host round trip (checkpoints, oracle parity)
    def state_dict(self) -> Dict[str, np.ndarray]:
        host = self.w.detach().float().cpu().numpy()
        out = {n: host[self.specs[n].offset: self.specs[n].offset + self.specs[n].size].reshape(self.specs[n].shape).copy()
               for n in self.order}
        mm, mv = self.bn_mm.cpu().numpy(), self.bn_mv.cpu().numpy()
        for bn in self.bns:
            out[bn.name + "/moving_mean"] = mm[bn.coff:bn.coff + bn.C].copy()
            out[bn.name + "/moving_variance"] = mv[bn.coff:bn.coff + bn.C].copy()
        return out

    def load_state_dict(self, sd: Dict[str, np.ndarray]):
        host = self.w.detach().cpu().numpy().copy()
        for n in self.order:
            sp = self.specs[n]
            a = np.asarray(sd[n], np.float32).reshape(-1)
            assert a.size == sp.size, (n, a.size, sp.size)
            host[sp.offset: sp.offset + sp.size] = a
        self.w.copy_(torch.from_numpy(host))
        self.ema.copy_(self.w)
        mm, mv = self.bn_mm.cpu().numpy(), self.bn_mv.cpu().numpy()
        for bn in self.bns:
            if bn.name + "/moving_mean" in sd:
                mm[bn.coff:bn.coff + bn.C] = sd[bn.name + "/moving_mean"]
                mv[bn.coff:bn.coff + bn.C] = sd[bn.name + "/moving_variance"]
        self.bn_mm.copy_(torch.from_numpy(mm))
        self.bn_mv.copy_(torch.from_numpy(mv))
        self.refresh_compute_copy()

    def grads_dict(self) -> Dict[str, np.ndarray]:
        host = self.g.detach().cpu().numpy()
        return {n: host[self.specs[n].offset: self.specs[n].offset + self.specs[n].size].reshape(self.specs[n].shape).copy()
                for n in self.order}


def _init_values(sp: ParamSpec, rng: np.random.Generator) -> np.ndarray:
    """Reference initialisers."""
    kind = sp.init[0]
    shape = sp.shape
    if kind == "const":
        return np.full(shape, sp.init[1], np.float32)
    if kind == "normal":  # utils/conv_kernel_initializer.py: N(0, sqrt(2 / fan_out))
        return rng.normal(0.0, sp.init[1], size=shape).astype(np.float32)
    if kind == "glorot":  # keras glorot_uniform: U(-l, l), l = sqrt(6 / (fan_in + fan_out))
        lim = math.sqrt(6.0 / (sp.init[1] + sp.init[2]))
        return rng.uniform(-lim, lim, size=shape).astype(np.float32)
    if kind == "vs_fan_in":  # keras VarianceScaling(): truncated normal, std sqrt(1/fan_in)/0.8796
        std = math.sqrt(1.0 / sp.init[1]) / 0.87962566103423978
        v = rng.normal(0.0, std, size=shape)
        bad = np.abs(v) > 2 * std
        while bad.any():
            v[bad] = rng.normal(0.0, std, size=int(bad.sum()))
            bad = np.abs(v) > 2 * std
        return v.astype(np.float32)
    raise ValueError(sp.init)


# --------------------------------------------------------------------------- tape
class GradRec:
    __slots__ = ("t", "ld", "scale", "bn_sums", "se_sums")

    def __init__(self, t: torch.Tensor, ld: int, scale: Optional[torch.Tensor] = None):
        self.t, self.ld, self.scale = t, ld, scale
        # fp64 [2][nseg][C] (dgamma, dbeta) BN-backward sums of the value's BatchNorm, already
        # accumulated by the kernel that wrote t (edet_dwconv_bwd's fold); None: not yet
        self.bn_sums = None
        # fp64 [5][B][C] SE-gated value sums (edet_gate_bn_reduce's), taken by the kernel that
        # wrote t (edet_conv1x1_dgrad_sesum); None: not yet
        self.se_sums = None


class Tape:
    """Explicit reverse-mode AD: one closure per forward op, run in reverse order."""

    def __init__(self, engine: "Engine", trace: Optional[list] = None):
        self.eng = engine
        self.entries: List = []
        self.g: Dict[Act, GradRec] = {}
        self.trace = trace  # debug: list receiving (act name, fp32 copy of d(value)) per take()
        # work gathered over the backward and launched once after the last closure:
        # key -> (fn(items), items) (the BiFPN fusion weight-gradient fold, ops.bifpn_fuse)
        self.finals: Dict[str, Tuple] = {}

    def record(self, fn):
        self.entries.append(fn)

    def dst(self, act: Act) -> Tuple[torch.Tensor, int]:
        """Destination for d(value of act): (buffer [rows][C], accumulate flag)."""
        rec = self.g.get(act)
        if rec is not None:
            assert rec.scale is None and rec.ld == act.C, "cannot accumulate into a scaled/strided grad"
            # a folded gradient already carries its BN-backward sums: a later contribution would
            # not be in them (a forward op that sends a gradient into `act` skipped consume())
            assert rec.bn_sums is None, f"gradient of {act} was folded; a later consumer cannot accumulate into it"
            return rec.t, 1
        t = self.eng.empty(act.pyr.rows, act.C)
        self.g[act] = GradRec(t, act.C)
        return t, 0

    def alias(self, act: Act, t: torch.Tensor, ld: int, scale=None, se_sums=None):
        assert act not in self.g, f"grad of {act} already exists"
        self.g[act] = GradRec(t, ld, scale)
        self.g[act].se_sums = se_sums

    def take(self, act: Act) -> Optional[GradRec]:
        rec = self.g.pop(act, None)
        if self.trace is not None and rec is not None:
            rows = [rec.t[act.pyr.seg_slice(s), : act.C].float() for s in range(act.pyr.nseg)]
            self.trace.append((act.name, torch.cat(rows, 0).clone(), None if rec.scale is None else rec.scale.clone()))
        return rec

    def collect(self, key: str, fn, item):
        """Add `item` to the list `fn` receives once, after every backward closure has run."""
        self.finals.setdefault(key, (fn, []))[1].append(item)

    def backward(self):
        entries, self.entries = self.entries, []
        # the weight-gradient split sums are deferred to one launch after the last closure
        # (edet_partials_defer / _flush): nothing reads a weight gradient before the optimizer
        arena = self.eng.partials_arena()
        if arena is not None:
            L.call("edet_partials_defer", _vp(arena), arena.numel())
        try:
            for fn in reversed(entries):
                fn()
            finals, self.finals = self.finals, {}
            for fn, items in finals.values():
                fn(items)
            self.g.clear()
            self.eng.join_side()
        finally:
            if arena is not None:
                need = ctypes.c_size_t(0)
                L.call("edet_partials_flush", ctypes.byref(need), stream())
                self.eng.note_partials(need.value)


# --------------------------------------------------------------------------- engine
# EDET_DEFER_PARTIALS=0: every weight-gradient split sum launched right after its kernel (the
# round-5 behaviour), for same-box A/B
DEFER_PARTIALS = os.environ.get("EDET_DEFER_PARTIALS", "1") != "0"
# EDET_OVERLAP=1: weight gradients on the side stream (Engine.overlap), for same-box A/B
OVERLAP = os.environ.get("EDET_OVERLAP", "0") == "1"
_WORKSPACE = {}
WORKSPACE_BYTES = 64 << 20


def ensure_workspace(device) -> torch.Tensor:
    """Register the library's split-reduction scratch (edet_set_workspace) for this process.
    Allocated once per device and never freed, so the registered pointer cannot dangle; the
    weight-gradient kernels use it instead of atomics (deterministic sums)."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    ws = _WORKSPACE.get(idx)
    if ws is None:
        ws = torch.empty(WORKSPACE_BYTES, dtype=torch.uint8, device=dev)
        _WORKSPACE[idx] = ws
    L.call("edet_set_workspace", _vp(ws), WORKSPACE_BYTES)
    return ws


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class Engine:
    """Per-model execution context: compute dtype, device, training flag, tape."""

    def __init__(self, dtype: str, device):
        assert dtype in ("bf16", "f32")
        self.dt = L.BF16 if dtype == "bf16" else L.F32
        self.tdtype = torch.bfloat16 if dtype == "bf16" else torch.float32
        self.device = torch.device(device)
        self.training = False
        self.tape: Optional[Tape] = None
        # fp64 accumulators (SE squeeze / gate gradient, BN-backward sums) are bump-allocated
        # from one arena zeroed by a single memset per forward (begin_scratch) instead of one
        # fill kernel each
        self._s64: Optional[torch.Tensor] = None
        self._s64_off = 0
        self._s64_need = 1 << 20
        self._s64_hw = 0  # high-water mark over all steps: the extent the memset must cover
        self._s64_overflow = []
        # Optional: weight gradients on a side stream (off the backward critical path: nothing
        # in the step reads them before the optimizer).  Tensors they read stay referenced
        # until join_side() orders the main stream after them, so the caching allocator cannot
        # hand their memory to a main-stream op while a side kernel may still read it.  Off by
        # default: measured 1351 vs 1388 img/s (D0 b32) -- the wide side kernels take the CUs
        # the main chain needs instead of filling idle ones.
        self.overlap = OVERLAP
        self._side = None
        self._side_used = False
        self._side_keep: list = []
        self._parts: Optional[torch.Tensor] = None
        self._parts_need = 256 << 20

    def partials_arena(self) -> Optional[torch.Tensor]:
        """Arena of the deferred weight-gradient split partials (edet_partials_defer), sized by
        the previous backward's need (256 MB to start; D0 B = 32 uses ~0.1 GB).  None: deferral
        off (EDET_DEFER_PARTIALS=0, or a library without it)."""
        if not DEFER_PARTIALS or self.device.type != "cuda" or not L.has("edet_partials_defer"):
            return None
        if self._parts is None or self._parts.numel() < self._parts_need:
            self._parts = torch.empty(self._parts_need, dtype=torch.uint8, device=self.device)
        return self._parts

    def note_partials(self, needed: int):
        """The arena a backward would have used: grow for the next one (this one fell back to
        immediate sums past the arena's end)."""
        if needed > self._parts_need:
            self._parts_need = round_up(int(needed * 1.25), 1 << 20)

    def empty(self, rows: int, C: int, dtype=None) -> torch.Tensor:
        return torch.empty((rows, C), dtype=dtype or self.tdtype, device=self.device)

    def begin_scratch(self):
        """Start of a forward: rewind the fp64 arena and zero it (one memset)."""
        self._s64_hw = max(self._s64_hw, self._s64_off)
        if self._s64 is None or self._s64.numel() < self._s64_need:
            self._s64 = torch.empty(self._s64_need, dtype=torch.float64, device=self.device)
            self._s64_hw = self._s64.numel()
        self._s64_off = 0
        self._s64_overflow = []
        memset0(self._s64[: min(self._s64_hw, self._s64.numel())])

    def zeros64(self, *shape) -> torch.Tensor:
        """Zeroed fp64 scratch valid until the next begin_scratch()."""
        n = int(np.prod(shape))
        start = round_up(self._s64_off, 32)  # 256-B aligned views
        if self._s64 is not None and start + n <= self._s64.numel():
            self._s64_off = start + n
            return self._s64[start:start + n].view(shape)
        # arena too small this step: plain zeroed tensor now, a larger arena from the next step
        self._s64_need = max(self._s64_need, 2 * (start + n))
        self._s64_off = start + n
        t = torch.zeros(shape, dtype=torch.float64, device=self.device)
        self._s64_overflow.append(t)
        return t

    def zeros_f32(self, *shape) -> torch.Tensor:
        t = torch.empty(shape, dtype=torch.float32, device=self.device)
        memset0(t)
        return t

    def record(self, fn):
        if self.training and self.tape is not None:
            self.tape.record(fn)

    def side(self, *keep):
        """Context for a weight-gradient launch: the side stream after the main stream's work
        so far (or the main stream itself when overlap is off)."""
        import contextlib
        if not self.overlap:
            return contextlib.nullcontext()
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        self._side.wait_stream(torch.cuda.current_stream(self.device))
        self._side_keep.extend(keep)
        self._side_used = True
        return torch.cuda.stream(self._side)

    def join_side(self):
        """Order the main stream after every side-stream launch; release their operands."""
        if self._side_used:
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            self._side_used = False
        self._side_keep.clear()


def memset0_many(ts):
    """Zero several device tensors in one launch (edet_zero_ranges), or one fill each with a
    library that lacks it."""
    ts = [t for t in ts if t.numel()]
    if not L.has("edet_zero_ranges") or len(ts) > 8 or any(t.data_ptr() % 16 for t in ts):
        for t in ts:
            memset0(t)
        return
    n = len(ts)
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
    sizes = (ctypes.c_size_t * n)(*[t.numel() * t.element_size() for t in ts])
    L.call("edet_zero_ranges", n, ptrs, sizes, stream())


def memset0(t: torch.Tensor):
    L.call("edet_memset_async", _vp(t), 0, t.numel() * t.element_size(), stream())


def memcpy(dst: torch.Tensor, src: torch.Tensor):
    n = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() >= n
    L.call("edet_memcpy_async", _vp(dst), _vp(src), n, stream())


vp = _vp
