"""Forward ops of the EfficientDet hot path, each with its recorded backward.

Every function launches libedet kernels on the current stream and, in training mode,
records a closure on the engine's tape that turns d(output value) into d(input values) and
accumulates weight gradients into the flat fp32 gradient buffer.

Reference call sites replaced (AIServer/ai_api/ai_models/...):
  stem            layers/stem.py:37-38
  conv1x1         layers/mb_conv_block.py:143-154, layers/resample_feature_map.py:43-47,
                  pointwise halves of SeparableConv2D (bifpn.py:27, class_net.py:89,97, box_net.py:90,97)
  dwconv          layers/mb_conv_block.py:147, depthwise halves of the SeparableConv2Ds
  squeeze_excite  layers/se.py:35-39
  maxpool         layers/resample_feature_map.py:48-49
  bifpn_fuse      layers/bifpn.py:59-66 (+ the swish of OpAfterCombine, bifpn.py:26)
  residual        layers/class_net.py:93-96, layers/box_net.py:93-95
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple


import torch

from . import _lib as L
from .runtime import Act, BNParam, Engine, GradRec, ParamStore, Pyr, SERec, memset0, seg_out, stat_out, stream, vp


def _stats_out(eng: Engine, bns: Optional[List[BNParam]]):
    if bns is None or not eng.training:
        return None
    return stat_out([(bn.tsum, bn.tsq) for bn in bns])


def _bn_grads(bns: List[BNParam]):
    return seg_out([(bn.dgamma, bn.dbeta) for bn in bns])


def _value_grad_tables(eng: Engine, out: Act, rec: GradRec):
    """The passes d(value) -> d(raw) needs before its apply: the SE gate gradient and SE backward
    (dsq), and the BN-backward sums (reduce pass, or folded earlier / into the SE pass).
    Returns (dsq or None, fp64 edet_bngrad64 sums or None, fp32 gamma/beta gradient SegOut or None)."""
    s = stream()
    lz = out.lazy()
    dsq = None
    # SE-gated swish(BN) value: the gate gradient and the BN-backward sums come out of one
    # pass over (x, dv) (edet_gate_bn_reduce); no separate reduce pass
    fused_se = (out.se is not None and out.bns is not None and len(out.bns) == 1 and out.act == L.ACT_SWISH
                and rec.scale is None and out.C <= 2048)
    sums5 = None
    if out.se is not None:
        se = out.se
        B = out.pyr.batch
        HW = out.pyr.H * out.pyr.W
        if fused_se and rec.se_sums is not None:  # taken by the dgrad that wrote dv
            sums5 = rec.se_sums
            dgate = sums5[0]
        elif fused_se:
            sums5 = eng.zeros64(5, B, out.C)
            L.call("edet_gate_bn_reduce", eng.dt, lz, B, HW, out.C, vp(rec.t), vp(sums5), s)
            dgate = sums5[0]
        else:
            dgate = eng.zeros64(B, out.C)
            L.call("edet_gate_grad", eng.dt, lz, B, HW, out.C, vp(rec.t), vp(dgate), s)
    grads = acc = None
    folded = rec.bn_sums is not None
    if out.bns is not None:
        grads = _bn_grads(out.bns)
        # fp64 dgamma/dbeta sums (edet_bngrad64): their order must not reach the rounding of dx
        acc_t = rec.bn_sums if folded else eng.zeros64(2, len(out.bns), L.stat_len(out.C))
        acc = L.BnGrad64()
        for i in range(len(out.bns)):
            acc.dgamma[i], acc.dbeta[i] = acc_t[0, i].data_ptr(), acc_t[1, i].data_ptr()
    if out.se is not None:
        dsq = torch.empty((B, out.C), dtype=torch.float32, device=eng.device)
        dz1 = torch.empty((B, se.R), dtype=torch.float32, device=eng.device)
        args = (B, out.C, se.R, HW, vp(se.s), vp(se.z1), vp(se.gate), vp(dgate), vp(se.w1), vp(se.w2),
                vp(se.dw1), vp(se.db1), vp(se.dw2), vp(se.db2), vp(dsq), vp(dz1))
        if fused_se:  # SE backward + the BN sums from sums5 (edet_se_bn_combine) in two launches
            L.call("edet_se_bwd_bn", *args, vp(sums5), acc, s)
        else:
            L.call("edet_se_bwd", *args, s)
    if out.bns is not None and not fused_se and not folded:
        L.call("edet_lazy_bwd_reduce", eng.dt, lz, out.pyr.c, out.C, vp(rec.t), vp(rec.scale), vp(dsq), acc, s)
    return dsq, acc, grads


def value_grad_to_raw(eng: Engine, out: Act, rec: GradRec) -> Tuple[torch.Tensor, int]:
    """d(value) -> d(raw) through the lazy transform act(bn(raw)) * gate (+ SE branch)."""
    if not out.has_transform and rec.scale is None:
        return rec.t, rec.ld
    assert rec.ld == out.C
    dsq, acc, grads = _value_grad_tables(eng, out, rec)
    dx = eng.empty(out.pyr.rows, out.C)
    L.call("edet_lazy_bwd_apply", eng.dt, out.lazy(), out.pyr.c, out.C, vp(rec.t), vp(rec.scale), vp(dsq), acc, grads,
           vp(dx), 0, stream())
    return dx, out.C


def value_grad_lazy(eng: Engine, out: Act, rec: GradRec) -> Tuple[L.DgradLazy, list]:
    """d(value) -> the edet_dgrad_lazy descriptor of d(raw): the same passes as
    value_grad_to_raw without its apply; the consumer builds d(raw) on load
    (edet_dwconv_bwd_lazy).  Returns the descriptor and the tensors it points into."""
    assert rec.ld == out.C and rec.scale is None
    dsq, acc, grads = _value_grad_tables(eng, out, rec)
    d = L.DgradLazy()
    d.dv = rec.t.data_ptr()
    d.y = out.lazy()
    d.dsq = dsq.data_ptr() if dsq is not None else None
    if acc is not None:
        d.acc = acc
        d.grads = grads
    return d, [rec.t, dsq]


# --------------------------------------------------------------------------- stem
def stem(eng: Engine, P: ParamStore, x: torch.Tensor, wname: str, bn: BNParam) -> Act:
    """Conv 3x3 s2 SAME (no bias) -> BN -> swish.  x: [B, H, W, 3] in the compute dtype."""
    B, H, W, _ = x.shape
    Cout = bn.C
    pyr = Pyr(B, [((H + 1) // 2, (W + 1) // 2)])
    y = eng.empty(pyr.rows, Cout)
    if eng.training:
        L.call("edet_stem_fwd", eng.dt, vp(x), B, H, W, vp(P.wcv(wname)), Cout, vp(y), vp(bn.tsum), vp(bn.tsq), stream())
    else:
        scratch = eng.zeros64(2, L.stat_len(Cout))
        L.call("edet_stem_fwd", eng.dt, vp(x), B, H, W, vp(P.wcv(wname)), Cout, vp(y), vp(scratch[0]),
               vp(scratch[1]), stream())
    out = Act(y, pyr, Cout, [bn], L.ACT_SWISH, training=eng.training, name="stem")

    def bwd():
        rec = eng.tape.take(out)
        if rec is None:
            return
        d, ld = value_grad_to_raw(eng, out, rec)
        assert ld == Cout
        with eng.side(x, d):
            L.call("edet_stem_wgrad", eng.dt, vp(x), B, H, W, vp(d), Cout, vp(P.grad(wname)), stream())

    eng.record(bwd)
    return out


# --------------------------------------------------------------------------- 1x1 conv
# output width from which the weight gradient reads a materialized copy of a lazy A operand
# (scripts/kbench.py)
WGRAD_MATERIALIZE_N = int(os.environ.get("EDET_WGRAD_MATERIALIZE_N", "64"))


def conv1x1(eng: Engine, P: ParamStore, x: Act, wname: str, N: int, bname: Optional[str] = None,
            bns: Optional[List[BNParam]] = None, act: int = L.ACT_NONE, ldy: Optional[int] = None,
            out_buf: Optional[torch.Tensor] = None, name: str = "") -> Act:
    """y = v(x) @ W^T (+ b); output is lazy BN/act when ``bns`` given.  W stored [N][K]."""
    K = x.C
    x.consume()
    ldy = N if ldy is None else ldy
    y = out_buf if out_buf is not None else eng.empty(x.pyr.rows, ldy)
    bias = P.view(bname) if bname else None
    L.call("edet_conv1x1_fwd", eng.dt, x.lazy(), x.pyr.c, K, vp(P.wcv(wname)), N, vp(bias), vp(y), ldy, 0,
           _stats_out(eng, bns), stream())
    out = Act(y, x.pyr, N, bns, act, ld=ldy, training=eng.training, name=name)

    def bwd():
        rec = eng.tape.take(out)
        if rec is None:
            return
        d, ld = value_grad_to_raw(eng, out, rec)
        with eng.side(x.raw, x.gate, d):
            a = x.lazy()
            if N >= WGRAD_MATERIALIZE_N and x.has_transform:
                # the weight gradient re-applies A's lazy transform once per 64-column tile
                # (N/64 times); for wide outputs one materialize pass is cheaper (same bf16
                # operand the kernel would stage, so dW is unchanged)
                xa = eng.empty(x.pyr.rows, K)
                L.call("edet_lazy_materialize", eng.dt, a, x.pyr.c, K, vp(xa), stream())
                a = Act(xa, x.pyr, K).lazy()
            L.call("edet_conv1x1_wgrad", eng.dt, a, x.pyr.c, K, vp(d), ld, N, vp(P.grad(wname)),
                   vp(P.grad(bname) if bname else None), stream())
        s = stream()
        dx, acc = eng.tape.dst(x)
        src = x.se_source
        if (SESUM_DGRAD and src is not None and acc == 0 and x.uses == 1 and src.bns is not None
                and len(src.bns) == 1 and src.act == L.ACT_SWISH and src.C == K and K <= 2048
                and _sesum_epilogue_route(eng, x.pyr, N, K)):
            # x is the materialised SE-gated depthwise output: its backward sums (the gate
            # gradient and the BN terms, edet_gate_bn_reduce's) come from this dgrad's epilogue
            sums5 = eng.zeros64(5, x.pyr.batch, K)
            L.call("edet_conv1x1_dgrad_sesum", eng.dt, vp(d), ld, x.pyr.c, N, vp(P.wtv(wname)), K, vp(dx), K,
                   src.lazy(), vp(sums5), s)
            eng.tape.g[x].se_sums = sums5
            return
        fold = _fold_dst(eng, x, acc) if FOLD_GEMM_BN else None
        if fold is not None:
            L.call("edet_conv1x1_dgrad_fold", eng.dt, vp(d), ld, x.pyr.c, N, vp(P.wtv(wname)), K, vp(dx), K, x.lazy(),
                   fold, s)
        else:
            L.call("edet_conv1x1_dgrad", eng.dt, vp(d), ld, x.pyr.c, N, vp(P.wtv(wname)), K, vp(dx), K, acc, s)

    eng.record(bwd)
    return out


# --------------------------------------------------------------------------- depthwise
# stride-1 backward as one fused pass (edet_dwconv_bwd), with the BN-backward fold of the
# input's BatchNorm when this op is the input's only consumer
FUSED_DW_BWD = os.environ.get("EDET_FUSED_DW", "1") != "0"
FOLD_DW_BN = os.environ.get("EDET_FOLD_DW_BN", "1") != "0"
# the 1x1 dgrad can take the BN-backward sums of its output's value in its epilogue
# (edet_conv1x1_dgrad_fold) when it owns that value's whole gradient.  Off by default: the whole
# D0 step measured no gain (13.777 vs 13.758 ms, three alternating runs each, r04j) -- the reduce
# pass it saves runs at ~5.8 TB/s, and the GEMMs it extends are latency-bound
FOLD_GEMM_BN = os.environ.get("EDET_FOLD_GEMM_BN", "0") != "0"
# the stride-2 depthwise dgrad with the same fold (edet_dwconv_dgrad_fold)
FOLD_DWS2_BN = os.environ.get("EDET_FOLD_DWS2_BN", "1") != "0"
# the stride-1 SE-gated depthwise output's BN-backward apply inside the fused backward's dy
# staging (edet_dwconv_bwd_lazy) instead of its own pass.  Off by default: it removes the 12
# applies (-417 us of kernel time) but the tiled backward grows by as much (+427 us: the
# transform -- a sigmoid per halo element -- sits between its loads and its stencil), and the
# whole D0 step measured 13.30 (off) vs 13.33 ms (on), same-box A/B r05b
LAZY_DY_DW = os.environ.get("EDET_LAZY_DY", "0") != "0"
# the SE-gated depthwise output's backward sums in the project conv's dgrad epilogue
# (edet_conv1x1_dgrad_sesum) instead of edet_gate_bn_reduce's pass over (y, dv).  Off by
# default: the 13 K-loop dgrads grew by 361 us (per element a sigmoid and the x tile in LDS,
# 3 -> 2 waves per SIMD at 64 x 128) against the 300 us of reduce passes removed (r05b kbench),
# whole step even to +0.03 ms
SESUM_DGRAD = os.environ.get("EDET_SESUM_DGRAD", "0") != "0"
# every switch that takes a BN-backward pass into the kernel producing or consuming the gradient
# (the test of the folds flips them all: tests/test_model_gpu.py::test_bn_backward_folds_equal_unfused_path)
FOLD_SWITCHES = ("FUSED_DW_BWD", "FOLD_DW_BN", "FOLD_GEMM_BN", "FOLD_DWS2_BN", "LAZY_DY_DW", "SESUM_DGRAD")


def _sesum_epilogue_route(eng: Engine, pyr: Pyr, N: int, K: int) -> bool:
    """edet_conv1x1_dgrad_sesum takes the sums in its K-loop epilogue for these shapes (its
    route rule, include/edet.h); elsewhere it would run dgrad + edet_gate_bn_reduce itself, so
    the caller keeps the two passes as separate calls (one kernel per entry point: the bench
    attributes each call's time and bytes to the kernel it launched)."""
    narrow = eng.dt == L.BF16 and N <= 32 and K <= 160
    return pyr.nseg == 1 and not narrow and (pyr.H * pyr.W) % 64 == 0 and pyr.row_off[0] == 0


def _dgrad_fold_kernel_route(k: int, pin: Pyr) -> bool:
    """edet_dwconv_dgrad_fold runs its folded kernel for k3 over >= 2^20 input rows (its route,
    dwconv.hip); elsewhere it runs dgrad + the reduce itself, so the caller makes them separate
    calls (one kernel per entry point)."""
    return k == 3 and sum(pin.seg_rows(s) for s in range(pin.nseg)) >= (1 << 20)


def _fold_dst(eng: Engine, x: Act, acc: int):
    """BN-backward fold destination for x's gradient when the op writing it owns all of it (x has
    one consumer, nothing accumulated yet) and x's value is BN(+act) without an SE gate: zeroed
    fp64 [2][nseg][stat_len(C)] replicated sums recorded on x's gradient (value_grad_to_raw then skips its reduce pass)
    and their edet_bngrad64 descriptor; else None."""
    if not (acc == 0 and x.uses == 1 and x.bns is not None and x.gate is None and x.se is None):
        return None
    sums = eng.zeros64(2, len(x.bns), L.stat_len(x.C))  # replicated (include/edet.h)
    fold = L.BnGrad64()
    for i in range(len(x.bns)):
        fold.dgamma[i], fold.dbeta[i] = sums[0, i].data_ptr(), sums[1, i].data_ptr()
    eng.tape.g[x].bn_sums = sums
    return fold

def dwconv(eng: Engine, P: ParamStore, x: Act, wname: str, k: int, stride: int,
           bns: Optional[List[BNParam]] = None, act: int = L.ACT_NONE, name: str = "",
           squeeze: Optional[torch.Tensor] = None) -> Act:
    """Depthwise conv.  `squeeze` (inference only): a zeroed fp64 [B][C] that receives the SE
    squeeze mean_hw act(bn(y)) of the output from the same launch (edet_dwconv_fwd_squeeze)."""
    C = x.C
    x.consume()
    pout = x.pyr.strided(stride)
    y = eng.empty(pout.rows, C)
    out = Act(y, pout, C, bns, act, training=eng.training, name=name)
    if squeeze is not None:
        assert not eng.training, "the fused squeeze needs y's BN affine before the launch (moving statistics)"
        L.call("edet_dwconv_fwd_squeeze", eng.dt, x.lazy(), x.pyr.c, C, k, stride, vp(P.wcv(wname)), vp(y),
               pout.c, out.lazy(), vp(squeeze), stream())
    else:
        L.call("edet_dwconv_fwd", eng.dt, x.lazy(), x.pyr.c, C, k, stride, vp(P.wcv(wname)), vp(y), pout.c,
               _stats_out(eng, bns), stream())

    def bwd():
        rec = eng.tape.take(out)
        if rec is None:
            return
        if (stride == 1 and FUSED_DW_BWD and LAZY_DY_DW and not eng.overlap and out.se is not None
                and rec.scale is None and rec.ld == C and C % 16 == 0):
            # the SE-gated swish(BN) output: its d(raw) is built inside the fused backward while
            # the dy window loads (edet_dwconv_bwd_lazy) -- no apply pass, no d(raw) round trip
            dyl, keep = value_grad_lazy(eng, out, rec)
            dx, acc = eng.tape.dst(x)
            fold = _fold_dst(eng, x, acc) if FOLD_DW_BN else None
            L.call("edet_dwconv_bwd_lazy", eng.dt, x.lazy(), x.pyr.c, C, k, dyl, pout.c, vp(P.wcv(wname)),
                   vp(dx), acc, vp(P.grad(wname)), fold, stream())
            del keep
            return
        d, ld = value_grad_to_raw(eng, out, rec)
        assert ld == C
        if stride == 1 and FUSED_DW_BWD and not eng.overlap:
            # one pass over (d, x): dx, the filter gradient and, when this op owns x's whole
            # gradient, x's BN-backward sums (the reduce pass of value_grad_to_raw is skipped)
            dx, acc = eng.tape.dst(x)
            fold = _fold_dst(eng, x, acc) if FOLD_DW_BN else None
            L.call("edet_dwconv_bwd", eng.dt, x.lazy(), x.pyr.c, C, k, stride, vp(d), pout.c, vp(P.wcv(wname)),
                   vp(dx), acc, vp(P.grad(wname)), fold, stream())
            return
        with eng.side(x.raw, x.gate, d):
            L.call("edet_dwconv_wgrad", eng.dt, x.lazy(), x.pyr.c, C, k, stride, vp(d), pout.c, vp(P.grad(wname)),
                   stream())
        s = stream()
        dx, acc = eng.tape.dst(x)
        fold = _fold_dst(eng, x, acc) if FOLD_DWS2_BN and _dgrad_fold_kernel_route(k, x.pyr) else None
        if fold is not None:
            L.call("edet_dwconv_dgrad_fold", eng.dt, vp(d), pout.c, C, k, stride, vp(P.wcv(wname)), vp(dx), x.pyr.c,
                   x.lazy(), fold, s)
        else:
            L.call("edet_dwconv_dgrad", eng.dt, vp(d), pout.c, C, k, stride, vp(P.wcv(wname)), vp(dx), x.pyr.c, acc, s)

    eng.record(bwd)
    return out


# --------------------------------------------------------------------------- SE
def squeeze_excite(eng: Engine, P: ParamStore, x: Act, prefix: str, R: int,
                   svec: Optional[torch.Tensor] = None):
    """Attach the SE gate to x (the swish(BN(dw)) value) in place: v -> v * sigmoid(...).
    `svec`: the squeeze already taken by the producer (dwconv(..., squeeze=svec))."""
    assert x.pyr.nseg == 1 and x.gate is None
    B, C = x.pyr.batch, x.C
    HW = x.pyr.H * x.pyr.W
    s = stream()
    if svec is None:
        svec = eng.zeros64(B, C)  # fp64 squeeze (edet.h)
        L.call("edet_se_squeeze", eng.dt, x.lazy(), B, HW, C, vp(svec), s)
    z1 = torch.empty((B, R), dtype=torch.float32, device=eng.device)
    gate = torch.empty((B, C), dtype=torch.float32, device=eng.device)
    w1, b1 = P.view(prefix + "/conv2d/kernel"), P.view(prefix + "/conv2d/bias")
    w2, b2 = P.view(prefix + "/conv2d_1/kernel"), P.view(prefix + "/conv2d_1/bias")
    L.call("edet_se_fwd", B, C, R, vp(svec), vp(w1), vp(b1), vp(w2), vp(b2), vp(z1), vp(gate), s)
    rec = SERec(svec, z1, gate, w1, b1, w2, b2, P.grad(prefix + "/conv2d/kernel"), P.grad(prefix + "/conv2d/bias"),
                P.grad(prefix + "/conv2d_1/kernel"), P.grad(prefix + "/conv2d_1/bias"), R)
    x.set_gate(gate, rec)
    return x


def materialize(eng: Engine, x: Act, name: str = "") -> Act:
    """Write v(x) once as a plain tensor (same bf16 rounding the GEMM A-operand staging
    applies, so the consumer's inputs are unchanged).  Backward: the gradient of the plain copy
    IS the gradient of x's value, handed to x's own backward as is."""
    x.consume()
    y = eng.empty(x.pyr.rows, x.C)
    L.call("edet_lazy_materialize", eng.dt, x.lazy(), x.pyr.c, x.C, vp(y), stream())
    out = Act(y, x.pyr, x.C, training=eng.training, name=name)
    if x.se is not None:
        out.se_source = x

    def bwd():
        rec = eng.tape.take(out)
        if rec is None:
            return
        eng.tape.alias(x, rec.t, rec.ld, rec.scale, se_sums=rec.se_sums)

    eng.record(bwd)
    return out


# --------------------------------------------------------------------------- resampling
def maxpool(eng: Engine, x: Act, name: str = "") -> Act:
    assert x.pyr.nseg == 1
    x.consume()
    B, H, W, C = x.pyr.batch, x.pyr.H, x.pyr.W, x.C
    pout = x.pyr.strided(2)
    y = eng.empty(pout.rows, C)
    # training: the forward records its window taps, the backward routes dy by them
    taps = (torch.empty((pout.rows, C), dtype=torch.uint8, device=eng.device)
            if eng.training and L.has("edet_maxpool_fwd_taps") else None)
    if taps is not None:
        L.call("edet_maxpool_fwd_taps", eng.dt, x.lazy(), B, H, W, C, vp(y), vp(taps), stream())
    else:
        L.call("edet_maxpool_fwd", eng.dt, x.lazy(), B, H, W, C, vp(y), stream())
    out = Act(y, pout, C, training=eng.training, name=name)

    def bwd():
        rec = eng.tape.take(out)
        if rec is None:
            return
        assert rec.ld == C
        dx, acc = eng.tape.dst(x)
        if taps is not None:
            L.call("edet_maxpool_bwd_taps", eng.dt, B, H, W, C, vp(taps), vp(rec.t), vp(dx), acc, stream())
        else:
            L.call("edet_maxpool_bwd", eng.dt, x.lazy(), B, H, W, C, vp(rec.t), vp(dx), acc, stream())

    eng.record(bwd)
    return out


# EDET_FUSE_DV=0: the two-pass fusion backward (d(value) -> d(raw) apply, then
# edet_bifpn_fuse_bwd) for same-box A/B against the one-pass edet_bifpn_fuse_bwd_dv
FUSE_DV = os.environ.get("EDET_FUSE_DV", "1") != "0"


def _fuse_fold(items):
    """One launch adding every node's weight-gradient records into its gradient view."""
    arr = (L.FuseFold * len(items))()
    for k, (part, wvec, grad, nparts, n) in enumerate(items):
        arr[k].part, arr[k].w, arr[k].dw = part.data_ptr(), wvec.data_ptr(), grad.data_ptr()
        arr[k].nparts, arr[k].n_in = nparts, n
    L.call("edet_bifpn_fuse_fold", len(items), arr, stream())


def bifpn_fuse(eng: Engine, P: ParamStore, inputs: Sequence[Tuple[Act, int]], wnames: Sequence[str],
               H: int, W: int, name: str = "") -> Act:
    """sum_i R_i(v_i) * w_i / (sum w + 1e-4); returned lazily as swish(sum) (OpAfterCombine)."""
    n = len(inputs)
    C = inputs[0][0].C
    B = inputs[0][0].pyr.batch
    wvec = P.view(wnames[0])  # the node's WSM_0..WSM_{n-1} scalars as one [n] parameter
    assert wvec.numel() == n
    fi = (L.FuseInput * n)()
    # max-pooled inputs: the forward records each output's window tap (1 byte per element)
    # so the backward neither re-evaluates the 3x3 windows nor re-applies their lazy BN/swish
    taps = [eng.empty(B * H * W, C, dtype=torch.uint8) if (mode == L.MODE_MAXPOOL and eng.training) else None
            for (_, mode) in inputs]
    for i, (a, mode) in enumerate(inputs):
        assert a.pyr.nseg == 1 and a.C == C
        a.consume()
        fi[i].v = a.lazy()
        fi[i].H, fi[i].W, fi[i].mode = a.pyr.H, a.pyr.W, mode
        fi[i].pool_arg = taps[i].data_ptr() if taps[i] is not None else None
    pyr = Pyr(B, [(H, W)])
    y = eng.empty(pyr.rows, C)
    L.call("edet_bifpn_fuse_fwd", eng.dt, n, fi, vp(wvec), B, H, W, C, vp(y), stream())
    out = Act(y, pyr, C, None, L.ACT_SWISH, training=eng.training, name=name)

    def bwd():
        rec = eng.tape.take(out)
        if rec is None:
            return
        fb = (L.FuseInput * n)()
        for i, (a, mode) in enumerate(inputs):
            fb[i].v = a.lazy()
            fb[i].H, fb[i].W, fb[i].mode = a.pyr.H, a.pyr.W, mode
            fb[i].pool_arg = taps[i].data_ptr() if taps[i] is not None else None
        # one pass from d(value) (ABI 10) where the library covers the node: d(raw) formed in
        # registers, the weight gradient as per-block records folded once after the backward
        nparts = ctypes.c_int(0)
        if (FUSE_DV and rec.scale is None and rec.ld == C and out.bns is None and out.gate is None
                and L.has("edet_bifpn_fuse_bwd_dv")):
            L.call("edet_bifpn_fuse_bwd_dv_parts", eng.dt, n, fb, B, H, W, C, ctypes.byref(nparts))
        dF = None
        if nparts.value == 0:
            dF, _ = value_grad_to_raw(eng, out, rec)
        for i, (a, _) in enumerate(inputs):
            dx, acc = eng.tape.dst(a)
            fb[i].dx = dx.data_ptr()
            fb[i].accumulate = acc
        if dF is not None:
            L.call("edet_bifpn_fuse_bwd", eng.dt, n, fb, vp(wvec), B, H, W, C, vp(y), vp(dF),
                   vp(P.grad(wnames[0])), stream())
            return
        part = torch.empty(nparts.value * 4, dtype=torch.float32, device=eng.device)
        L.call("edet_bifpn_fuse_bwd_dv", eng.dt, n, fb, vp(wvec), B, H, W, C, vp(y), vp(rec.t),
               1 if out.act == L.ACT_SWISH else 0, vp(part), nparts.value, stream())
        eng.tape.collect("bifpn_fuse_fold", _fuse_fold, (part, wvec, P.grad(wnames[0]), nparts.value, n))

    eng.record(bwd)
    return out


# --------------------------------------------------------------------------- heads
def residual(eng: Engine, x: Act, res: Act, scale: Optional[torch.Tensor], name: str = "") -> Act:
    """out = v(x) * scale[level][image] + v(res)  (drop-connect survival scale, 1 at inference)."""
    C = x.C
    x.consume()
    res.consume()
    y = eng.empty(x.pyr.rows, C)
    L.call("edet_residual_fwd", eng.dt, x.lazy(), res.lazy(), x.pyr.c, C, vp(scale), vp(y), stream())
    out = Act(y, x.pyr, C, training=eng.training, name=name)

    def bwd():
        rec = eng.tape.take(out)
        if rec is None:
            return
        # d v(x) = dout * scale ; d v(res) = dout (aliased: x's backward reads it before res's
        # remaining consumer accumulates into it — x is produced from res)
        eng.tape.alias(x, rec.t, rec.ld, scale)
        eng.tape.alias(res, rec.t, rec.ld)

    eng.record(bwd)
    return out


def assemble_pyramid(eng: Engine, buf: torch.Tensor, pyr: Pyr, parts: Sequence[Act], bns: List[BNParam],
                     name: str = "") -> Act:
    """The last BiFPN cell writes its five node outputs into one pyramid buffer; this op is
    the (copy-free) join and, backwards, the split of the pyramid gradient into views."""
    C = parts[0].C
    for a in parts:
        a.consume()
    out = Act(buf, pyr, C, bns, L.ACT_NONE, training=eng.training, name=name)

    def bwd():
        rec = eng.tape.take(out)
        if rec is None:
            return
        assert rec.ld == C and rec.scale is None
        for s, a in enumerate(parts):
            eng.tape.alias(a, rec.t[pyr.seg_slice(s)], C)

    eng.record(bwd)
    return out
