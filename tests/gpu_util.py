"""Helpers for the GPU parity tests: descriptors for raw tensors and CPU fp64 references."""
import ctypes

import numpy as np
import torch

from tf2mv_amd import _lib as L
from tf2mv_amd.runtime import Pyr, stream, vp

DEV = "cuda"
TDT = {"f32": torch.float32, "bf16": torch.bfloat16}
DT = {"f32": L.F32, "bf16": L.BF16}
TOL = {"f32": dict(rtol=2e-5, atol=2e-5), "bf16": dict(rtol=3e-2, atol=3e-2)}


def g(t, dt="f32"):
    return t.to(DEV, TDT[dt]).contiguous()


class LazyDesc:
    """Lazy value spec + its CPU fp64 evaluation."""

    def __init__(self, x, pyr: Pyr, C, bn=None, act=0, gate=None, eps=1e-3, ld=None):
        # x: device tensor [rows, ld];  bn: list per seg of (sum, sq, gamma, beta) device fp32
        self.x, self.pyr, self.C, self.bn, self.act, self.gate, self.eps = x, pyr, C, bn, act, gate, eps
        self.ld = ld or C
        lz = L.Lazy()
        lz.x = x.data_ptr()
        lz.gate = gate.data_ptr() if gate is not None else None
        lz.ld, lz.act = self.ld, act
        self._rep = []  # the replicated statistics vectors the descriptor points at (ABI 9)
        if bn:
            lz.bn.enabled = 1
            lz.bn.eps = eps
            for s, (a, b, c, d) in enumerate(bn):
                ra, rb = rep64(a), rep64(b)
                self._rep += [ra, rb]
                lz.bn.sum[s], lz.bn.sq[s], lz.bn.gamma[s], lz.bn.beta[s] = ra.data_ptr(), rb.data_ptr(), c.data_ptr(), d.data_ptr()
        self.c = lz

    def cpu_value(self):
        x = self.x[:, : self.C].double().cpu()
        out = x.clone()
        for s in range(self.pyr.nseg):
            sl = self.pyr.seg_slice(s)
            v = x[sl]
            if self.bn:
                su, sq, ga, be = (t.double().cpu() for t in self.bn[s])
                n = self.pyr.seg_rows(s)
                mean = su / n
                var = torch.clamp(sq / n - mean * mean, min=0)
                v = (v - mean) / torch.sqrt(var + self.eps) * ga + be
            if self.act:
                v = v * torch.sigmoid(v)
            if self.gate is not None:
                hw = self.pyr.sizes[s][0] * self.pyr.sizes[s][1]
                gt = self.gate.double().cpu()
                v = v * gt.repeat_interleave(hw, 0)
            out[sl] = v
        return out


def make_bn(x, pyr: Pyr, C, rng, shift=0.0):
    """Random BN params and *exact* batch stats of x per segment (fp32 device)."""
    segs = []
    xc = x[:, :C].double().cpu()
    for s in range(pyr.nseg):
        v = xc[pyr.seg_slice(s)]
        su = v.sum(0).to(DEV)  # fp64 statistics arena (edet_bn.sum / sq)
        sq = (v * v).sum(0).to(DEV)
        ga = torch.tensor(rng.uniform(0.5, 1.5, C), dtype=torch.float32, device=DEV)
        be = torch.tensor(rng.uniform(-0.5, 0.5, C) + shift, dtype=torch.float32, device=DEV)
        segs.append((su, sq, ga, be))
    return segs


def zeros64(*shape):
    return torch.zeros(shape, dtype=torch.float64, device=DEV)


def rep64(v):
    """A plain fp64 statistics vector (last dim C) in the library's replicated layout (replica 0)."""
    v = v if isinstance(v, Folded) else torch.as_tensor(v, dtype=torch.float64, device=DEV)
    return v.raw if isinstance(v, Folded) else L.stat_unfold(v.to(DEV, torch.float64))


class Folded:
    """A replicated fp64 statistics buffer (include/edet.h "Statistics vectors", ABI 9) that the
    kernels write; indexing / .v read its values (replicas summed in the library's order)."""

    def __init__(self, lead, C):
        self.C = C
        self.raw = torch.zeros(*lead, L.stat_len(C), dtype=torch.float64, device=DEV)
        self.dtype = self.raw.dtype

    def data_ptr(self):
        return self.raw.data_ptr()

    @property
    def v(self):
        return L.stat_fold(self.raw, self.C)

    def __getitem__(self, idx):
        return self.v[idx]

    def abs(self):
        return self.v.abs()

    def __len__(self):
        return self.raw.shape[0]


class _Slice:
    """Folded[i] as a statistics destination (pointer into the raw buffer) and value."""

    def __init__(self, parent, idx):
        self.parent, self.idx, self.dtype = parent, idx, torch.float64

    def data_ptr(self):
        return self.parent.raw[self.idx].data_ptr()

    @property
    def v(self):
        return self.parent.v[self.idx]


def stats_out(nseg, C):
    """[(sum, sq)] per segment: replicated destinations for a producer's BN statistics."""
    return [(Folded((), C), Folded((), C)) for _ in range(nseg)]


def fv(t):
    """The values of a Folded (or a plain tensor as is)."""
    return t.v if isinstance(t, (Folded, _Slice)) else t


def stat_out(pairs):
    so = L.StatOut()
    for i, (a, b) in enumerate(pairs):
        assert a.dtype == torch.float64 and b.dtype == torch.float64
        so.sum[i], so.sq[i] = a.data_ptr(), b.data_ptr()
    return so


def bngrad64(nseg, C):
    """fp64 dgamma / dbeta accumulators [2][nseg][C] (replicated, a Folded: index it for values)
    and their edet_bngrad64 descriptor."""
    t = Folded((2, nseg), C)
    d = L.BnGrad64()
    for i in range(nseg):
        d.dgamma[i], d.dbeta[i] = t.raw[0, i].data_ptr(), t.raw[1, i].data_ptr()
    return t, d


def seg_out(pairs):
    so = L.SegOut()
    for i, (a, b) in enumerate(pairs):
        so.a[i], so.b[i] = a.data_ptr(), b.data_ptr()
    return so


def zeros(*shape):
    return torch.zeros(shape, dtype=torch.float32, device=DEV)


def close(a, b, dt, scale=None, **kw):
    a, b = fv(a), fv(b)
    a = a.double().cpu() if isinstance(a, torch.Tensor) else torch.as_tensor(a, dtype=torch.float64)
    b = b.double().cpu() if isinstance(b, torch.Tensor) else torch.as_tensor(b, dtype=torch.float64)
    tol = dict(TOL[dt])
    tol.update(kw)
    if scale is not None:
        tol["atol"] = tol["atol"] * scale
    torch.testing.assert_close(a, b, **tol)
