"""Kernel parity at the model's own sizes (M up to 2^17 rows, pyramids of 5 segments).

The small-shape tests in test_kernels_gpu.py keep every workgroup on one tile.  These shapes
make the persistent kernels (GEMM row-tile loop, depthwise tile loop, BN-backward chunk loop)
walk many tiles and cross segment boundaries.  Each kernel runs twice: outputs written
without atomics must be bit-identical between runs (a race shows up here first), and both
runs are checked against the fp64 CPU reference.
"""
import math

import numpy as np
import pytest
import torch

from tf2mv_amd import _lib as L
from tf2mv_amd.runtime import Pyr, stream, vp
from gpu_util import DEV, DT, TDT, LazyDesc, bngrad64, close, fv, g, make_bn, rep64, seg_out, stat_out, stats_out, zeros, zeros64

pytestmark = pytest.mark.gpu
DTS = ["f32", "bf16"]
PYR5 = [(64, 64), (32, 32), (16, 16), (8, 8), (4, 4)]


def rnd(rng, *shape, scale=1.0):
    return torch.tensor(rng.standard_normal(shape) * scale, dtype=torch.float32)


def make_pyr(kind):
    if kind == "p5":
        return Pyr(2, PYR5)
    return Pyr(kind[0], [kind[1]])


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("kind,K,N,lazy", [((2, (64, 64)), 32, 16, 1), ((2, (64, 64)), 16, 96, 2),
                                           ((8, (128, 128)), 16, 96, 2), ((8, (128, 128)), 32, 16, 1),
                                           ((8, (64, 64)), 40, 240, 1), ((4, (16, 16)), 192, 1152, 1),
                                           ("p5", 64, 64, 3), ("p5", 64, 810, 3)])
def test_conv1x1_fwd_large(dt, kind, K, N, lazy):
    rng = np.random.default_rng(K * 31 + N)
    pyr = make_pyr(kind)
    x = g(rnd(rng, pyr.rows, K), dt)
    bn = make_bn(x, pyr, K, rng) if lazy else None
    gate = g(torch.rand(pyr.batch, K), "f32") if lazy == 1 else None
    lz = LazyDesc(x, pyr, K, bn=bn, act=1 if lazy in (1, 3) else 0, gate=gate)
    w = g(rnd(rng, N, K, scale=1 / math.sqrt(K)), dt)
    b = g(rnd(rng, N), "f32")
    ys, sts = [], []
    for _ in range(2):
        y = torch.full((pyr.rows, N), float("nan"), dtype=TDT[dt], device=DEV)
        st = stats_out(pyr.nseg, N)
        L.call("edet_conv1x1_fwd", DT[dt], lz.c, pyr.c, K, vp(w), N, vp(b), vp(y), N, 0, stat_out(st), stream())
        ys.append(y)
        sts.append(st)
    torch.cuda.synchronize()
    ref = lz.cpu_value() @ w.double().cpu().t() + b.double().cpu()
    for s in range(pyr.nseg):
        sl = pyr.seg_slice(s)
        assert torch.equal(ys[0][sl], ys[1][sl]), f"segment {s}: output differs between runs"
        close(ys[0][sl], ref[sl], dt)
        n = pyr.seg_rows(s)
        close(sts[0][s][0], ref[sl].sum(0), dt, scale=n ** 0.5 * 4)
        close(sts[0][s][1], (ref[sl] ** 2).sum(0), dt, scale=n ** 0.5 * 8, rtol=5e-2 if dt == "bf16" else 1e-4)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("kind,K,N,lazy", [((8, (128, 128)), 16, 96, 2), ((8, (64, 64)), 144, 24, 1),
                                           ("p5", 64, 64, 3), ("p5", 64, 36, 0), ((4, (64, 64)), 672, 112, 1)])
def test_conv1x1_wgrad_large(dt, kind, K, N, lazy, workspace_mode):
    rng = np.random.default_rng(K * 7 + N)
    pyr = make_pyr(kind)
    x = g(rnd(rng, pyr.rows, K), dt)
    bn = make_bn(x, pyr, K, rng) if lazy else None
    gate = g(torch.rand(pyr.batch, K), "f32") if lazy == 1 else None
    lz = LazyDesc(x, pyr, K, bn=bn, act=1 if lazy in (1, 3) else 0, gate=gate)
    ld = (N + 7) // 8 * 8
    dy = torch.zeros(pyr.rows, ld)
    dy[:, :N] = rnd(rng, pyr.rows, N)
    dy = g(dy, dt)
    dw, db = zeros(N, K), zeros(N)
    L.call("edet_conv1x1_wgrad", DT[dt], lz.c, pyr.c, K, vp(dy), ld, N, vp(dw), vp(db), stream())
    v = lz.cpu_value()
    d = dy[:, :N].double().cpu()
    refw = torch.zeros(N, K, dtype=torch.float64)
    refb = torch.zeros(N, dtype=torch.float64)
    for s in range(pyr.nseg):
        sl = pyr.seg_slice(s)
        refw += d[sl].t() @ v[sl]
        refb += d[sl].sum(0)
    close(dw, refw, dt, scale=pyr.rows ** 0.5 * 2)
    close(db, refb, dt, scale=pyr.rows ** 0.5 * 2)


def _dw_ref(v, pin, k, s, w):
    import torch.nn.functional as Fn
    outs = []
    C = v.shape[1]
    for sg in range(pin.nseg):
        H, W = pin.sizes[sg]
        xs = v[pin.seg_slice(sg)].reshape(pin.batch, H, W, C).permute(0, 3, 1, 2)
        OH, OW = -(-H // s), -(-W // s)
        ph = max((OH - 1) * s + k - H, 0)
        pw = max((OW - 1) * s + k - W, 0)
        xs = Fn.pad(xs, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
        wk = w.reshape(k, k, C).permute(2, 0, 1).unsqueeze(1)
        outs.append(Fn.conv2d(xs, wk, stride=s, groups=C).permute(0, 2, 3, 1).reshape(-1, C))
    return outs


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("k,s,kind,C,lazy", [(3, 1, (2, (64, 64)), 32, 1), (3, 2, (4, (64, 64)), 96, 1),
                                             (5, 2, (2, (32, 32)), 144, 1), (3, 1, "p5", 64, 3)])
def test_dwconv_fwd_large(dt, k, s, kind, C, lazy):
    rng = np.random.default_rng(k * 10 + C)
    pin = make_pyr(kind)
    pout = pin.strided(s)
    x = g(rnd(rng, pin.rows, C), dt)
    bn = make_bn(x, pin, C, rng) if lazy else None
    gate = g(torch.rand(pin.batch, C), "f32") if lazy == 1 else None
    lz = LazyDesc(x, pin, C, bn=bn, act=1, gate=gate)
    w = g(rnd(rng, k * k, C, scale=0.3), dt)
    ys, sts = [], []
    for _ in range(2):
        y = torch.full((pout.rows, C), float("nan"), dtype=TDT[dt], device=DEV)
        st = stats_out(pin.nseg, C)
        L.call("edet_dwconv_fwd", DT[dt], lz.c, pin.c, C, k, s, vp(w), vp(y), pout.c, stat_out(st), stream())
        ys.append(y)
        sts.append(st)
    torch.cuda.synchronize()
    refs = _dw_ref(lz.cpu_value(), pin, k, s, w.double().cpu())
    for sg in range(pin.nseg):
        sl = pout.seg_slice(sg)
        assert torch.equal(ys[0][sl], ys[1][sl]), f"segment {sg}: output differs between runs"
        close(ys[0][sl], refs[sg], dt)
        close(sts[0][sg][0], refs[sg].sum(0), dt, scale=pout.seg_rows(sg) ** 0.5 * 4)
        close(sts[0][sg][1], (refs[sg] ** 2).sum(0), dt, scale=pout.seg_rows(sg) ** 0.5 * 8,
              rtol=5e-2 if dt == "bf16" else 1e-4)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("kind,C,act", [((8, (128, 128)), 16, 0), ((8, (64, 64)), 96, 1), ("p5", 64, 1)])
def test_lazy_bwd_large(dt, kind, C, act):
    rng = np.random.default_rng(C + 5)
    pyr = make_pyr(kind)
    x = g(rnd(rng, pyr.rows, C), dt)
    bn = make_bn(x, pyr, C, rng)
    lz = LazyDesc(x, pyr, C, bn=bn, act=act)
    dv = g(rnd(rng, pyr.rows, C), dt)
    grads = [(zeros(C), zeros(C)) for _ in range(pyr.nseg)]  # (dgamma, dbeta)
    acc_t, acc = bngrad64(pyr.nseg, C)
    L.call("edet_lazy_bwd_reduce", DT[dt], lz.c, pyr.c, C, vp(dv), None, None, acc, stream())
    dx = torch.full((pyr.rows, C), float("nan"), dtype=TDT[dt], device=DEV)
    L.call("edet_lazy_bwd_apply", DT[dt], lz.c, pyr.c, C, vp(dv), None, None, acc, seg_out(grads), vp(dx), 0, stream())
    torch.cuda.synchronize()
    xc = x.double().cpu().requires_grad_(True)
    dvc = dv.double().cpu()
    for s in range(pyr.nseg):
        sl = pyr.seg_slice(s)
        su, sq, ga, be = (t.double().cpu() for t in bn[s])
        ga = ga.clone().requires_grad_(True)
        be = be.clone().requires_grad_(True)
        xs = xc[sl]
        mean = xs.mean(0)
        var = ((xs - mean) ** 2).mean(0)
        u = (xs - mean) / torch.sqrt(var + 1e-3) * ga + be
        v = u * torch.sigmoid(u) if act else u
        (v * dvc[sl]).sum().backward()
        n = pyr.seg_rows(s)
        close(grads[s][1], be.grad, dt, scale=n ** 0.5 * 2)
        close(grads[s][0], ga.grad, dt, scale=n ** 0.5 * 2)
    for s in range(pyr.nseg):
        sl = pyr.seg_slice(s)
        close(dx[sl], xc.grad[sl], dt)
