"""Per-kernel parity: libedet (HIP, through the C-ABI) vs fp64 torch-CPU references.

fp32 storage must match to ~1e-5; bf16 storage to bf16 rounding (3e-2 relative on O(1)
values).  Shapes include ragged sizes, odd spatial extents (TF SAME asymmetric padding),
channel counts that are not tile multiples and 2-segment pyramids with padding rows.
"""
import ctypes
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from tf2mv_amd import _lib as L
from tf2mv_amd.runtime import Pyr, stream, vp
from gpu_util import DEV, DT, TDT, LazyDesc, bngrad64, close, fv, g, make_bn, rep64, seg_out, stat_out, stats_out, zeros, zeros64

pytestmark = pytest.mark.gpu
DTS = ["f32", "bf16"]


def rnd(rng, *shape, scale=1.0):
    return torch.tensor(rng.standard_normal(shape) * scale, dtype=torch.float32)


def pyr_data(rng, pyr, C, dt, scale=1.0):
    x = rnd(rng, pyr.rows, C, scale=scale)
    return g(x, dt)


# ----------------------------------------------------------------- conv1x1
@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("M,K,N,lazy,nseg", [(300, 24, 40, 0, 1), (1000, 96, 144, 1, 1), (777, 64, 729, 2, 1),
                                            (513, 40, 64, 3, 2), (4096, 192, 1152, 1, 1), (700, 480, 80, 1, 1),
                                            (600, 16, 96, 1, 1), (300, 1152, 320, 1, 1), (260, 320, 1152, 0, 1),
                                            (640, 672, 112, 0, 1),
                                            # D4's 224-channel BiFPN / head convs (B-resident form)
                                            (900, 224, 224, 3, 2), (1100, 224, 224, 0, 1), (500, 224, 729, 3, 1),
                                            # narrow outputs over a deeper plain A (wave-streaming form)
                                            (2000, 96, 16, 0, 1), (1500, 144, 24, 0, 1), (900, 160, 32, 0, 2),
                                            (700, 240, 40, 0, 1),
                                            # route rules of round 3: lazy K <= 64 into N <= 64 (wave
                                            # streaming), lazy K > 64 into N > 320 (K loop), plain without
                                            # statistics (K loop; the stats-free call is below)
                                            (1000, 40, 64, 1, 1), (700, 80, 480, 3, 1),
                                            # route rules of round 4: lazy K > 64 into 192 < N <= 320
                                            # (K loop), plain K = 224 into N >= 192 with statistics at
                                            # M <= 8192 (A-resident; without them the K loop), the
                                            # class predict's K = 64 into N = 729 over M >= 131072
                                            # without statistics (B-resident)
                                            (800, 160, 224, 3, 1), (800, 160, 224, 1, 1), (131072, 64, 729, 0, 1),
                                            # round-5 K-loop tiles at 8192 / 32768 rows: plain with
                                            # statistics 64 x 64 / 128 x 64 (and stats-free 8192
                                            # rows), lazy into N > 320 64 x 128, lazy with
                                            # statistics into 64 columns 64 x 64 / 128 x 64
                                            (8192, 1152, 192, 0, 1), (32768, 480, 112, 0, 1),
                                            (8192, 192, 1152, 1, 1), (8192, 320, 64, 3, 1), (32768, 112, 64, 2, 1),
                                            # round 6: the column-sliced wave-streaming form (lazy A,
                                            # K <= 128 into N > 160 over >= 32768 rows; a gated
                                            # K > 64 stays on the K loop)
                                            (32768, 112, 672, 3, 1), (32768, 40, 240, 2, 1), (32768, 80, 480, 1, 1),
                                            (32768, 24, 168, 1, 1)])
def test_conv1x1_fwd(dt, M, K, N, lazy, nseg):
    """conv1x1 forward with BN statistics (and without them for plain inputs: the stats-free
    route) against fp64."""
    rng = np.random.default_rng(M + K + N)
    pyr = Pyr(2, [(13, 11), (7, 5)]) if nseg == 2 else Pyr(1, [(M, 1)])
    x = pyr_data(rng, pyr, K, dt)
    bn = make_bn(x, pyr, K, rng) if lazy else None
    gate = g(torch.rand(pyr.batch, K), "f32") if lazy == 1 else None
    lz = LazyDesc(x, pyr, K, bn=bn, act=1 if lazy in (1, 3) else 0, gate=gate)
    w = g(rnd(rng, N, K, scale=1 / math.sqrt(K)), dt)
    b = g(rnd(rng, N), "f32")
    y = torch.empty(pyr.rows, N, dtype=TDT[dt], device=DEV)
    st = stats_out(nseg, N)
    L.call("edet_conv1x1_fwd", DT[dt], lz.c, pyr.c, K, vp(w), N, vp(b), vp(y), N, 0, stat_out(st), stream())
    ref = lz.cpu_value() @ w.double().cpu().t() + b.double().cpu()
    for s in range(nseg):
        sl = pyr.seg_slice(s)
        close(y[sl], ref[sl], dt)
        close(st[s][0], ref[sl].sum(0), dt, scale=pyr.seg_rows(s) ** 0.5 * 4)
        close(st[s][1], (ref[sl] ** 2).sum(0), dt, scale=pyr.seg_rows(s) ** 0.5 * 8, rtol=5e-2 if dt == "bf16" else 1e-4)
    if not lazy:  # the same product without statistics (box / class predict convs) takes another route
        y2 = torch.empty_like(y)
        L.call("edet_conv1x1_fwd", DT[dt], lz.c, pyr.c, K, vp(w), N, vp(b), vp(y2), N, 0, None, stream())
        close(y2, ref, dt)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("M,N,K,ldy", [(300, 40, 24, 40), (777, 729, 64, 736), (2048, 1152, 192, 1152),
                                       (500, 320, 1152, 320), (300, 36, 64, 40), (1000, 224, 224, 224),
                                       (600, 729, 224, 736), (2000, 96, 16, 96), (1500, 144, 24, 144),
                                       # round-5 K-loop tiles at 8192 rows: 128 x 64 / 64 x 64
                                       (8192, 320, 1152, 320), (8192, 1152, 192, 1152),
                                       # round-6 tiles: short K into wide dx (64 x 64 / 64 x 128),
                                       # the class head's deep dgrad (128 x 64)
                                       (131072, 40, 240, 40), (32768, 80, 240, 80),
                                       (131200, 729, 64, 736)])
def test_conv1x1_dgrad(dt, M, N, K, ldy):
    rng = np.random.default_rng(M * 7 + N)
    pyr = Pyr(1, [(M, 1)])
    dy = torch.zeros(M, ldy)
    dy[:, :N] = rnd(rng, M, N)
    dy = g(dy, dt)
    w = g(rnd(rng, N, K, scale=1 / math.sqrt(N)), dt)
    ldn = (N + 7) // 8 * 8
    wkn = torch.zeros(K, ldn)
    wkn[:, :N] = w.float().cpu().t()
    wkn = g(wkn, dt)  # the transposed compute copy the dgrad GEMM consumes
    dx = g(torch.full((M, K), 0.5), dt)
    L.call("edet_conv1x1_dgrad", DT[dt], vp(dy), ldy, pyr.c, N, vp(wkn), K, vp(dx), K, 1, stream())
    ref = dy[:, :N].double().cpu() @ w.double().cpu() + 0.5
    # accumulate rounds (old + dy W) once to the storage type (the bf16 bar
    # is one bf16 rounding, 2^-9 relative, with room for the fp32 accumulation order)
    close(dx, ref, dt, **({} if dt == "f32" else dict(rtol=5e-3, atol=5e-3)))


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("M,N,K,act,nseg", [
    # wave-streaming routes: N <= 96 / K <= 64, N <= 48 / K <= 256 (the D0 expand dgrads: 96 -> 16,
    # 144 -> 24, 240 -> 40), then the K loop (480 -> 80 with 64-row tiles over M >= 32768,
    # 1152 -> 192, a 5-level pyramid, an act-free and a swish value)
    (2000, 96, 16, 0, 1), (1500, 144, 24, 0, 1), (1100, 240, 40, 1, 1), (900, 64, 64, 1, 1),
    (32768, 480, 80, 0, 1), (1000, 1152, 192, 0, 1), (700, 672, 112, 1, 1), (0, 64, 64, 1, 5),
    (0, 160, 96, 0, 2)])
def test_conv1x1_dgrad_fold(dt, M, N, K, act, nseg):
    """edet_conv1x1_dgrad_fold: dx as edet_conv1x1_dgrad, and the BN-backward sums of the value
    dx is the gradient of equal to edet_lazy_bwd_reduce over (x, dx) -- the pass the fold
    replaces (same fp64 destinations; the fold sums the stored dx, so only the order of the
    fp32 partial sums differs) and to fp64."""
    rng = np.random.default_rng(M + 3 * N + K + act)
    if nseg == 5:
        pyr = Pyr(2, [(16, 16), (8, 8), (4, 4), (2, 2), (1, 1)])
    elif nseg == 2:
        pyr = Pyr(3, [(13, 11), (7, 5)])
    else:
        pyr = Pyr(1, [(M, 1)])
    dy = g(rnd(rng, pyr.rows, N), dt)
    w = g(rnd(rng, N, K, scale=1 / math.sqrt(N)), dt)
    ldn = (N + 7) // 8 * 8
    wkn = torch.zeros(K, ldn)
    wkn[:, :N] = w.float().cpu().t()
    wkn = g(wkn, dt)
    x = pyr_data(rng, pyr, K, dt, scale=2.0)
    for sg in range(nseg - 1):  # padding rows between levels are never read
        x[pyr.row_off[sg] + pyr.seg_rows(sg):pyr.row_off[sg + 1]] = float("nan")
    bn = make_bn(x.nan_to_num(0.0), pyr, K, rng)
    lz = LazyDesc(x, pyr, K, bn=bn, act=act)
    dx = torch.empty(pyr.rows, K, dtype=TDT[dt], device=DEV)
    acc_t, acc = bngrad64(nseg, K)
    L.call("edet_conv1x1_dgrad_fold", DT[dt], vp(dy), N, pyr.c, N, vp(wkn), K, vp(dx), K, lz.c, acc, stream())
    dx2 = torch.empty_like(dx)
    L.call("edet_conv1x1_dgrad", DT[dt], vp(dy), N, pyr.c, N, vp(wkn), K, vp(dx2), K, 0, stream())
    ref_t, ref = bngrad64(nseg, K)
    L.call("edet_lazy_bwd_reduce", DT[dt], lz.c, pyr.c, K, vp(dx2), None, None, ref, stream())
    for sg in range(nseg):
        sl = pyr.seg_slice(sg)
        assert torch.equal(dx[sl], dx2[sl])
        n = pyr.seg_rows(sg)
        close(acc_t[:, sg], ref_t[:, sg], "f32", scale=n ** 0.5, rtol=1e-4)
        # fp64 from the stored dx
        xs = x[sl].double().cpu()
        su, sq, ga, be = (t.double().cpu() for t in bn[sg])
        mean = su / n
        rstd = 1 / torch.sqrt(torch.clamp(sq / n - mean * mean, min=0) + 1e-3)
        u = (xs - mean) * rstd * ga + be
        du = dx2[sl].double().cpu()
        if act:
            sg_ = torch.sigmoid(u)
            du = du * sg_ * (1 + u * (1 - sg_))
        close(acc_t[1, sg], du.sum(0), dt, scale=n ** 0.5)
        close(acc_t[0, sg], (du * (xs - mean) * rstd).sum(0), dt, scale=n ** 0.5)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("K,N,lazy,nseg", [(24, 40, 0, 1), (96, 144, 1, 1), (64, 729, 0, 2), (40, 64, 2, 2),
                                           (16, 96, 0, 1), (32, 16, 0, 1), (144, 24, 0, 1), (1152, 320, 0, 1),
                                           (112, 672, 0, 1), (64, 36, 0, 2), (240, 40, 0, 1), (40, 240, 0, 2),
                                           (64, 64, 1, 1), (64, 64, 2, 2), (320, 64, 0, 1)])
def test_conv1x1_wgrad(dt, K, N, lazy, nseg):
    rng = np.random.default_rng(K * 13 + N)
    pyr = Pyr(3, [(17, 9), (5, 3)]) if nseg == 2 else Pyr(2, [(37, 29)])
    x = pyr_data(rng, pyr, K, dt)
    # poison padding rows: they must be ignored
    x[pyr.seg_rows(0):pyr.row_off[-1]] = float("nan")
    bn = make_bn(x.nan_to_num(0.0), pyr, K, rng) if lazy else None
    gate = g(torch.rand(pyr.batch, K), "f32") if (lazy == 1 and nseg == 1) else None
    lz = LazyDesc(x, pyr, K, bn=bn, act=1 if lazy else 0, gate=gate)
    ld = N if N % 8 == 0 else N + (8 - N % 8)
    dy = torch.zeros(pyr.rows, ld)
    dy[:, :N] = rnd(rng, pyr.rows, N)
    dy = g(dy, dt)
    dy[pyr.seg_rows(0):pyr.row_off[-1]] = float("nan")
    dw = zeros(N, K)
    db = zeros(N)
    L.call("edet_conv1x1_wgrad", DT[dt], lz.c, pyr.c, K, vp(dy), ld, N, vp(dw), vp(db), stream())
    v = lz.cpu_value()
    d = dy[:, :N].double().cpu()
    refw = torch.zeros(N, K, dtype=torch.float64)
    refb = torch.zeros(N, dtype=torch.float64)
    for s in range(nseg):
        sl = pyr.seg_slice(s)
        refw += d[sl].t() @ v[sl]
        refb += d[sl].sum(0)
    close(dw, refw, dt, scale=pyr.rows ** 0.5 * 2)
    close(db, refb, dt, scale=pyr.rows ** 0.5 * 2)


@pytest.mark.parametrize("arena_mb", [256, 1])
def test_partials_deferred_flush(arena_mb):
    """edet_partials_defer / edet_partials_flush (ABI 10): the weight-gradient split sums of a
    backward recorded and launched once give the immediate sums (to the order of the fp32
    atomics that add chunk sums, and of two jobs adding into the same dW: a weight used twice)
    for the 1x1 split partials (one 64 x 64 tile over a long M),
    the wave-streaming form (2M x 16 -> 96) and the stem.  A 1 MB arena overflows: the calls
    that do not fit sum immediately and the flush reports the arena they needed."""
    rng = np.random.default_rng(3)
    M = 1 << 21
    jobs = []
    for (m, K, N) in [(174592, 64, 64), (M, 16, 96), (174592, 64, 64)]:
        pyr = Pyr(1, [(m, 1)])
        jobs.append((pyr, K, N, g(rnd(rng, m, K), "bf16"), g(rnd(rng, m, N), "bf16")))
    xs = g(rnd(rng, 4 * 64 * 64, 3), "bf16")
    dys = g(rnd(rng, 4 * 32 * 32, 32), "bf16")

    def run(defer):
        outs = [zeros(N, K) for (_, K, N, _, _) in jobs[:2]]
        dbs = [zeros(N) for (_, K, N, _, _) in jobs[:2]]
        dstem = zeros(27 * 32)
        arena = torch.empty(arena_mb << 20, dtype=torch.uint8, device=DEV)
        if defer:
            L.call("edet_partials_defer", vp(arena), arena.numel())
        for i, (pyr, K, N, x, dy) in enumerate(jobs):
            o = 0 if i == 2 else i  # the third adds into the first's dW / db
            L.call("edet_conv1x1_wgrad", L.BF16, LazyDesc(x, pyr, K).c, pyr.c, K, vp(dy), N, N, vp(outs[o]),
                   vp(dbs[o]), stream())
        L.call("edet_stem_wgrad", L.BF16, vp(xs), 4, 64, 64, vp(dys), 32, vp(dstem), stream())
        need = ctypes.c_size_t(0)
        if defer:
            L.call("edet_partials_flush", ctypes.byref(need), stream())
        torch.cuda.synchronize()
        return outs, dbs, dstem, need.value

    (o0, b0, s0, _), (o1, b1, s1, need) = run(False), run(True)
    # (sums of more than 32 splits add their chunk sums with fp32 atomics in both paths)
    for a, b in zip(o1 + b1 + [s1], o0 + b0 + [s0]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-3)
    assert need > 0
    if arena_mb == 1:
        assert need > (1 << 20)
    with pytest.raises(L.EdetError, match="no deferral window"):
        L.call("edet_partials_flush", None, stream())


# ----------------------------------------------------------------- depthwise
def dw_ref(v, pyr_in, k, s, w):  # v: fp64 [rows, C] values; returns [rows_out, C]
    outs = []
    C = v.shape[1]
    pout = pyr_in.strided(s)
    res = torch.zeros(pout.rows, C, dtype=torch.float64)
    for sg in range(pyr_in.nseg):
        H, W = pyr_in.sizes[sg]
        xi = v[pyr_in.seg_slice(sg)].view(pyr_in.batch, H, W, C).permute(0, 3, 1, 2)
        OH, OW = (H + s - 1) // s, (W + s - 1) // s
        ph = max((OH - 1) * s + k - H, 0)
        pw = max((OW - 1) * s + k - W, 0)
        xi = Fn.pad(xi, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
        wt = w.t().reshape(C, 1, k, k)
        y = Fn.conv2d(xi, wt, stride=s, groups=C)
        res[pout.seg_slice(sg)] = y.permute(0, 2, 3, 1).reshape(-1, C)
    return res


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("k,s,H,W,C,lazy,nseg", [(3, 1, 16, 16, 32, 0, 1), (3, 2, 17, 13, 96, 1, 1),
                                                 (5, 2, 20, 9, 144, 1, 1), (5, 1, 11, 12, 40, 2, 1),
                                                 (3, 1, 9, 9, 64, 3, 2), (3, 1, 6, 7, 2112, 1, 1),
                                                 (5, 2, 9, 8, 2112, 1, 1),
                                                 # forms chosen per shape in round 2 (dw_form):
                                                 # k5 C = 1152 rows wgrad, k3 C = 480 rows fwd,
                                                 # C = 64 tiles fwd / pipelined-tile wgrad
                                                 (5, 1, 10, 11, 1152, 1, 1), (3, 1, 8, 9, 480, 1, 1),
                                                 (3, 1, 12, 10, 64, 1, 1)])
def test_dwconv_fwd_bwd(dt, k, s, H, W, C, lazy, nseg, workspace_mode):
    rng = np.random.default_rng(k * 100 + s * 10 + H)
    B = 2
    pin = Pyr(B, [(H, W), ((H + 1) // 2, (W + 1) // 2)]) if nseg == 2 else Pyr(B, [(H, W)])
    pout = pin.strided(s)
    x = pyr_data(rng, pin, C, dt)
    bn = make_bn(x, pin, C, rng) if lazy else None
    gate = g(torch.rand(B, C), "f32") if lazy == 1 else None
    lz = LazyDesc(x, pin, C, bn=bn, act=1 if lazy in (1, 3) else 0, gate=gate)
    w = g(rnd(rng, k * k, C, scale=0.3), dt)
    y = torch.empty(pout.rows, C, dtype=TDT[dt], device=DEV)
    st = stats_out(nseg, C)
    L.call("edet_dwconv_fwd", DT[dt], lz.c, pin.c, C, k, s, vp(w), vp(y), pout.c, stat_out(st), stream())
    v = lz.cpu_value().requires_grad_(True)
    wr = w.double().cpu().requires_grad_(True)
    ref = dw_ref(v, pin, k, s, wr)
    for sg in range(nseg):
        sl = pout.seg_slice(sg)
        close(y[sl], ref[sl].detach(), dt)
        close(st[sg][0], ref[sl].detach().sum(0), dt, scale=pout.seg_rows(sg) ** 0.5 * 4)
    # backward
    dy = pyr_data(rng, pout, C, dt)
    dyc = dy.double().cpu()
    mask = torch.zeros(pout.rows, 1, dtype=torch.float64)
    for sg in range(nseg):
        mask[pout.seg_slice(sg)] = 1
    (ref * dyc * mask).sum().backward()
    dx = g(torch.full((pin.rows, C), 0.25), dt)
    L.call("edet_dwconv_dgrad", DT[dt], vp(dy), pout.c, C, k, s, vp(w), vp(dx), pin.c, 1, stream())
    for sg in range(nseg):
        sl = pin.seg_slice(sg)
        close(dx[sl], v.grad[sl] + 0.25, dt)
    dw = zeros(k * k, C)
    L.call("edet_dwconv_wgrad", DT[dt], lz.c, pin.c, C, k, s, vp(dy), pout.c, vp(dw), stream())
    close(dw, wr.grad, dt, scale=pout.rows ** 0.5 * 3)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("k,H,W,C,act,nseg,fold,acc,B", [
    (3, 16, 16, 32, 1, 1, True, 0, 2), (5, 11, 12, 40, 1, 1, True, 0, 2), (3, 9, 9, 64, 1, 2, True, 0, 2),
    (5, 10, 11, 1152, 1, 1, True, 0, 2), (3, 34, 37, 96, 0, 1, True, 0, 2), (5, 33, 20, 144, 1, 1, False, 1, 2),
    (3, 8, 9, 480, 1, 1, False, 0, 2), (5, 70, 66, 64, 1, 1, True, 0, 2),
    # enough tiles for several tiles per block: the tiled form's chunks then span images
    # (one 16 x 16 tile per image; a two-level pyramid of one-tile planes)
    (5, 16, 16, 1152, 1, 1, True, 0, 64), (3, 8, 8, 64, 1, 2, True, 0, 400)])
def test_dwconv_bwd_fused(dt, k, H, W, C, act, nseg, fold, acc, B):
    """edet_dwconv_bwd (stride 1): dx, the filter gradient and the folded BN-backward sums of
    the input's BatchNorm from one pass, against fp64 autograd and against the separate entry
    points (dgrad, wgrad, lazy_bwd_reduce over the same dx)."""
    rng = np.random.default_rng(k * 1000 + H * 10 + C)
    pin = Pyr(B, [(H, W), ((H + 1) // 2, (W + 1) // 2)]) if nseg == 2 else Pyr(B, [(H, W)])
    x = pyr_data(rng, pin, C, dt, scale=2.0)
    bn = make_bn(x, pin, C, rng)
    lz = LazyDesc(x, pin, C, bn=bn, act=act)
    w = g(rnd(rng, k * k, C, scale=0.3), dt)
    dy = pyr_data(rng, pin, C, dt)
    base = 0.25 if acc else 0.0
    dx = g(torch.full((pin.rows, C), base), dt)
    dw = zeros(k * k, C)
    sums_t, sums = bngrad64(nseg, C) if fold else (None, None)
    L.call("edet_dwconv_bwd", DT[dt], lz.c, pin.c, C, k, 1, vp(dy), pin.c, vp(w), vp(dx), acc, vp(dw), sums,
           stream())
    # fp64 autograd reference through v = act(bn(x)) and the stencil
    v = lz.cpu_value().requires_grad_(True)
    wr = w.double().cpu().requires_grad_(True)
    mask = torch.zeros(pin.rows, 1, dtype=torch.float64)
    for sg in range(nseg):
        mask[pin.seg_slice(sg)] = 1
    (dw_ref(v, pin, k, 1, wr) * dy.double().cpu() * mask).sum().backward()
    for sg in range(nseg):
        sl = pin.seg_slice(sg)
        close(dx[sl], v.grad[sl] + base, dt)
    close(dw, wr.grad, dt, scale=pin.rows ** 0.5 * 3)
    # the separate entry points agree
    dx2 = g(torch.full((pin.rows, C), base), dt)
    L.call("edet_dwconv_dgrad", DT[dt], vp(dy), pin.c, C, k, 1, vp(w), vp(dx2), pin.c, acc, stream())
    dw2 = zeros(k * k, C)
    L.call("edet_dwconv_wgrad", DT[dt], lz.c, pin.c, C, k, 1, vp(dy), pin.c, vp(dw2), stream())
    for sg in range(nseg):
        sl = pin.seg_slice(sg)
        close(dx[sl], dx2[sl].double(), dt)
    close(dw, dw2, "f32", rtol=1e-4, atol=1e-4 * pin.rows ** 0.5)
    if not fold:
        return
    # folded sums = the reduce pass over (x, dv = dx), and = fp64 du / du * xhat sums
    acc2_t, acc2 = bngrad64(nseg, C)
    L.call("edet_lazy_bwd_reduce", DT[dt], lz.c, pin.c, C, vp(dx), None, None, acc2, stream())
    xc = x[:, :C].double().cpu()
    for sg in range(nseg):
        sl = pin.seg_slice(sg)
        n = pin.seg_rows(sg)
        su, sq, ga, be = (t.double().cpu() for t in bn[sg])
        mean = su / n
        rstd = 1.0 / torch.sqrt(torch.clamp(sq / n - mean * mean, min=0) + 1e-3)
        xhat = (xc[sl] - mean) * rstd
        u = xhat * ga + be
        sgm = torch.sigmoid(u)
        du = v.grad[sl] * (sgm * (1 + u * (1 - sgm)) if act else 1.0)
        close(sums_t[1, sg], du.sum(0), dt, scale=n ** 0.5 * 2)
        close(sums_t[0, sg], (du * xhat).sum(0), dt, scale=n ** 0.5 * 2)
        # every fold kernel sums the stored (rounded) dx the reduce pass reads: the two differ in
        # the fp32 partial-sum order only (bf16 bar 1e-3)
        tol = dict(rtol=1e-4, atol=1e-4 * n ** 0.5) if dt == "f32" else dict(rtol=1e-3, atol=1e-3 * n ** 0.5)
        torch.testing.assert_close(sums_t[:, sg].cpu(), acc2_t[:, sg].cpu(), **tol)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("B,H,W,N,K", [(4, 16, 16, 192, 1152), (2, 32, 32, 80, 480), (3, 8, 8, 40, 144),
                                       (2, 32, 32, 112, 672), (5, 16, 16, 320, 1152),
                                       # the separate-pass routes: a narrow dgrad, a 7 x 7 plane
                                       (2, 16, 16, 24, 144), (3, 7, 7, 80, 480)])
def test_conv1x1_dgrad_sesum_equals_dgrad_then_gate_bn_reduce(dt, B, H, W, N, K):
    """edet_conv1x1_dgrad_sesum (the project conv's dgrad with the SE-gated depthwise output's
    five per-image backward sums in its epilogue) against the two passes it replaces:
    edet_conv1x1_dgrad, then edet_gate_bn_reduce over (y, dv = dx)."""
    rng = np.random.default_rng(B * 100 + N + K)
    pyr = Pyr(B, [(H, W)])
    M = pyr.rows
    dy = g(rnd(rng, M, N), dt)
    w = g(rnd(rng, N, K, scale=1 / math.sqrt(N)), dt)
    ldn = (N + 7) // 8 * 8
    wkn = torch.zeros(K, ldn)
    wkn[:, :N] = w.float().cpu().t()
    wkn = g(wkn, dt)
    y = pyr_data(rng, pyr, K, dt, scale=1.5)
    lzy = LazyDesc(y, pyr, K, bn=make_bn(y, pyr, K, rng), act=1, gate=g(torch.rand(B, K) + 0.5, "f32"))
    dx1 = torch.empty(M, K, dtype=TDT[dt], device=DEV)
    L.call("edet_conv1x1_dgrad", DT[dt], vp(dy), N, pyr.c, N, vp(wkn), K, vp(dx1), K, 0, stream())
    s1 = zeros64(5, B, K)
    L.call("edet_gate_bn_reduce", DT[dt], lzy.c, B, H * W, K, vp(dx1), vp(s1), stream())
    dx2 = torch.empty(M, K, dtype=TDT[dt], device=DEV)
    s2 = zeros64(5, B, K)
    L.call("edet_conv1x1_dgrad_sesum", DT[dt], vp(dy), N, pyr.c, N, vp(wkn), K, vp(dx2), K, lzy.c, vp(s2), stream())
    torch.cuda.synchronize()
    close(dx2, dx1.double(), dt, rtol=1e-5 if dt == "f32" else 8e-3, atol=1e-5 if dt == "f32" else 8e-3)
    # the sums of (slightly) different dx roundings in bf16: compare against the fp64 sums of
    # each kernel's own dx, then the two paths against each other at the fp32-order level
    ref2 = zeros64(5, B, K)
    L.call("edet_gate_bn_reduce", DT[dt], lzy.c, B, H * W, K, vp(dx2), vp(ref2), stream())
    torch.cuda.synchronize()
    for q in range(5):
        close(s2[q], ref2[q], "f32", rtol=1e-4, atol=1e-4 * (H * W) ** 0.5 * float(ref2[q].abs().max() + 1e-30) / 4)
        if dt == "f32":
            close(s2[q], s1[q], "f32", rtol=1e-4, atol=1e-4 * (H * W) ** 0.5 * float(s1[q].abs().max() + 1e-30) / 4)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("k,H,W,C,B,fold,acc,yact,gate,dsq", [
    (3, 16, 16, 32, 2, True, 0, 1, 1, 1), (5, 11, 12, 48, 2, True, 0, 1, 1, 1), (5, 9, 9, 1152, 2, True, 0, 1, 1, 1),
    (3, 17, 20, 144, 3, False, 1, 1, 1, 1), (3, 40, 33, 96, 2, True, 0, 1, 1, 0), (5, 32, 32, 240, 4, True, 0, 0, 0, 1),
    (3, 8, 8, 672, 8, True, 0, 1, 1, 1)])
def test_dwconv_bwd_lazy_equals_apply_then_bwd(dt, k, H, W, C, B, fold, acc, yact, gate, dsq):
    """edet_dwconv_bwd_lazy (the SE-gated MBConv depthwise backward with d(raw y) built while
    the dy window loads) against the pass it replaces: edet_lazy_bwd_apply writing d(raw y),
    then edet_dwconv_bwd over it.  Same dx (the built dy is rounded to the storage dtype as the
    apply stores it), filter gradient, input-BN fold sums and y's gamma / beta gradients."""
    rng = np.random.default_rng(k * 1000 + H * 10 + C + B)
    pin = Pyr(B, [(H, W)])
    x = pyr_data(rng, pin, C, dt, scale=2.0)
    lzx = LazyDesc(x, pin, C, bn=make_bn(x, pin, C, rng), act=1)  # the expand output swish(bn0(x))
    y = pyr_data(rng, pin, C, dt, scale=1.5)  # the depthwise output's raw y: swish(bn1(y)) * gate
    gt = g(torch.rand(B, C) + 0.5, "f32") if gate else None
    lzy = LazyDesc(y, pin, C, bn=make_bn(y, pin, C, rng), act=yact, gate=gt)
    dv = pyr_data(rng, pin, C, dt)
    dsqt = g(rnd(rng, B, C) * 0.1, "f32") if dsq else None
    accy_t, accy = bngrad64(1, C)  # y's final BN-backward sums (the reduce over (y, dv))
    L.call("edet_lazy_bwd_reduce", DT[dt], lzy.c, pin.c, C, vp(dv), None, vp(dsqt), accy, stream())
    w = g(rnd(rng, k * k, C, scale=0.3), dt)
    base = 0.25 if acc else 0.0
    # unfused: apply pass, then the fused backward over the materialised d(raw y)
    gr1 = [(zeros(C), zeros(C))]
    draw = torch.empty(pin.rows, C, dtype=TDT[dt], device=DEV)
    L.call("edet_lazy_bwd_apply", DT[dt], lzy.c, pin.c, C, vp(dv), None, vp(dsqt), accy, seg_out(gr1), vp(draw), 0,
           stream())
    dx1, dw1 = g(torch.full((pin.rows, C), base), dt), zeros(k * k, C)
    f1_t, f1 = bngrad64(1, C) if fold else (None, None)
    L.call("edet_dwconv_bwd", DT[dt], lzx.c, pin.c, C, k, 1, vp(draw), pin.c, vp(w), vp(dx1), acc, vp(dw1), f1,
           stream())
    # fused: the lazy dy
    gr2 = [(zeros(C), zeros(C))]
    d = L.DgradLazy()
    d.dv, d.y, d.dsq, d.acc, d.grads = dv.data_ptr(), lzy.c, dsqt.data_ptr() if dsq else None, accy, seg_out(gr2)
    dx2, dw2 = g(torch.full((pin.rows, C), base), dt), zeros(k * k, C)
    f2_t, f2 = bngrad64(1, C) if fold else (None, None)
    L.call("edet_dwconv_bwd_lazy", DT[dt], lzx.c, pin.c, C, k, d, pin.c, vp(w), vp(dx2), acc, vp(dw2), f2, stream())
    torch.cuda.synchronize()
    assert torch.equal(gr2[0][0], gr1[0][0]) and torch.equal(gr2[0][1], gr1[0][1])
    assert torch.equal(gr2[0][0], accy_t[0, 0].float())
    rms = float(dx1.double().pow(2).mean().sqrt())
    if dt == "f32":
        close(dx2, dx1, "f32", rtol=1e-5, atol=1e-5 * rms)
    else:  # one bf16 rounding of dx (the unfused fp32 path may take a different kernel order)
        close(dx2, dx1, "bf16", rtol=8e-3, atol=8e-3 * rms)
    n = pin.rows
    close(dw2, dw1, "f32", rtol=1e-4, atol=(1e-4 if dt == "f32" else 1e-3) * float(dw1.abs().max()))
    if fold:
        close(f2_t, f1_t, "f32", scale=n ** 0.5, rtol=1e-3 if dt == "bf16" else 1e-4)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("k,s,H,W,C,act,nseg,B", [(3, 2, 17, 13, 96, 1, 1, 3), (5, 2, 20, 9, 144, 1, 1, 3),
                                                 (3, 2, 33, 32, 240, 1, 1, 3), (5, 2, 9, 8, 672, 0, 1, 3),
                                                 (5, 2, 12, 12, 1152, 1, 1, 3), (3, 1, 0, 0, 64, 1, 2, 3),
                                                 # >= 2^20 input rows: the folded k_dw4_dgrad kernel
                                                 # itself (the D0 B=32 256^2 stride-2 layer's route;
                                                 # the shapes above take dgrad + reduce)
                                                 (3, 2, 256, 256, 96, 1, 1, 16), (3, 2, 255, 250, 32, 0, 1, 17),
                                                 (3, 2, -1, -1, 32, 1, 2, 16)])
def test_dwconv_dgrad_fold(dt, k, s, H, W, C, act, nseg, B):
    """edet_dwconv_dgrad_fold (the stride-2 MBConv depthwise backward): dx equal to
    edet_dwconv_dgrad's, and the fold sums of the input's BN equal to edet_lazy_bwd_reduce over
    (x, dx) -- the pass it replaces (fp32 partial-sum order only)."""
    rng = np.random.default_rng(k * 100 + s * 10 + C + act + H)
    if H < 0:  # two-segment pyramid past the fold kernel's row threshold
        pin = Pyr(B, [(256, 256), (31, 17)])
    else:
        pin = Pyr(B, [(11, 7), (6, 4)]) if nseg == 2 else Pyr(B, [(H, W)])
    pout = pin.strided(s)
    x = pyr_data(rng, pin, C, dt, scale=2.0)
    bn = make_bn(x, pin, C, rng)
    lz = LazyDesc(x, pin, C, bn=bn, act=act)
    dy = pyr_data(rng, pout, C, dt)
    w = g(rnd(rng, k * k, C, scale=0.3), dt)
    dx = torch.empty(pin.rows, C, dtype=TDT[dt], device=DEV)
    acc_t, acc = bngrad64(nseg, C)
    L.call("edet_dwconv_dgrad_fold", DT[dt], vp(dy), pout.c, C, k, s, vp(w), vp(dx), pin.c, lz.c, acc, stream())
    dx2 = torch.empty_like(dx)
    L.call("edet_dwconv_dgrad", DT[dt], vp(dy), pout.c, C, k, s, vp(w), vp(dx2), pin.c, 0, stream())
    ref_t, ref = bngrad64(nseg, C)
    L.call("edet_lazy_bwd_reduce", DT[dt], lz.c, pin.c, C, vp(dx2), None, None, ref, stream())
    for sg in range(nseg):
        sl = pin.seg_slice(sg)
        if pin.rows < (1 << 20):  # dgrad + reduce: the same dgrad kernel
            assert torch.equal(dx[sl], dx2[sl])
        else:  # the folded patch kernel against the plain dgrad route: same taps, own tiling
            close(dx[sl], dx2[sl].double(), dt)
        close(acc_t[:, sg], ref_t[:, sg], "f32", scale=pin.seg_rows(sg) ** 0.5, rtol=1e-4)


@pytest.mark.parametrize("k,s,B,H,C", [(5, 1, 16, 64, 240), (3, 1, 8, 100, 64), (5, 2, 16, 72, 144)])
def test_dwconv_long_blocks(k, s, B, H, C):
    """Forward and weight gradient at batch sizes where a row-streaming block walks many
    output rows (its LDS ring of K+S input rows wraps several times) and strips end inside
    the image."""
    rng = np.random.default_rng(k + H)
    pin = Pyr(B, [(H, H)])
    pout = pin.strided(s)
    x = pyr_data(rng, pin, C, "bf16")
    lz = LazyDesc(x, pin, C, bn=make_bn(x, pin, C, rng), act=1, gate=g(torch.rand(B, C), "f32"))
    w = g(rnd(rng, k * k, C, scale=0.3), "bf16")
    y = torch.empty(pout.rows, C, dtype=TDT["bf16"], device=DEV)
    st = stats_out(1, C)
    L.call("edet_dwconv_fwd", DT["bf16"], lz.c, pin.c, C, k, s, vp(w), vp(y), pout.c, stat_out(st), stream())
    ref = dw_ref(lz.cpu_value(), pin, k, s, w.double().cpu())
    close(y, ref, "bf16")
    close(st[0][0], ref.sum(0), "bf16", scale=pout.rows ** 0.5 * 4)
    close(st[0][1], (ref * ref).sum(0), "bf16", scale=pout.rows ** 0.5 * 4)
    # weight gradient over the same blocks
    v = lz.cpu_value()
    wr = w.double().cpu().requires_grad_(True)
    dy = pyr_data(rng, pout, C, "bf16")
    (dw_ref(v, pin, k, s, wr) * dy.double().cpu()).sum().backward()
    dw = zeros(k * k, C)
    L.call("edet_dwconv_wgrad", DT["bf16"], lz.c, pin.c, C, k, s, vp(dy), pout.c, vp(dw), stream())
    close(dw, wr.grad, "bf16", scale=pout.rows ** 0.5 * 3)


# ----------------------------------------------------------------- lazy backward (BN train bwd)
@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("C,act,gate,dsq,scale,nseg", [(40, 0, 0, 0, 0, 1), (96, 1, 1, 1, 0, 1), (64, 1, 0, 0, 1, 2),
                                                        (144, 1, 0, 0, 0, 1), (24, 0, 0, 0, 0, 1), (240, 1, 1, 0, 0, 1),
                                                        (672, 1, 1, 1, 0, 1), (672, 1, 0, 0, 0, 1),
                                                        # the channel-sliced apply (C >= 1024, M <= 16384)
                                                        (1152, 1, 1, 1, 0, 1), (1152, 1, 0, 0, 1, 2)])
def test_lazy_backward(dt, C, act, gate, dsq, scale, nseg):
    rng = np.random.default_rng(C + act * 7 + nseg)
    B = 3
    pyr = Pyr(B, [(11, 7), (6, 4)]) if nseg == 2 else Pyr(B, [(9, 10)])
    if C == 672:  # M = 32768: the long-chunk plans of the wide layers
        B = 32
        pyr = Pyr(B, [(32, 32)])
    elif C == 1152 and nseg == 1:  # M = 8192: 18 channel slices x 64 chunks
        B = 32
        pyr = Pyr(B, [(16, 16)])
    x = pyr_data(rng, pyr, C, dt, scale=2.0)
    bn = make_bn(x, pyr, C, rng)
    gt = g(torch.rand(B, C) + 0.5, "f32") if gate else None
    lz = LazyDesc(x, pyr, C, bn=bn, act=act, gate=gt)
    dv = pyr_data(rng, pyr, C, dt)
    dsqt = g(rnd(rng, B, C) * 0.1, "f32") if dsq else None
    sc = g(torch.tensor(rng.choice([0.0, 1.25], size=(nseg, B)), dtype=torch.float32), "f32") if scale else None
    grads = [(zeros(C), zeros(C)) for _ in range(nseg)]
    so = seg_out(grads)
    acc_t, acc = bngrad64(nseg, C)
    L.call("edet_lazy_bwd_reduce", DT[dt], lz.c, pyr.c, C, vp(dv), vp(sc), vp(dsqt), acc, stream())
    dx = torch.empty(pyr.rows, C, dtype=TDT[dt], device=DEV)
    L.call("edet_lazy_bwd_apply", DT[dt], lz.c, pyr.c, C, vp(dv), vp(sc), vp(dsqt), acc, so, vp(dx), 0, stream())
    for sg in range(nseg):  # fp32 parameter gradients are the fp64 sums, written once
        assert torch.equal(grads[sg][0], acc_t[0, sg].float()) and torch.equal(grads[sg][1], acc_t[1, sg].float())
    # reference: autograd through BN(train, batch stats recomputed) -> act -> gate, with dsq term
    xc = x.double().cpu()
    for sg in range(nseg):
        sl = pyr.seg_slice(sg)
        xs = xc[sl].clone().requires_grad_(True)
        su, sq, ga, be = (t.double().cpu() for t in bn[sg])
        ga = ga.clone().requires_grad_(True)
        be = be.clone().requires_grad_(True)
        n = xs.shape[0]
        mean = xs.mean(0)
        var = ((xs - mean) ** 2).mean(0)
        u = (xs - mean) / torch.sqrt(var + 1e-3) * ga + be
        a = u * torch.sigmoid(u) if act else u
        hw = pyr.sizes[sg][0] * pyr.sizes[sg][1]
        d = dv[sl].double().cpu()
        if sc is not None:
            d = d * sc[sg].double().cpu().repeat_interleave(hw)[:, None]
        if gt is not None:
            d = d * gt.double().cpu().repeat_interleave(hw, 0)
        if dsqt is not None:
            d = d + dsqt.double().cpu().repeat_interleave(hw, 0)
        (a * d).sum().backward()
        close(dx[sl], xs.grad, dt, scale=4)
        close(grads[sg][1], be.grad, dt, scale=n ** 0.5 * 2)
        close(grads[sg][0], ga.grad, dt, scale=n ** 0.5 * 2)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("k,s,H,W,C", [(3, 1, 16, 16, 32), (3, 2, 17, 13, 96), (5, 2, 20, 9, 144),
                                       (5, 1, 11, 12, 40), (3, 1, 8, 9, 480), (5, 1, 10, 11, 1152),
                                       (3, 1, 6, 7, 2112), (5, 2, 9, 8, 672), (3, 1, 40, 70, 64)])
def test_dwconv_fwd_squeeze(dt, k, s, H, W, C):
    """Inference (layers/se.py:36 on mb_conv_block.py:147-150, call(training=False)):
    edet_dwconv_fwd_squeeze writes y = dwconv(v(x)) and, from the same pass, the SE squeeze
    mean_hw swish(bn(y)) of y as stored, with y's BN on moving statistics.  y against the fp64
    stencil; the squeeze against edet_se_squeeze over the y it wrote (same inputs, only the
    fp32 partial-sum order differs) and against fp64 of that y."""
    rng = np.random.default_rng(k * 1000 + s * 100 + C)
    B = 3
    pin = Pyr(B, [(H, W)])
    pout = pin.strided(s)
    OH, OW = pout.sizes[0]
    x = pyr_data(rng, pin, C, dt)
    lz = LazyDesc(x, pin, C, bn=make_bn(x, pin, C, rng), act=1)
    w = g(rnd(rng, k * k, C, scale=0.3), dt)
    y = torch.empty(pout.rows, C, dtype=TDT[dt], device=DEV)
    # y's BatchNorm in inference form: sums that give the moving mean / variance over pout.rows
    n = pout.rows
    mean, var = rng.normal(0, 0.3, C), rng.uniform(0.2, 2.0, C)
    ybn = [(torch.tensor(mean * n, dtype=torch.float64, device=DEV),
            torch.tensor((var + mean * mean) * n, dtype=torch.float64, device=DEV),
            torch.tensor(rng.uniform(0.5, 1.5, C), dtype=torch.float32, device=DEV),
            torch.tensor(rng.uniform(-0.5, 0.5, C), dtype=torch.float32, device=DEV))]
    ylz = LazyDesc(y, pout, C, bn=ybn, act=1)
    sq = zeros64(B, C)
    L.call("edet_dwconv_fwd_squeeze", DT[dt], lz.c, pin.c, C, k, s, vp(w), vp(y), pout.c, ylz.c, vp(sq), stream())
    ref = dw_ref(lz.cpu_value(), pin, k, s, w.double().cpu())
    close(y, ref, dt)
    sep = zeros64(B, C)
    L.call("edet_se_squeeze", DT[dt], ylz.c, B, OH * OW, C, vp(sep), stream())
    close(sq, sep, "f32", rtol=1e-5, atol=1e-6)
    close(sq, ylz.cpu_value().view(B, OH * OW, C).mean(1), "f32", rtol=1e-5, atol=1e-5)
    # a gate on the squeezed value is refused (the squeeze is of the pre-gate value)
    bad = LazyDesc(y, pout, C, bn=ybn, act=1, gate=zeros(B, C))
    with pytest.raises(L.EdetError):
        L.call("edet_dwconv_fwd_squeeze", DT[dt], lz.c, pin.c, C, k, s, vp(w), vp(y), pout.c, bad.c, vp(sq),
               stream())


# ----------------------------------------------------------------- SE
@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("C,R,B", [(96, 4, 3), (1152, 48, 3), (520, 100, 3), (200, 70, 40)])
def test_squeeze_excite(dt, C, R, B):
    """SE forward and backward (layers/se.py:35-39) against fp64 autograd; R > 64 and B > 32
    take the weight-gradient tiles' r-batch and image-chunk loops."""
    rng = np.random.default_rng(5 + C)
    H, W = 9, 7
    pyr = Pyr(B, [(H, W)])
    x = pyr_data(rng, pyr, C, dt)
    bn = make_bn(x, pyr, C, rng)
    lz = LazyDesc(x, pyr, C, bn=bn, act=1)
    w1, b1 = g(rnd(rng, R, C, scale=0.2)), g(rnd(rng, R, scale=0.1))
    w2, b2 = g(rnd(rng, C, R, scale=0.3)), g(rnd(rng, C, scale=0.1))
    s = zeros64(B, C)
    L.call("edet_se_squeeze", DT[dt], lz.c, B, H * W, C, vp(s), stream())
    z1, gate = zeros(B, R), zeros(B, C)
    L.call("edet_se_fwd", B, C, R, vp(s), vp(w1), vp(b1), vp(w2), vp(b2), vp(z1), vp(gate), stream())
    v = lz.cpu_value()
    sref = v.view(B, H * W, C).mean(1)
    close(s, sref, dt)
    W1, B1, W2, B2 = (t.double().cpu().requires_grad_(True) for t in (w1, b1, w2, b2))
    sr = sref.clone().requires_grad_(True)
    zr = sr @ W1.t() + B1
    gr = torch.sigmoid((zr * torch.sigmoid(zr)) @ W2.t() + B2)
    close(gate, gr.detach(), dt)
    # backward given dgate
    dgate = rnd(rng, B, C).double().to(DEV)  # fp64 gate-gradient accumulator (edet_gate_grad)
    dws = [zeros(R, C), zeros(R), zeros(C, R), zeros(C)]
    dsq = zeros(B, C)
    L.call("edet_se_bwd", B, C, R, H * W, vp(s), vp(z1), vp(gate), vp(dgate), vp(w1), vp(w2), vp(dws[0]), vp(dws[1]),
           vp(dws[2]), vp(dws[3]), vp(dsq), vp(zeros(B, R)), stream())
    (gr * dgate.double().cpu()).sum().backward()
    for a, b in zip(dws, (W1.grad, B1.grad, W2.grad, B2.grad)):
        close(a, b, "f32", rtol=1e-4, atol=1e-4)
    close(dsq, sr.grad / (H * W), "f32", rtol=1e-4, atol=1e-5)
    # gate grad: sum_hw dv * v
    dv = pyr_data(rng, pyr, C, dt)
    dg = zeros64(B, C)
    L.call("edet_gate_grad", DT[dt], lz.c, B, H * W, C, vp(dv), vp(dg), stream())
    close(dg, (dv.double().cpu() * v).view(B, H * W, C).sum(1), dt, scale=8)


# ----------------------------------------------------------------- maxpool / fuse / residual / stem
def maxpool_ref(v, B, H, W, C):
    xi = v.view(B, H, W, C).permute(0, 3, 1, 2)
    OH, OW = (H + 1) // 2, (W + 1) // 2
    ph, pw = max((OH - 1) * 2 + 3 - H, 0), max((OW - 1) * 2 + 3 - W, 0)
    xi = Fn.pad(xi, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=-math.inf)
    return Fn.max_pool2d(xi, 3, 2).permute(0, 2, 3, 1).reshape(-1, C)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("H,W", [(16, 16), (9, 7)])
def test_maxpool(dt, H, W):
    rng = np.random.default_rng(H * W)
    B, C = 2, 64
    pyr = Pyr(B, [(H, W)])
    x = pyr_data(rng, pyr, C, dt)
    bn = make_bn(x, pyr, C, rng)
    lz = LazyDesc(x, pyr, C, bn=bn)
    OH, OW = (H + 1) // 2, (W + 1) // 2
    y = torch.empty(B * OH * OW, C, dtype=TDT[dt], device=DEV)
    L.call("edet_maxpool_fwd", DT[dt], lz.c, B, H, W, C, vp(y), stream())
    v = lz.cpu_value().requires_grad_(True)
    ref = maxpool_ref(v, B, H, W, C)
    close(y, ref.detach(), dt)
    dy = g(rnd(rng, B * OH * OW, C), dt)
    (ref * dy.double().cpu()).sum().backward()
    dx = torch.empty(B * H * W, C, dtype=TDT[dt], device=DEV)
    L.call("edet_maxpool_bwd", DT[dt], lz.c, B, H, W, C, vp(dy), vp(dx), 0, stream())
    if dt == "f32":
        close(dx, v.grad, dt)
    else:  # bf16 ties may route differently; totals must agree
        close(dx.double().cpu().sum(0), v.grad.sum(0), dt, scale=8)


@pytest.mark.parametrize("H,W", [(16, 16), (9, 7), (8, 8), (4, 4), (3, 5)])
def test_maxpool_bwd_bf16_exact(H, W):
    """bf16 max-pool backward (the 5 x 5 neighbourhood gather) routes every dy to its window's
    argmax exactly: per-channel distinct integer inputs (no ties) and integer dy, so the expected
    dx is exact in bf16 (resample_feature_map.py's max_pooling2d, SAME padding)."""
    rng = np.random.default_rng(7 * H + W)
    B, C = 2, 64
    pyr = Pyr(B, [(H, W)])
    xn = np.stack([np.stack([rng.permutation(H * W) for _ in range(C)], axis=1) for _ in range(B)])
    x = torch.tensor(xn.reshape(B * H * W, C), dtype=torch.bfloat16, device=DEV)
    lz = LazyDesc(x, pyr, C)
    OH, OW = (H + 1) // 2, (W + 1) // 2
    dy = torch.tensor(rng.integers(-4, 5, (B * OH * OW, C)), dtype=torch.bfloat16, device=DEV)
    dx = torch.empty(B * H * W, C, dtype=torch.bfloat16, device=DEV)
    L.call("edet_maxpool_bwd", DT["bf16"], lz.c, B, H, W, C, vp(dy), vp(dx), 0, stream())
    v = torch.tensor(xn.reshape(B * H * W, C), dtype=torch.float64).requires_grad_(True)
    (maxpool_ref(v, B, H, W, C) * dy.double().cpu()).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(dx.double().cpu(), v.grad)


def test_zero_ranges():
    """edet_zero_ranges (the train step's per-step accumulators in one launch): ranges of odd
    byte counts inside one guarded buffer are zeroed exactly, their neighbours untouched."""
    buf = torch.full((1 << 22,), 7, dtype=torch.uint8, device=DEV)
    spans = [(0, 40), (256, 1 << 20), (2 << 20, 17), (3 << 20, 16), (3 << 20 | 4096, 15 * 16 + 9), (4000000, 0)]
    ptrs = (ctypes.c_void_p * len(spans))(*[buf.data_ptr() + o for o, _ in spans])
    sizes = (ctypes.c_size_t * len(spans))(*[n for _, n in spans])
    L.call("edet_zero_ranges", len(spans), ptrs, sizes, stream())
    torch.cuda.synchronize()
    want = torch.full((1 << 22,), 7, dtype=torch.uint8)
    for o, n in spans:
        want[o:o + n] = 0
    assert torch.equal(buf.cpu(), want)
    with pytest.raises(L.EdetError):  # a misaligned range is refused
        L.call("edet_zero_ranges", 1, (ctypes.c_void_p * 1)(buf.data_ptr() + 8), (ctypes.c_size_t * 1)(16), stream())


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("H,W", [(16, 16), (9, 7), (8, 8), (3, 5), (64, 64)])
@pytest.mark.parametrize("acc", [0, 1])
def test_maxpool_taps_equal_recompute(dt, H, W, acc):
    """edet_maxpool_fwd_taps / _bwd_taps (the training route of ops.maxpool, resample_p6/p7)
    against edet_maxpool_fwd / _bwd, which re-evaluate the windows: the same pooled values and,
    bit for bit, the same dx (the taps record the forward's own argmax, ties included -- bf16
    inputs with many ties), accumulating into dx or not."""
    rng = np.random.default_rng(3 * H + W + acc)
    B, C = 3, 64
    pyr = Pyr(B, [(H, W)])
    x = pyr_data(rng, pyr, C, dt)
    if dt == "bf16":  # coarse values: many exact ties inside the windows
        x = (x.float() * 4).round().to(torch.bfloat16) / 4
    bn = make_bn(x, pyr, C, rng)
    lz = LazyDesc(x, pyr, C, bn=bn)
    OH, OW = (H + 1) // 2, (W + 1) // 2
    y0 = torch.empty(B * OH * OW, C, dtype=TDT[dt], device=DEV)
    y1 = torch.empty_like(y0)
    taps = torch.full((B * OH * OW, C), 255, dtype=torch.uint8, device=DEV)
    L.call("edet_maxpool_fwd", DT[dt], lz.c, B, H, W, C, vp(y0), stream())
    L.call("edet_maxpool_fwd_taps", DT[dt], lz.c, B, H, W, C, vp(y1), vp(taps), stream())
    dy = g(rnd(rng, B * OH * OW, C), dt)
    base = g(rnd(rng, B * H * W, C), dt)
    dx0, dx1 = base.clone(), base.clone()
    L.call("edet_maxpool_bwd", DT[dt], lz.c, B, H, W, C, vp(dy), vp(dx0), acc, stream())
    L.call("edet_maxpool_bwd_taps", DT[dt], B, H, W, C, vp(taps), vp(dy), vp(dx1), acc, stream())
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert int(taps.max()) <= 8
    assert torch.equal(dx0, dx1)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("B,H,W", [(2, 8, 8), (4, 136, 136)])  # the second exceeds the forward's 2048-block grid
def test_bifpn_fuse(dt, B, H, W):
    rng = np.random.default_rng(11)
    C = 64
    ins = []
    specs = [((H, W), L.MODE_SAME), ((H // 2, W // 2), L.MODE_UPSAMPLE), ((H * 2, W * 2), L.MODE_MAXPOOL)]
    descs = []
    fi = (L.FuseInput * 3)()
    dxs = []
    for i, ((h, w), mode) in enumerate(specs):
        pyr = Pyr(B, [(h, w)])
        x = pyr_data(rng, pyr, C, dt)
        bn = make_bn(x, pyr, C, rng) if i != 1 else None
        d = LazyDesc(x, pyr, C, bn=bn)
        descs.append((d, h, w, mode))
        fi[i].v, fi[i].H, fi[i].W, fi[i].mode = d.c, h, w, mode
        dx = g(torch.full((pyr.rows, C), 0.5 if i == 0 else 0.0), dt)
        dxs.append(dx)
        fi[i].dx, fi[i].accumulate = dx.data_ptr(), 1 if i == 0 else 0
    wv = g(torch.tensor([1.0, 0.7, 1.3]))
    out = torch.empty(B * H * W, C, dtype=TDT[dt], device=DEV)
    L.call("edet_bifpn_fuse_fwd", DT[dt], 3, fi, vp(wv), B, H, W, C, vp(out), stream())
    vs = [d.cpu_value().requires_grad_(True) for d, *_ in descs]
    wr = wv.double().cpu().requires_grad_(True)
    den = wr.sum() + 1e-4
    r0 = vs[0]
    up = vs[1].view(B, H // 2, W // 2, C)[:, torch.arange(H) // 2][:, :, torch.arange(W) // 2].reshape(-1, C)
    r2 = maxpool_ref(vs[2], B, H * 2, W * 2, C)
    ref = r0 * wr[0] / den + up * wr[1] / den + r2 * wr[2] / den
    close(out, ref.detach(), dt)
    dout = g(rnd(rng, B * H * W, C), dt)
    (ref * dout.double().cpu()).sum().backward()
    dw = zeros(3)
    L.call("edet_bifpn_fuse_bwd", DT[dt], 3, fi, vp(wv), B, H, W, C, vp(out), vp(dout), vp(dw), stream())
    close(dxs[0], vs[0].grad + 0.5, dt)
    close(dxs[1], vs[1].grad, dt)
    if dt == "f32":
        close(dxs[2], vs[2].grad, dt)
    close(dw, wr.grad, dt, scale=30)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("pool_in", [(16, 14), (15, 13)])
def test_bifpn_fuse_stored_pool_taps(dt, pool_in):
    """The forward's recorded max-pool window taps (edet_fuse_input.pool_arg) give the same
    backward as re-evaluating the windows: input gradients bit-exact, the weight gradient up to
    the order of its cross-block fp32 atomics."""
    rng = np.random.default_rng(12)
    B, C, H, W = 2, 64, 8, 7
    specs = [((H, W), L.MODE_SAME), (pool_in, L.MODE_MAXPOOL)]
    assert all(((h + 1) // 2, (w + 1) // 2) == (H, W) for (h, w), m in specs if m == L.MODE_MAXPOOL)
    descs = []
    for i, ((h, w), mode) in enumerate(specs):
        pyr = Pyr(B, [(h, w)])
        x = pyr_data(rng, pyr, C, dt, scale=2.0)
        descs.append((LazyDesc(x, pyr, C, bn=make_bn(x, pyr, C, rng), act=1), pyr, h, w, mode))
    wv = g(torch.tensor([0.9, 1.2]))
    dout = g(rnd(rng, B * H * W, C), dt)
    res = []
    for stored in (False, True):
        taps = torch.full((B * H * W, C), 77, dtype=torch.uint8, device=DEV)
        fi = (L.FuseInput * 2)()
        dxs = []
        for i, (d, pyr, h, w, mode) in enumerate(descs):
            fi[i].v, fi[i].H, fi[i].W, fi[i].mode = d.c, h, w, mode
            dx = torch.zeros(pyr.rows, C, dtype=TDT[dt], device=DEV)
            dxs.append(dx)
            fi[i].dx, fi[i].accumulate = dx.data_ptr(), 0
            fi[i].pool_arg = taps.data_ptr() if (stored and mode == L.MODE_MAXPOOL) else None
        out = torch.empty(B * H * W, C, dtype=TDT[dt], device=DEV)
        L.call("edet_bifpn_fuse_fwd", DT[dt], 2, fi, vp(wv), B, H, W, C, vp(out), stream())
        dw = zeros(2)
        L.call("edet_bifpn_fuse_bwd", DT[dt], 2, fi, vp(wv), B, H, W, C, vp(out), vp(dout), vp(dw), stream())
        torch.cuda.synchronize()
        if stored:
            assert int(taps.max()) <= 8  # every output recorded a tap of its 3x3 window
        res.append((out.clone(), [d.clone() for d in dxs], dw.clone()))
    (o0, d0, w0), (o1, d1, w1) = res
    assert torch.equal(o0, o1)
    for a, b in zip(d0, d1):
        assert torch.equal(a, b)
    assert torch.allclose(w0, w1, rtol=1e-5, atol=1e-6)


_FMODE = {"S": L.MODE_SAME, "U": L.MODE_UPSAMPLE, "P": L.MODE_MAXPOOL}


def _fuse_node(rng, B, C, H, W, modes, act_in, pool_odd):
    descs = []
    for m in modes:
        h, w = {"S": (H, W), "U": (H // 2, W // 2),
                "P": (2 * H - 1, 2 * W - 1) if pool_odd else (2 * H, 2 * W)}[m]
        pyr = Pyr(B, [(h, w)])
        x = pyr_data(rng, pyr, C, "bf16", scale=2.0)
        descs.append((LazyDesc(x, pyr, C, bn=make_bn(x, pyr, C, rng), act=act_in), pyr, h, w, _FMODE[m]))
    return descs


def _fuse_inputs(descs, taps, prefill, C=64):
    fi = (L.FuseInput * len(descs))()
    dxs = []
    for i, (d, pyr, h, w, mode) in enumerate(descs):
        fi[i].v, fi[i].H, fi[i].W, fi[i].mode = d.c, h, w, mode
        dx = torch.full((pyr.rows, C), 0.5 if prefill[i] else 0.0, dtype=torch.bfloat16, device=DEV)
        dxs.append(dx)
        fi[i].dx, fi[i].accumulate = dx.data_ptr(), int(prefill[i])
        fi[i].pool_arg = taps.data_ptr() if mode == L.MODE_MAXPOOL else None
    return fi, dxs


@pytest.mark.parametrize("modes,H,W,act_in,out_act,pool_odd", [
    ("SU", 8, 8, 1, 1, False), ("SU", 64, 64, 0, 1, False), ("SSP", 8, 6, 1, 1, False),
    ("SSP", 7, 5, 1, 0, True), ("SP", 16, 16, 1, 1, False), ("SP", 5, 3, 0, 1, True),
    ("SSU", 32, 32, 1, 1, False), ("SSU", 4, 6, 1, 0, False), ("SS", 9, 7, 1, 1, False),
    ("SS", 33, 31, 0, 0, False)])
def test_bifpn_fuse_bwd_dv(modes, H, W, act_in, out_act, pool_odd):
    """The one-pass fusion backward from d(value) (edet_bifpn_fuse_bwd_dv + edet_bifpn_fuse_fold,
    ABI 10) against the two-pass one it replaces (d(raw) = dv * act'(F) formed here, then
    edet_bifpn_fuse_bwd, whose own parity is test_bifpn_fuse) on the same forward and the same
    recorded pool taps, and the weight gradient against the fp64 autograd of bifpn.py:59-66.
    Covers every BiFPN input-mode combination, odd extents (partial output quads), odd max-pool
    inputs, accumulation into an existing dx, and both output activations."""
    rng = np.random.default_rng(H * 31 + W + len(modes))
    B, C = 2, 64
    n = len(modes)
    descs = _fuse_node(rng, B, C, H, W, modes, act_in, pool_odd)
    wv = g(torch.tensor([1.0, 0.7, 1.3][:n]))
    taps = torch.full((B * H * W, C), 77, dtype=torch.uint8, device=DEV)
    prefill = [i == 0 for i in range(n)]
    fi, _ = _fuse_inputs(descs, taps, prefill)
    out = torch.empty(B * H * W, C, dtype=torch.bfloat16, device=DEV)
    L.call("edet_bifpn_fuse_fwd", L.BF16, n, fi, vp(wv), B, H, W, C, vp(out), stream())
    dv = g(rnd(rng, B * H * W, C), "bf16")
    F = out.float()
    dF = (dv.float() * (torch.sigmoid(F) * (1 + F * (1 - torch.sigmoid(F)))) if out_act else dv.float())
    # two-pass reference path
    fa, dxa = _fuse_inputs(descs, taps, prefill)
    dwa = zeros(n)
    L.call("edet_bifpn_fuse_bwd", L.BF16, n, fa, vp(wv), B, H, W, C, vp(out), vp(dF.to(torch.bfloat16)),
           vp(dwa), stream())
    # one pass
    fb, dxb = _fuse_inputs(descs, taps, prefill)
    nparts = ctypes.c_int(-1)
    L.call("edet_bifpn_fuse_bwd_dv_parts", L.BF16, n, fb, B, H, W, C, ctypes.byref(nparts))
    assert nparts.value > 0
    part = torch.full((nparts.value * 4,), float("nan"), dtype=torch.float32, device=DEV)
    L.call("edet_bifpn_fuse_bwd_dv", L.BF16, n, fb, vp(wv), B, H, W, C, vp(out), vp(dv), out_act, vp(part),
           nparts.value, stream())
    dwb = g(torch.full((n,), 0.25))
    item = (L.FuseFold * 1)()
    item[0].part, item[0].w, item[0].dw, item[0].nparts, item[0].n_in = part.data_ptr(), wv.data_ptr(), \
        dwb.data_ptr(), nparts.value, n
    L.call("edet_bifpn_fuse_fold", 1, item, stream())
    torch.cuda.synchronize()
    for a, b in zip(dxa, dxb):
        close(b, a, "bf16", rtol=2e-2, atol=2e-2)
    # weight gradient: fp64 autograd over the stored inputs with the kernel's own pool taps
    wr = wv.double().cpu().requires_grad_(True)
    den = wr.sum() + 1e-4
    vs = [d.cpu_value() for d, *_ in descs]
    Fr = 0
    tcpu = taps.long().cpu()
    for i, (d, pyr, h, w, mode) in enumerate(descs):
        v = vs[i].view(B, h, w, C)
        if mode == L.MODE_SAME:
            r = v
        elif mode == L.MODE_UPSAMPLE:
            r = v[:, torch.arange(H) // 2][:, :, torch.arange(W) // 2]
        else:
            pt, pl = max((H - 1) * 2 + 3 - h, 0) // 2, max((W - 1) * 2 + 3 - w, 0) // 2
            t = tcpu.view(B, H, W, C)
            iy = (torch.arange(H).view(1, H, 1, 1) * 2 - pt + t // 3).clamp(0, h - 1)
            ix = (torch.arange(W).view(1, 1, W, 1) * 2 - pl + t % 3).clamp(0, w - 1)
            bi = torch.arange(B).view(B, 1, 1, 1).expand(B, H, W, C)
            ci = torch.arange(C).view(1, 1, 1, C).expand(B, H, W, C)
            r = v[bi, iy, ix, ci]
        Fr = Fr + r.reshape(-1, C) * wr[i] / den
    Fd = Fr.detach()
    dFr = dv.double().cpu() * ((torch.sigmoid(Fd) * (1 + Fd * (1 - torch.sigmoid(Fd)))) if out_act else 1.0)
    (Fr * dFr).sum().backward()
    close(dwb - 0.25, wr.grad, "bf16", scale=30)
    close(dwb - 0.25, dwa, "bf16", scale=30)


def test_bifpn_fuse_fold_many_items():
    """edet_bifpn_fuse_fold over more items than one launch takes (EDET_FUSE_FOLD_MAX): every
    node's records summed in fp64 and divided by its (sum w + 1e-4), added into dw."""
    rng = np.random.default_rng(5)
    n_items = L.FUSE_FOLD_MAX + 9
    arr = (L.FuseFold * n_items)()
    keep, expect = [], []
    for k in range(n_items):
        n_in = 2 + k % 2
        nparts = int(rng.integers(1, 700))
        p = rng.standard_normal((nparts, 4)).astype(np.float32)
        w = rng.uniform(0.1, 2.0, n_in).astype(np.float32)
        pt, wt, dw = g(torch.tensor(p.reshape(-1))), g(torch.tensor(w)), g(torch.full((n_in,), 1.0))
        keep += [pt, wt, dw]
        arr[k].part, arr[k].w, arr[k].dw, arr[k].nparts, arr[k].n_in = pt.data_ptr(), wt.data_ptr(), \
            dw.data_ptr(), nparts, n_in
        den = float(np.float32(w.sum(dtype=np.float32) + np.float32(1e-4)))
        expect.append((dw, 1.0 + p[:, :n_in].astype(np.float64).sum(0) / den))
    L.call("edet_bifpn_fuse_fold", n_items, arr, stream())
    torch.cuda.synchronize()
    for dw, e in expect:
        np.testing.assert_allclose(dw.cpu().numpy(), e, rtol=1e-5, atol=1e-5)


def test_bifpn_fuse_bwd_dv_coverage():
    """edet_bifpn_fuse_bwd_dv_parts reports 0 (caller falls back) for fp32, a max-pooled input
    without recorded taps and an upsample that is not exactly x2; the launch refuses them."""
    B, C, H, W = 2, 64, 8, 8
    x = torch.zeros(B * 16 * 16, C, dtype=torch.bfloat16, device=DEV)
    fi = (L.FuseInput * 2)()
    for i, (h, w, mode) in enumerate([(H, W, L.MODE_SAME), (2 * H, 2 * W, L.MODE_MAXPOOL)]):
        fi[i].v.x, fi[i].v.ld, fi[i].H, fi[i].W, fi[i].mode = x.data_ptr(), C, h, w, mode
        fi[i].dx = x.data_ptr()
    nparts = ctypes.c_int(-1)
    L.call("edet_bifpn_fuse_bwd_dv_parts", L.BF16, 2, fi, B, H, W, C, ctypes.byref(nparts))
    assert nparts.value == 0  # no pool taps
    fi[1].pool_arg = x.data_ptr()
    L.call("edet_bifpn_fuse_bwd_dv_parts", L.BF16, 2, fi, B, H, W, C, ctypes.byref(nparts))
    assert nparts.value > 0
    L.call("edet_bifpn_fuse_bwd_dv_parts", L.F32, 2, fi, B, H, W, C, ctypes.byref(nparts))
    assert nparts.value == 0
    fi[1].H, fi[1].W, fi[1].mode, fi[1].pool_arg = 3, 3, L.MODE_UPSAMPLE, None  # 3 -> 8 is not x2
    L.call("edet_bifpn_fuse_bwd_dv_parts", L.BF16, 2, fi, B, H, W, C, ctypes.byref(nparts))
    assert nparts.value == 0
    wv = g(torch.tensor([1.0, 1.0]))
    part = torch.zeros(64, dtype=torch.float32, device=DEV)
    with pytest.raises(L.EdetError, match="not covered"):
        L.call("edet_bifpn_fuse_bwd_dv", L.BF16, 2, fi, vp(wv), B, H, W, C, vp(x), vp(x), 1, vp(part), 16,
               stream())


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("kind", ["gate", "pyramid", "wide", "wide_pyramid"])
def test_lazy_materialize(dt, kind):
    """wide: C = 1152 over 16x16 images (the channel-sliced plan, C >= 1024 and M <= 16384)."""
    rng = np.random.default_rng(31)
    C = 1152 if kind.startswith("wide") else 48
    pyr = {"gate": Pyr(3, [(5, 7)]), "pyramid": Pyr(2, [(4, 4), (2, 2)]), "wide": Pyr(32, [(16, 16)]),
           "wide_pyramid": Pyr(2, [(9, 7), (3, 4)])}[kind]
    if kind == "wide_pyramid":
        kind = "pyramid"
    x = g(rnd(rng, pyr.rows, C), dt)
    gate = g(torch.rand(pyr.batch, C), "f32") if kind in ("gate", "wide") else None
    lz = LazyDesc(x, pyr, C, bn=make_bn(x, pyr, C, rng), act=1, gate=gate)
    out = torch.full((pyr.rows, C), float("nan"), dtype=TDT[dt], device=DEV)
    L.call("edet_lazy_materialize", DT[dt], lz.c, pyr.c, C, vp(out), stream())
    ref = lz.cpu_value()
    for s in range(pyr.nseg):
        sl = pyr.seg_slice(s)
        close(out[sl], ref[sl], dt)


@pytest.mark.parametrize("dt", DTS)
def test_residual(dt):
    rng = np.random.default_rng(3)
    pyr = Pyr(2, [(8, 8), (4, 4)])
    C = 64
    x = pyr_data(rng, pyr, C, dt)
    r = pyr_data(rng, pyr, C, dt)
    lx = LazyDesc(x, pyr, C, bn=make_bn(x, pyr, C, rng), act=1)
    lr = LazyDesc(r, pyr, C, bn=make_bn(r, pyr, C, rng))
    sc = g(torch.tensor([[1.25, 0.0], [0.0, 1.25]]))
    out = torch.empty(pyr.rows, C, dtype=TDT[dt], device=DEV)
    L.call("edet_residual_fwd", DT[dt], lx.c, lr.c, pyr.c, C, vp(sc), vp(out), stream())
    vx, vr = lx.cpu_value(), lr.cpu_value()
    for s in range(2):
        sl = pyr.seg_slice(s)
        m = sc[s].double().cpu().repeat_interleave(pyr.sizes[s][0] * pyr.sizes[s][1])[:, None]
        close(out[sl], vx[sl] * m + vr[sl], dt)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("shape", [(2, 21, 18, 32), (3, 34, 40, 48), (2, 64, 64, 32),
                                   # one output row per weight-gradient strip (OW >= 129)
                                   (1, 8, 512, 32), (2, 7, 300, 32)])
def test_stem(dt, shape, workspace_mode):
    rng = np.random.default_rng(9)
    B, H, W, Co = shape
    x = g(torch.rand(B, H, W, 3), dt)
    w = g(rnd(rng, 3, 3, 3, Co, scale=0.3), dt)
    OH, OW = (H + 1) // 2, (W + 1) // 2
    y = torch.empty(B * OH * OW, Co, dtype=TDT[dt], device=DEV)
    su, sq = stats_out(1, Co)[0]
    L.call("edet_stem_fwd", DT[dt], vp(x), B, H, W, vp(w), Co, vp(y), vp(su.raw), vp(sq.raw), stream())
    xc = x.double().cpu().permute(0, 3, 1, 2)
    ph, pw = max((OH - 1) * 2 + 3 - H, 0), max((OW - 1) * 2 + 3 - W, 0)
    xp = Fn.pad(xc, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
    wr = w.double().cpu().permute(3, 2, 0, 1).clone().requires_grad_(True)
    ref = Fn.conv2d(xp, wr, stride=2).permute(0, 2, 3, 1).reshape(-1, Co)
    close(y, ref.detach(), dt)
    close(su, ref.detach().sum(0), dt, scale=20)
    dy = g(rnd(rng, B * OH * OW, Co), dt)
    (ref * dy.double().cpu()).sum().backward()
    dw = zeros(3, 3, 3, Co)
    L.call("edet_stem_wgrad", DT[dt], vp(x), B, H, W, vp(dy), Co, vp(dw), stream())
    close(dw, wr.grad.permute(2, 3, 1, 0), dt, scale=20)


# ----------------------------------------------------------------- loss
@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("NC,ldc,sizes", [(5, 48, [(4, 4), (2, 2)]),
                                          # the D0 headline geometry: 81 classes, 729 logits in
                                          # rows of 736 (the NC >= 8 stepping path of k_loss)
                                          (81, 736, [(8, 8), (4, 4), (2, 2), (1, 1), (1, 1)]),
                                          (8, 72, [(6, 5), (3, 3)])])
def test_detection_loss(dt, NC, ldc, sizes):
    rng = np.random.default_rng(21 + NC)
    A = 9
    pyr = Pyr(2, sizes)
    ldb = 40
    cls = torch.zeros(pyr.rows, ldc)
    cls[:, : A * NC] = rnd(rng, pyr.rows, A * NC, scale=3.0)
    box = torch.zeros(pyr.rows, ldb)
    box[:, : A * 4] = rnd(rng, pyr.rows, A * 4, scale=0.2)
    cls_g, box_g = g(cls, dt), g(box, dt)
    ct = torch.tensor(rng.integers(0, NC, (pyr.rows, A)), dtype=torch.int32)
    bt = rnd(rng, pyr.rows, A, 4, scale=0.2)
    bt[rng.random((pyr.rows, A, 4)) < 0.5] = 0.0
    for s in range(pyr.nseg - 1):  # padding rows between the levels: never read
        pad = slice(pyr.row_off[s] + pyr.seg_rows(s), pyr.row_off[s + 1])
        ct[pad] = 0
        bt[pad] = 0.0
    mask = (ct > 0).to(torch.uint8)
    npos = zeros(1)
    mask_g = mask.to(DEV)
    for s in range(pyr.nseg):
        sl = pyr.seg_slice(s)
        L.call("edet_count_positives", vp(mask_g[sl]), pyr.seg_rows(s) * A, vp(npos), stream())
    loss = zeros(1)
    parts = zeros(10)
    ctg, btg = ct.to(DEV), bt.to(DEV)
    L.call("edet_detection_loss", DT[dt], vp(cls_g), ldc, vp(box_g), ldb, pyr.c, A, NC, vp(ctg), vp(btg), vp(npos),
           0.25, 1.5, 0.1, 50.0, 1.0, vp(cls_g), vp(box_g), vp(loss), vp(parts), stream())
    # reference (oracle formulas, fp64)
    from oracle.ref_model import RefEfficientDet
    npr = float(mask.sum()) + 1.0
    tot = 0.0
    xs = cls[:, : A * NC].double().requires_grad_(True)
    bs = box[:, : A * 4].double().requires_grad_(True)
    for s in range(pyr.nseg):
        sl = pyr.seg_slice(s)
        x = xs[sl].view(-1, A, NC)
        y = Fn.one_hot(ct[sl].long(), NC).double()
        p = torch.sigmoid(x)
        pt = y * p + (1 - y) * (1 - p)
        at = y * 0.25 + (1 - y) * 0.75
        ce = torch.clamp(x, min=0) - x * y + torch.log1p(torch.exp(-x.abs()))
        tot = tot + (at * (1 - pt) ** 1.5 * ce / npr).sum() / x.numel()
        t = bt[sl].double().view(-1, A * 4)
        e = bs[sl] - t
        hub = torch.where(e.abs() <= 0.1, 0.5 * e ** 2, 0.005 + 0.1 * (e.abs() - 0.1))
        tot = tot + 50.0 * (hub * (t != 0)).sum() / (4 * npr)
    tot.backward()
    close(npos, torch.tensor([npr - 1]), "f32")
    close(loss, tot.detach().reshape(1), "f32", rtol=1e-4 if dt == "f32" else 2e-2)
    for s in range(pyr.nseg):  # padding rows between levels are never touched
        sl = pyr.seg_slice(s)
        close(cls_g[sl, : A * NC], xs.grad[sl], dt, scale=1e-3)
        close(box_g[sl, : A * 4], bs.grad[sl], dt, scale=1e-1)
        if ldc > A * NC:
            assert float(cls_g[sl, A * NC:].abs().max()) == 0.0


# ----------------------------------------------------------------- optimizer
def _sched_lr(step, adj=0.08, init=0.008, warm=10, total=100):
    """CosineLrSchedule.__call__ (efficientnet/train.py:55-63)."""
    if step < warm:
        return init + step / warm * (adj - init)
    return 0.5 * adj * (1 + np.cos(np.pi * step / (total - warm)))


@pytest.mark.parametrize("steps,start,clip", [(1, 3, 10.0), (4, 8, 10.0), (3, 57, 10.0), (2, 20, 50.0)])
def test_optimizer_step(steps, start, clip):
    """L2 + clip_by_global_norm + SGD momentum + EMA over several consecutive steps, through
    the warm-up -> cosine switch (start 8, 4 steps) and deep in the cosine phase."""
    rng = np.random.default_rng(2 + start)
    n, n_l2 = 10000, 6000
    w = g(rnd(rng, n))
    v = g(rnd(rng, n) * 0.1)
    ema = g(rnd(rng, n))
    sc = L.Sched()
    sc.adjusted_lr, sc.warmup_init, sc.warmup_steps, sc.total_steps = 0.08, 0.008, 10, 100
    sc.momentum, sc.ema_decay, sc.clip_norm, sc.l2_weight = 0.9, 0.9998, clip, 4e-5
    scal = zeros(8)
    parts = torch.zeros(2 * L.OPT_NORM_BLOCKS, dtype=torch.float64, device=DEV)
    step = torch.tensor([start], dtype=torch.int32, device=DEV)
    W, V, E = (t.double().cpu() for t in (w, v, ema))
    wc = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    for i in range(steps):
        gr = g(rnd(rng, n) * 3)
        G0 = gr.double().cpu()
        W0 = W.clone()
        L.call("edet_opt_norm", vp(w), vp(gr), n, n_l2, sc, vp(scal), vp(parts), vp(step), stream())
        L.call("edet_opt_apply", vp(w), vp(gr), vp(v), vp(ema), n, n_l2, sc, vp(scal), vp(parts), L.BF16, vp(wc),
               vp(step), stream())
        gg = G0.clone()
        gg[:n_l2] += 4e-5 * W0[:n_l2]
        gn = gg.norm()
        lr = _sched_lr(start + i)
        gg *= clip / max(float(gn), clip)
        V = 0.9 * V - lr * gg
        W = W0 + V
        E = E - (1 - 0.9998) * (E - W)
        close(scal[3], gn, "f32", rtol=1e-5)
        close(scal[4], torch.tensor(lr), "f32", rtol=2e-6, atol=1e-9)
    close(w, W, "f32", rtol=1e-5, atol=1e-6)
    close(v, V, "f32", rtol=1e-5, atol=1e-6)
    close(ema, E, "f32", rtol=1e-5, atol=1e-6)
    close(wc, W, "bf16")
    assert int(step.item()) == start + steps


def test_optimizer_norm_is_bit_reproducible():
    """The clip factor depends on gnorm; data-parallel replicas apply it to the same
    all-reduced gradient and must get the same bits: repeated norm passes over one
    gradient give identical gnorm and identical updated weights, with clipping active."""
    rng = np.random.default_rng(5)
    n, n_l2 = 3_000_000, 2_000_000
    gr = g(rnd(rng, n) * 30)
    w0 = g(rnd(rng, n))
    sc = L.Sched()
    sc.fixed_lr, sc.momentum, sc.ema_decay, sc.clip_norm, sc.l2_weight = 0.01, 0.9, 0.9998, 1.0, 4e-5
    outs = []
    for _ in range(3):
        w, v, ema = w0.clone(), torch.zeros_like(w0), w0.clone()
        scal = zeros(8)
        parts = torch.zeros(2 * L.OPT_NORM_BLOCKS, dtype=torch.float64, device=DEV)
        step = torch.zeros(1, dtype=torch.int32, device=DEV)
        L.call("edet_opt_norm", vp(w), vp(gr), n, n_l2, sc, vp(scal), vp(parts), vp(step), stream())
        L.call("edet_opt_apply", vp(w), vp(gr), vp(v), vp(ema), n, n_l2, sc, vp(scal), vp(parts), L.F32, None,
               vp(step), stream())
        outs.append((scal.clone(), w))
    assert float(outs[0][0][3]) > 10 * sc.clip_norm  # clipping active
    for s, w in outs[1:]:
        assert torch.equal(s[3], outs[0][0][3]) and torch.equal(w, outs[0][1])


@pytest.mark.parametrize("bad", [float("nan"), float("inf")])
def test_optimizer_skips_nonfinite_step(bad):
    """SURVEY §5 failure detection: with sched.skip_nonfinite a step whose gradient norm is not
    finite leaves w, v, ema, the compute copy and the step counter unchanged and reports
    scalars[6] = 1; the next finite step applies normally (scalars[6] = 0).  Without the flag the
    update is applied as the reference does (the weights become non-finite)."""
    rng = np.random.default_rng(11)
    n, n_l2 = 5000, 3000
    sc = L.Sched()
    sc.fixed_lr, sc.momentum, sc.ema_decay, sc.clip_norm, sc.l2_weight = 0.01, 0.9, 0.9998, 10.0, 4e-5
    for flag in (1, 0):
        sc.skip_nonfinite = flag
        w, v, ema = g(rnd(rng, n)), g(rnd(rng, n) * 0.1), g(rnd(rng, n))
        wc = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        L.call("edet_cast_f32", L.BF16, vp(w), vp(wc), n, stream())
        w0, v0, e0, c0 = w.clone(), v.clone(), ema.clone(), wc.clone()
        scal = zeros(8)
        parts = torch.zeros(2 * L.OPT_NORM_BLOCKS, dtype=torch.float64, device=DEV)
        step = torch.tensor([7], dtype=torch.int32, device=DEV)
        gr = g(rnd(rng, n))
        gr[1234] = bad
        L.call("edet_opt_norm", vp(w), vp(gr), n, n_l2, sc, vp(scal), vp(parts), vp(step), stream())
        L.call("edet_opt_apply", vp(w), vp(gr), vp(v), vp(ema), n, n_l2, sc, vp(scal), vp(parts), L.BF16, vp(wc),
               vp(step), stream())
        torch.cuda.synchronize()
        assert not math.isfinite(float(scal[3]))
        if flag:
            assert float(scal[6]) == 1.0 and int(step.item()) == 7
            assert torch.equal(w, w0) and torch.equal(v, v0) and torch.equal(ema, e0) and torch.equal(wc, c0)
            gr = g(rnd(rng, n))  # a finite step afterwards is applied and clears the flag
            L.call("edet_opt_norm", vp(w), vp(gr), n, n_l2, sc, vp(scal), vp(parts), vp(step), stream())
            L.call("edet_opt_apply", vp(w), vp(gr), vp(v), vp(ema), n, n_l2, sc, vp(scal), vp(parts), L.BF16,
                   vp(wc), vp(step), stream())
            torch.cuda.synchronize()
            assert float(scal[6]) == 0.0 and int(step.item()) == 8 and not torch.equal(w, w0)
            assert bool(torch.isfinite(w).all())
        else:
            assert float(scal[6]) == 0.0 and int(step.item()) == 8
            assert not bool(torch.isfinite(w).all())


def test_bn_moving_update_and_inference_stats():
    rng = np.random.default_rng(4)
    n = 300
    su = (rnd(rng, n) * 50).double().to(DEV)  # fp64 statistics arena (values)
    sq = (torch.rand(n) * 500 + 2500).double().to(DEV)
    sur, sqr = rep64(su), rep64(sq)  # the replicated layout the kernels read (ABI 9)
    # the value split over the four replicas: the kernel must sum them
    sur[L.stat_idx(5, 2)] += 3.0
    sur[L.stat_idx(5, 0)] -= 3.0
    cnt = g(torch.full((n,), 100.0))
    mm, mv = g(rnd(rng, n)), g(torch.rand(n) + 0.5)
    MM, MV = mm.double().cpu(), mv.double().cpu()
    L.call("edet_bn_update_moving", n, vp(sur), vp(sqr), vp(cnt), 0.99, None, vp(mm), vp(mv), stream())
    mean = su.double().cpu() / 100
    var = sq.double().cpu() / 100 - mean ** 2
    close(mm, MM - (MM - mean) * 0.01, "f32", rtol=1e-5)
    close(mv, MV - (MV - var * 100 / 99) * 0.01, "f32", rtol=1e-5)
    s2, q2 = stats_out(1, n)[0]
    L.call("edet_bn_inference_stats", n, vp(mm), vp(mv), vp(cnt), vp(s2.raw), vp(q2.raw), stream())
    m2 = s2.v.double().cpu() / 100
    close(m2, mm, "f32", rtol=1e-6)
    close(q2.v.double().cpu() / 100 - m2 ** 2, mv, "f32", rtol=1e-3, atol=1e-4)
    # the optimizer's skip flag (scalars[6]) set: a skipped step leaves the moving statistics
    # alone, NaN batch sums included; flag clear: the update runs
    skip = g(torch.tensor([1.0]))
    sur[L.stat_idx(7, 1)] = float("nan")
    mm0, mv0 = mm.clone(), mv.clone()
    L.call("edet_bn_update_moving", n, vp(sur), vp(sqr), vp(cnt), 0.99, vp(skip), vp(mm), vp(mv), stream())
    torch.cuda.synchronize()
    assert torch.equal(mm, mm0) and torch.equal(mv, mv0)
    skip.zero_()
    L.call("edet_bn_update_moving", n, vp(sur), vp(sqr), vp(cnt), 0.99, vp(skip), vp(mm), vp(mv), stream())
    torch.cuda.synchronize()
    assert not torch.equal(mm, mm0) and math.isnan(float(mm[7]))


def test_dropmask():
    out = torch.empty(4000, device=DEV)
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    L.call("edet_dropmask", vp(out), 4000, 0.8, 7, vp(step), stream())
    o = out.cpu()
    vals = set(np.round(o.numpy(), 5).tolist())
    assert vals <= {0.0, 1.25}
    frac = float((o > 0).float().mean())
    assert 0.76 < frac < 0.84


@pytest.mark.parametrize("dt", DTS)
def test_transpose_cast(dt):
    rng = np.random.default_rng(8)
    shapes = [(729, 64), (24, 144), (1152, 192)]
    src = torch.zeros(sum(n * k for n, k in shapes) + 64)
    table, off, toff, outs = [], 0, 0, []
    for n, k in shapes:
        w = rnd(rng, n, k)
        src[off: off + n * k] = w.reshape(-1)
        ldn = (n + 7) // 8 * 8
        table.append([off, toff, n, k])
        outs.append((w, toff, ldn))
        off += n * k
        toff += k * ldn
    dst = torch.full((toff,), 7.0, dtype=TDT[dt], device=DEV)
    tab = torch.tensor(table, dtype=torch.int64, device=DEV)
    mt = max(((n + 31) // 32) * ((k + 31) // 32) for n, k in shapes)
    L.call("edet_transpose_cast", DT[dt], vp(g(src)), vp(dst), vp(tab), len(shapes), mt, stream())
    for w, o, ldn in outs:
        n, k = w.shape
        got = dst[o: o + k * ldn].view(k, ldn).float().cpu()
        close(got[:, :n], w.t(), dt)
        assert float(got[:, n:].abs().max() if ldn > n else 0) == 0.0


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("C,HW", [(48, 9 * 10), (144, 23 * 17),
                                  # round 5: C >= 480 over H*W <= 4096 takes one block per (image,
                                  # 64-channel slice) with plain stores; a partial last slice (520)
                                  (480, 16 * 16), (1152, 7 * 9), (520, 10 * 10), (672, 64 * 64)])
def test_gate_bn_reduce_equals_separate_passes(dt, C, HW):
    """edet_gate_bn_reduce + edet_se_bn_combine (one pass) == edet_gate_grad + se_bwd's dsq +
    edet_lazy_bwd_reduce (two passes) on an SE-gated swish(BN) value."""
    rng = np.random.default_rng(C + HW)
    B = 3
    pyr = Pyr(B, [(HW, 1)])
    x = pyr_data(rng, pyr, C, dt, scale=2.0)
    bn = make_bn(x, pyr, C, rng)
    gt = g(torch.rand(B, C) + 0.5, "f32")
    lz = LazyDesc(x, pyr, C, bn=bn, act=1, gate=gt)
    dv = pyr_data(rng, pyr, C, dt)
    dsq = g(rnd(rng, B, C) * 0.1, "f32")
    # two-pass reference path
    dg = zeros64(B, C)
    L.call("edet_gate_grad", DT[dt], lz.c, B, HW, C, vp(dv), vp(dg), stream())
    acc_t, acc = bngrad64(1, C)
    L.call("edet_lazy_bwd_reduce", DT[dt], lz.c, pyr.c, C, vp(dv), None, vp(dsq), acc, stream())
    # fused
    s5 = zeros64(5, B, C)
    L.call("edet_gate_bn_reduce", DT[dt], lz.c, B, HW, C, vp(dv), vp(s5), stream())
    acc2_t, acc2 = bngrad64(1, C)
    L.call("edet_se_bn_combine", B, C, vp(gt), vp(dsq), vp(s5), acc2, stream())
    torch.cuda.synchronize()
    # fp32 partial sums over the image in another order than edet_gate_grad's: the bar grows
    # with the terms summed (the sliced form sums 32 row groups of H*W / 32 rows)
    torch.testing.assert_close(s5[0], dg, rtol=1e-5, atol=1e-6 * max(1.0, HW / 64))
    scale = float(acc_t.abs().max())
    torch.testing.assert_close(acc2_t.v, acc_t.v, rtol=1e-4, atol=1e-5 * scale)
    # edet_se_bwd_bn == edet_se_bwd then edet_se_bn_combine (its dsq): the SE gradients bit for
    # bit, the fp64 BN sums to fp64 rounding (the combine kernel adds the images as a tree)
    R = 8
    sq = g(torch.rand(B, C).double(), "f32").double()
    z1 = g(rnd(rng, B, R))
    w1, w2 = g(rnd(rng, R, C, scale=0.2)), g(rnd(rng, C, R, scale=0.3))
    outs = []
    for fused in (False, True):
        dws = [zeros(R, C), zeros(R), zeros(C, R), zeros(C)]
        dsq2, dz1 = zeros(B, C), zeros(B, R)
        a_t, a = bngrad64(1, C)
        args = (B, C, R, HW, vp(sq), vp(z1), vp(gt), vp(s5[0]), vp(w1), vp(w2), *(vp(t) for t in dws), vp(dsq2), vp(dz1))
        if fused:
            L.call("edet_se_bwd_bn", *args, vp(s5), a, stream())
        else:
            L.call("edet_se_bwd", *args, stream())
            L.call("edet_se_bn_combine", B, C, vp(gt), vp(dsq2), vp(s5), a, stream())
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in dws] + [dsq2.cpu(), a_t.v.cpu()])
    for u, v in zip(outs[0][:-1], outs[1][:-1]):
        assert torch.equal(u, v)
    torch.testing.assert_close(outs[1][-1], outs[0][-1], rtol=1e-12, atol=1e-12 * float(outs[0][-1].abs().max()))
