"""Timing of statistics-producing launches (GEMM fwd +stats, depthwise fwd +stats) -- run once
with the production library and once with EDET_LIB pointing at an experiment build."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
from tf2mv_amd import _lib as L
from tf2mv_amd.runtime import Pyr, stream, vp
from gpu_util import LazyDesc, make_bn, stat_out

def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps

big = lambda n: torch.zeros(n + 9 * 4096, dtype=torch.float64, device="cuda")
rng = np.random.default_rng(0)
s = stream()
for M, K, N in [(32768, 672, 112), (32768, 480, 80), (8192, 1152, 192), (32768, 112, 672), (131072, 40, 240)]:
    pyr = Pyr(M // 1024, [(32, 32)])
    x = torch.randn(pyr.rows, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    y = torch.empty(pyr.rows, N, device="cuda", dtype=torch.bfloat16)
    so = stat_out([(big(N), big(N))])
    lz = LazyDesc(x, pyr, K)
    t0 = timeit(lambda: L.call("edet_conv1x1_fwd", L.BF16, lz.c, pyr.c, K, vp(w), N, None, vp(y), N, 0, None, s))
    t1 = timeit(lambda: L.call("edet_conv1x1_fwd", L.BF16, lz.c, pyr.c, K, vp(w), N, None, vp(y), N, 0, so, s))
    print(f"gemm M={M} K={K} N={N}: plain {t0:.1f} us, +stats {t1:.1f} us", flush=True)
for B, H, C, k, st in [(32, 32, 672, 5, 1), (32, 64, 240, 5, 1), (32, 16, 1152, 5, 1), (32, 128, 144, 3, 1)]:
    pin = Pyr(B, [(H, H)]); pout = pin.strided(st)
    x = torch.randn(pin.rows, C, device="cuda").to(torch.bfloat16)
    lz = LazyDesc(x, pin, C, bn=make_bn(x, pin, C, rng), act=1)
    w = torch.randn(k * k, C, device="cuda").to(torch.bfloat16)
    y = torch.empty(pout.rows, C, device="cuda", dtype=torch.bfloat16)
    so = stat_out([(big(C), big(C))])
    t0 = timeit(lambda: L.call("edet_dwconv_fwd", L.BF16, lz.c, pin.c, C, k, st, vp(w), vp(y), pout.c, None, s))
    t1 = timeit(lambda: L.call("edet_dwconv_fwd", L.BF16, lz.c, pin.c, C, k, st, vp(w), vp(y), pout.c, so, s))
    print(f"dw B={B} H={H} C={C} k={k}: plain {t0:.1f} us, +stats {t1:.1f} us", flush=True)
