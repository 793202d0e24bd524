"""Isolated timing of edet_conv1x1_fwd / dgrad / wgrad variants at one shape.

  python scripts/gemm_probe.py M K N
Prints us per launch for: plain fwd, fwd+stats, lazy bn fwd, lazy bn+swish fwd, lazy bn+swish+gate fwd,
dgrad, wgrad (plain and lazy).  Timing: 20 back-to-back launches between HIP events.
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tf2mv_amd import _lib as L  # noqa: E402
from tf2mv_amd.runtime import Pyr, ensure_workspace, stream, vp  # noqa: E402
from gpu_util import LazyDesc, make_bn, stat_out, stats_out, zeros64  # noqa: E402


KERN = {}


def timeit(fn, reps=20):
    if os.environ.get("ONLY"):
        reps = 5
    L.launched_kernels()
    fn()
    KERN["last"] = ",".join(sorted(set(k.split("<")[0].replace("(", "") for k in L.launched_kernels())))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    only = os.environ.get("ONLY", "")  # run just one variant (for rocprofv3 --pmc passes)
    shapes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or [(8192, 1152, 320)]
    rng = np.random.default_rng(0)
    if os.environ.get("NO_WS", "0") != "1":
        ensure_workspace(torch.device("cuda"))  # as the model runs: split partials, not atomics
    for (M, K, N) in shapes:
        # images of hw = 256 rows (16x16) as in the MBConv stage 5/6 tensors
        hw = 256 if M % 256 == 0 else M
        pyr = Pyr(M // hw, [(16, hw // 16)] if hw % 16 == 0 else [(1, hw)])
        x = torch.randn(pyr.rows, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
        wt = w.t().contiguous()
        b = torch.randn(N, device="cuda")
        y = torch.empty(pyr.rows, N, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(pyr.rows, N, device="cuda").to(torch.bfloat16)
        dx = torch.empty(pyr.rows, K, device="cuda", dtype=torch.bfloat16)
        dw = torch.zeros(N, K, device="cuda")
        db = torch.zeros(N, device="cuda")
        bn = make_bn(x, pyr, K, rng)
        gate = torch.rand(pyr.batch, K, device="cuda")
        plain = LazyDesc(x, pyr, K)
        lz_b = LazyDesc(x, pyr, K, bn=bn, act=0)
        lz_bs = LazyDesc(x, pyr, K, bn=bn, act=1)
        lz_bsg = LazyDesc(x, pyr, K, bn=bn, act=1, gate=gate)
        st = stats_out(1, N)
        so = stat_out(st)
        s = stream()
        es = 2
        algo = (M * (K + N) + K * N) * es
        res, kern = {}, {}
        if (not only or only == "fwd plain"):
            res["fwd plain"] = timeit(lambda: L.call("edet_conv1x1_fwd", L.BF16, plain.c, pyr.c, K, vp(w), N, vp(b), vp(y), N, 0, None, s))
            kern["fwd plain"] = KERN["last"]
        if (not only or only == "fwd +stats"):
            res["fwd +stats"] = timeit(lambda: L.call("edet_conv1x1_fwd", L.BF16, plain.c, pyr.c, K, vp(w), N, vp(b), vp(y), N, 0, so, s))
            kern["fwd +stats"] = KERN["last"]
        if (not only or only == "fwd bn"):
            res["fwd bn"] = timeit(lambda: L.call("edet_conv1x1_fwd", L.BF16, lz_b.c, pyr.c, K, vp(w), N, vp(b), vp(y), N, 0, so, s))
            kern["fwd bn"] = KERN["last"]
        if (not only or only == "fwd bn -stats"):
            res["fwd bn -stats"] = timeit(lambda: L.call("edet_conv1x1_fwd", L.BF16, lz_b.c, pyr.c, K, vp(w), N, vp(b), vp(y), N, 0, None, s))
            kern["fwd bn -stats"] = KERN["last"]
        if (not only or only == "fwd bn+sw"):
            res["fwd bn+sw"] = timeit(lambda: L.call("edet_conv1x1_fwd", L.BF16, lz_bs.c, pyr.c, K, vp(w), N, vp(b), vp(y), N, 0, so, s))
            kern["fwd bn+sw"] = KERN["last"]
        if (not only or only == "fwd bn+sw+g"):
            res["fwd bn+sw+g"] = timeit(lambda: L.call("edet_conv1x1_fwd", L.BF16, lz_bsg.c, pyr.c, K, vp(w), N, vp(b), vp(y), N, 0, so, s))
            kern["fwd bn+sw+g"] = KERN["last"]
        if (not only or only == "dgrad") and K % 8 == 0 and N % 8 == 0:
            res["dgrad"] = timeit(lambda: L.call("edet_conv1x1_dgrad", L.BF16, vp(dy), N, pyr.c, N, vp(wt), K, vp(dx), K, 0, s))
            kern["dgrad"] = KERN["last"]
        if (not only or only == "wgrad plain") and N % 8 == 0:
            res["wgrad plain"] = timeit(lambda: L.call("edet_conv1x1_wgrad", L.BF16, plain.c, pyr.c, K, vp(dy), N, N, vp(dw), vp(db), s))
            kern["wgrad plain"] = KERN["last"]
        if (not only or only == "wgrad bn+sw+g") and N % 8 == 0:
            res["wgrad bn+sw+g"] = timeit(lambda: L.call("edet_conv1x1_wgrad", L.BF16, lz_bsg.c, pyr.c, K, vp(dy), N, N, vp(dw), vp(db), s))
            kern["wgrad bn+sw+g"] = KERN["last"]
        print(f"M={M} K={K} N={N}  algorithmic {algo / 1e6:.1f} MB")
        for k, us in res.items():
            print(f"  {k:14s} {us:8.1f} us  {algo / (us * 1e3):8.1f} GB/s  {kern.get(k, '')}")


if __name__ == "__main__":
    main()
