"""Isolated timing of the depthwise entry points at one shape (for A/B and rocprofv3 --pmc).

  python scripts/dw_probe.py B H W C k s
ONLY=fwd|dgrad|wgrad restricts to one entry point (5 launches) for counter passes.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tf2mv_amd import _lib as L  # noqa: E402
from tf2mv_amd.runtime import Pyr, stream, vp  # noqa: E402
from gpu_util import LazyDesc, make_bn, stat_out, stats_out, zeros64  # noqa: E402


def timeit(fn, reps):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    B, H, W, C, k, st = (int(v) for v in sys.argv[1:7])
    only = os.environ.get("ONLY", "")
    reps = 5 if only else 20
    rng = np.random.default_rng(0)
    pin = Pyr(B, [(H, W)])
    pout = pin.strided(st)
    x = torch.randn(pin.rows, C, device="cuda").to(torch.bfloat16)
    lz = LazyDesc(x, pin, C, bn=make_bn(x, pin, C, rng), act=1)
    w = torch.randn(k * k, C, device="cuda").to(torch.bfloat16)
    y = torch.empty(pout.rows, C, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(pout.rows, C, device="cuda").to(torch.bfloat16)
    dx = torch.empty(pin.rows, C, device="cuda", dtype=torch.bfloat16)
    dw = torch.zeros(k * k, C, device="cuda")
    so = stat_out(stats_out(1, C))
    s = stream()
    es = 2
    byt = (pin.rows + pout.rows) * C * es
    res = {}
    if not only or only == "fwd":
        res["fwd"] = timeit(lambda: L.call("edet_dwconv_fwd", L.BF16, lz.c, pin.c, C, k, st, vp(w), vp(y), pout.c, so, s), reps)
    if not only or only == "dgrad":
        res["dgrad"] = timeit(lambda: L.call("edet_dwconv_dgrad", L.BF16, vp(dy), pout.c, C, k, st, vp(w), vp(dx), pin.c, 0, s), reps)
    if not only or only == "wgrad":
        res["wgrad"] = timeit(lambda: L.call("edet_dwconv_wgrad", L.BF16, lz.c, pin.c, C, k, st, vp(dy), pout.c, vp(dw), s), reps)
    print(f"B={B} H={H} W={W} C={C} k={k} s={st}  algorithmic {byt / 1e6:.1f} MB")
    for n, us in res.items():
        print(f"  {n:6s} {us:8.1f} us  {byt / (us * 1e3):8.1f} GB/s")


if __name__ == "__main__":
    main()
