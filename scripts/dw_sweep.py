"""Depthwise forward timing over the D0 b32 shapes, one line per shape (library from EDET_LIB).

    python scripts/dw_sweep.py [fwd|dgrad|wgrad]"""
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

SHAPES = [(32, 256, 256, 32, 3, 1), (32, 256, 256, 96, 3, 2), (32, 128, 128, 144, 3, 1), (32, 128, 128, 144, 5, 2),
          (32, 64, 64, 240, 5, 1), (32, 64, 64, 240, 3, 2), (32, 32, 32, 480, 3, 1), (32, 32, 32, 480, 5, 1),
          (32, 32, 32, 672, 5, 1), (32, 32, 32, 672, 5, 2), (32, 16, 16, 1152, 5, 1), (32, 16, 16, 1152, 3, 1),
          (32, 0, 0, 64, 3, 1), (32, 64, 64, 64, 3, 1)]  # H = 0: the D0 P3-P7 pyramid
D0_PYR = [(64, 64), (32, 32), (16, 16), (8, 8), (4, 4)]


def timeit(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "fwd"
    rng = np.random.default_rng(0)
    s = stream()
    tot = 0.0
    for B, H, W, C, k, st in SHAPES:
        pin = Pyr(B, D0_PYR if H == 0 else [(H, W)])
        pout = pin.strided(st)
        x = torch.randn(pin.rows, C, device="cuda").to(torch.bfloat16)
        lz = LazyDesc(x, pin, C, bn=make_bn(x, pin, C, rng), act=1)
        w = torch.randn(k * k, C, device="cuda").to(torch.bfloat16)
        y = torch.empty(pout.rows, C, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(pout.rows, C, device="cuda").to(torch.bfloat16)
        dx = torch.empty(pin.rows, C, device="cuda", dtype=torch.bfloat16)
        dw = torch.zeros(k * k, C, device="cuda")
        so = stat_out(stats_out(pin.nseg, C))
        if which == "fwd":
            f = lambda: L.call("edet_dwconv_fwd", L.BF16, lz.c, pin.c, C, k, st, vp(w), vp(y), pout.c, so, s)
        elif which == "dgrad":
            f = lambda: L.call("edet_dwconv_dgrad", L.BF16, vp(dy), pout.c, C, k, st, vp(w), vp(dx), pin.c, 0, s)
        else:
            f = lambda: L.call("edet_dwconv_wgrad", L.BF16, lz.c, pin.c, C, k, st, vp(dy), pout.c, vp(dw), s)
        us = timeit(f)
        tot += us
        byt = (pin.rows + pout.rows) * C * 2
        print(f"{which} B={B} H={H} C={C} k={k} s={st}: {us:7.1f} us {byt / (us * 1e3):7.1f} GB/s", flush=True)
        del x, y, dy, dx
    print(f"{which} total {tot:.1f} us")


if __name__ == "__main__":
    main()
