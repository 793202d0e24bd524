"""Depthwise backward A/B over the D0 b32 stride-1 shapes (development; EDET_DEV library).

For each shape: the separate path (edet_dwconv_dgrad + edet_dwconv_wgrad + the BN-backward
reduce of the input) against the fused edet_dwconv_bwd (with the fold), the latter at several
block targets (development slot 16), and the forward at several block targets (slot 6).

    EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so python tools/dw_bwd_probe.py [targets]
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
from gpu_util import LazyDesc, bngrad64, make_bn, stat_out, zeros64  # noqa: E402

SHAPES = [(32, 256, 256, 32, 3), (32, 128, 128, 144, 3), (32, 64, 64, 240, 5), (32, 32, 32, 480, 3),
          (32, 32, 32, 480, 5), (32, 32, 32, 672, 5), (32, 16, 16, 1152, 5), (32, 16, 16, 1152, 3),
          (32, 0, 0, 64, 3), (32, 64, 64, 64, 3)]  # H = 0: the D0 P3-P7 pyramid
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
    targets = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 512, 2048, 4096, 8192]
    dev = L.lib().fns["edet_dev_set"]
    rng = np.random.default_rng(0)
    s = stream()
    tot = {}
    for B, H, W, C, k in SHAPES:
        pin = Pyr(B, D0_PYR if H == 0 else [(H, W)])
        x = torch.randn(pin.rows, C, device="cuda").to(torch.bfloat16)
        lz = LazyDesc(x, pin, C, bn=make_bn(x, pin, C, rng), act=1)
        w = torch.randn(k * k, C, device="cuda").to(torch.bfloat16)
        y = torch.empty(pin.rows, C, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(pin.rows, C, device="cuda").to(torch.bfloat16)
        dx = torch.empty(pin.rows, C, device="cuda", dtype=torch.bfloat16)
        dw = torch.zeros(k * k, C, device="cuda")
        so = stat_out([(zeros64(C), zeros64(C)) for _ in range(pin.nseg)])
        _, acc = bngrad64(pin.nseg, C)
        row = {}
        row["dgrad"] = timeit(lambda: L.call("edet_dwconv_dgrad", L.BF16, vp(dy), pin.c, C, k, 1, vp(w), vp(dx), pin.c, 0, s))
        row["wgrad"] = timeit(lambda: L.call("edet_dwconv_wgrad", L.BF16, lz.c, pin.c, C, k, 1, vp(dy), pin.c, vp(dw), s))
        row["reduce"] = timeit(lambda: L.call("edet_lazy_bwd_reduce", L.BF16, lz.c, pin.c, C, vp(dx), None, None, acc, s))
        for t in targets:
            dev(16, t)
            row[f"bwd@{t}"] = timeit(lambda: L.call("edet_dwconv_bwd", L.BF16, lz.c, pin.c, C, k, 1, vp(dy), pin.c,
                                                     vp(w), vp(dx), 0, vp(dw), acc, s))
        dev(16, 0)
        for t in targets:
            dev(6, t)
            row[f"fwd@{t}"] = timeit(lambda: L.call("edet_dwconv_fwd", L.BF16, lz.c, pin.c, C, k, 1, vp(w), vp(y),
                                                     pin.c, so, s))
        dev(6, 0)
        mb = pin.rows * C * 2 / 1e6
        sep = row["dgrad"] + row["wgrad"] + row["reduce"]
        print(f"B={B} H={H} C={C} k={k} ({mb:.0f} MB/tensor): separate {sep:.1f} "
              f"(dgrad {row['dgrad']:.1f} wgrad {row['wgrad']:.1f} reduce {row['reduce']:.1f}) | "
              + " ".join(f"{n} {v:.1f}" for n, v in row.items() if "@" in n), flush=True)
        for n, v in row.items():
            tot[n] = tot.get(n, 0.0) + v
        del x, y, dy, dx
    print("totals: " + " ".join(f"{n} {v:.1f}" for n, v in tot.items()))


if __name__ == "__main__":
    main()
