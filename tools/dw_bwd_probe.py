"""Depthwise backward A/B over the D0 b32 stride-1 shapes (development; EDET_DEV library).

For each shape: the separate path (edet_dwconv_dgrad + edet_dwconv_wgrad + the BN-backward
reduce of the input) against the fused edet_dwconv_bwd (with the fold), and the forward, each
under several development-slot settings ("slot=value+slot=value", comma-separated variants;
bwd: 16 = block target, 17 = 2 for two rows in flight; fwd: 6 = block target, 18 = 2).

    EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so python tools/dw_bwd_probe.py \
        "16=0,17=2,16=2048+17=2" "6=0,18=2"
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
    def variants(arg):
        out = []
        for v in arg.split(","):
            out.append((v, [tuple(int(a) for a in kv.split("=")) for kv in v.split("+") if kv]))
        return out
    bwd_vars = variants(sys.argv[1] if len(sys.argv) > 1 else "16=0")
    fwd_vars = variants(sys.argv[2] if len(sys.argv) > 2 else "6=0")
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
        for name, kvs in bwd_vars:
            for a, b in kvs:
                dev(a, b)
            row[f"bwd@{name}"] = timeit(lambda: L.call("edet_dwconv_bwd", L.BF16, lz.c, pin.c, C, k, 1, vp(dy), pin.c,
                                                        vp(w), vp(dx), 0, vp(dw), acc, s))
            for a, _ in kvs:
                dev(a, 0)
        for name, kvs in fwd_vars:
            for a, b in kvs:
                dev(a, b)
            row[f"fwd@{name}"] = timeit(lambda: L.call("edet_dwconv_fwd", L.BF16, lz.c, pin.c, C, k, 1, vp(w), vp(y),
                                                        pin.c, so, s))
            for a, _ in kvs:
                dev(a, 0)
        # every variant must give the default's results bit for bit (same arithmetic order)
        def outputs(kvs):
            for a, b in kvs:
                dev(a, b)
            dw.zero_()
            L.call("edet_dwconv_bwd", L.BF16, lz.c, pin.c, C, k, 1, vp(dy), pin.c, vp(w), vp(dx), 0, vp(dw), None, s)
            L.call("edet_dwconv_fwd", L.BF16, lz.c, pin.c, C, k, 1, vp(w), vp(y), pin.c, None, s)
            torch.cuda.synchronize()
            for a, _ in kvs:
                dev(a, 0)
            return dx.clone(), y.clone()
        ref_dx, ref_y = outputs([])
        same = all(torch.equal(a, b) for _, kvs in bwd_vars + fwd_vars for a, b in zip(outputs(kvs), (ref_dx, ref_y)))
        mb = pin.rows * C * 2 / 1e6
        sep = row["dgrad"] + row["wgrad"] + row["reduce"]
        print(f"B={B} H={H} C={C} k={k} ({mb:.0f} MB/tensor) identical={same}: separate {sep:.1f} "
              f"(dgrad {row['dgrad']:.1f} wgrad {row['wgrad']:.1f} reduce {row['reduce']:.1f}) | "
              + " ".join(f"{n} {v:.1f}" for n, v in row.items() if "@" in n), flush=True)
        for n, v in row.items():
            tot[n] = tot.get(n, 0.0) + v
        del x, y, dy, dx
    print("totals: " + " ".join(f"{n} {v:.1f}" for n, v in tot.items()))


if __name__ == "__main__":
    main()
