"""A/B of the fused stride-1 depthwise backward forms over the D0 b32 shapes (development;
EDET_DEV library): the row-streaming kernels (edet_dev_set slot 29 = 2) against the tiled form
k_dwt (slot 29 = 1; slots 30 / 31 = block floor / tiles per block).  Per shape: us per launch of
each, and the tiled form's dx / filter gradient / fold sums against the production route's
(fp32 summation order only: relative differences ~1e-6 in fp32, a few bf16 ulp in bf16).

    EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so python tools/dwt_ab.py [bf16|f32] ["30=1024,31=2"]

DWT_A / DWT_B (slot=value lists, default "29=2" / "29=1") choose the two forms, e.g.
DWT_A=29=1 DWT_B=29=1,41=2 for the tiled form against its next-tile DMA variant.
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
from gpu_util import LazyDesc, bngrad64, make_bn  # noqa: E402

SHAPES = [(32, 256, 256, 32, 3), (32, 128, 128, 144, 3), (32, 64, 64, 240, 5), (32, 32, 32, 480, 3),
          (32, 32, 32, 480, 5), (32, 32, 32, 672, 5), (32, 16, 16, 1152, 5), (32, 16, 16, 1152, 3),
          (32, 0, 0, 64, 3), (32, 64, 64, 64, 3), (32, 32, 32, 64, 3), (32, 16, 16, 64, 3)]
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


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    extra = [tuple(int(v) for v in kv.split("=")) for kv in (sys.argv[2].split(",") if len(sys.argv) > 2 else []) if kv]
    tdt, edt = (torch.bfloat16, L.BF16) if dt == "bf16" else (torch.float32, L.F32)
    dev = L.lib().fns["edet_dev_set"]
    rng = np.random.default_rng(0)
    s = stream()
    tot = [0.0, 0.0]
    for B, H, W, C, k in SHAPES:
        pin = Pyr(B, D0_PYR if H == 0 else [(H, W)])
        x = torch.randn(pin.rows, C, device="cuda").to(tdt)
        lz = LazyDesc(x, pin, C, bn=make_bn(x, pin, C, rng), act=1)
        w = (torch.randn(k * k, C, device="cuda") * 0.3).to(tdt)
        dy = torch.randn(pin.rows, C, device="cuda").to(tdt)
        outs, us = [], []
        forms = [os.environ.get("DWT_A", "29=2"), os.environ.get("DWT_B", "29=1")]
        for form in forms:
            slots = [tuple(int(v) for v in kv.split("=")) for kv in form.split(",") if kv] + extra
            for a, b in slots:
                dev(a, b)
            dx = torch.empty(pin.rows, C, device="cuda", dtype=tdt)
            dw = torch.zeros(k * k, C, device="cuda")
            acc_t, acc = bngrad64(pin.nseg, C)
            L.call("edet_dwconv_bwd", edt, lz.c, pin.c, C, k, 1, vp(dy), pin.c, vp(w), vp(dx), 0, vp(dw), acc, s)
            torch.cuda.synchronize()
            outs.append((dx.clone(), dw.clone(), acc_t.clone()))
            us.append(timeit(lambda: L.call("edet_dwconv_bwd", edt, lz.c, pin.c, C, k, 1, vp(dy), pin.c, vp(w),
                                            vp(dx), 0, vp(dw), acc, s)))
            for a, _ in slots:
                dev(a, 0)
        valid = torch.cat([torch.arange(pin.row_off[i], pin.row_off[i] + pin.seg_rows(i)) for i in range(pin.nseg)])
        (dx0, dw0, f0), (dx1, dw1, f1) = outs
        e_dx, e_dw, e_f = rel(dx1[valid], dx0[valid]), rel(dw1, dw0), rel(f1, f0)
        mb = pin.rows * C * 2 / 1e6
        bad = "" if (e_dx < (2e-2 if dt == "bf16" else 1e-5) and e_dw < 1e-3 and e_f < 1e-3) else "  <<< MISMATCH"
        print(f"H={H:3d} C={C:5d} k={k} ({mb:6.1f} MB): A {us[0]:7.1f} us  B {us[1]:7.1f} us  "
              f"x{us[0] / us[1]:.2f} | dx {e_dx:.1e} dw {e_dw:.1e} fold {e_f:.1e}{bad}", flush=True)
        tot[0] += us[0]
        tot[1] += us[1]
    print(f"total A {tot[0]:.1f} us  B {tot[1]:.1f} us  (A = {forms[0]}, B = {forms[1]})")


if __name__ == "__main__":
    main()
