"""Isolated check + timing of edet_conv1x1_wgrad (bf16 A) at the D0 step's shapes.

    python scripts/wg_probe.py [--slot S] [--lazy] [mode ...]   modes via edet_dev_set(S, mode) (S = 0)
Prints per shape: relative error vs a torch fp32 reference (--lazy: A = swish(bn(x)) applied on
load, errors against the first mode's result), us per launch, achieved GB/s (algorithmic bytes =
M (K + N) * 2)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tf2mv_amd import _lib as L  # noqa: E402
from tf2mv_amd.runtime import Pyr, ensure_workspace, stream, vp  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tests"))

D0_LEVELS = [(64, 64), (32, 32), (16, 16), (8, 8), (4, 4)]
SHAPES = [  # (rows layout, K, N, lddy)
    ((32, [(256, 256)]), 16, 96, 96), ((32, [(256, 256)]), 32, 16, 16), ((32, [(128, 128)]), 24, 144, 144),
    ((32, [(128, 128)]), 144, 24, 24), ((32, [(128, 128)]), 96, 24, 24), ((32, [(64, 64)]), 40, 240, 240),
    ((32, [(64, 64)]), 240, 40, 40), ((32, [(64, 64)]), 144, 40, 40), ((32, [(64, 64)]), 40, 64, 64),
    ((32, [(64, 64)]), 64, 64, 64), ((32, D0_LEVELS), 64, 64, 64), ((32, D0_LEVELS), 64, 729, 736),
    ((32, D0_LEVELS), 64, 36, 40), ((32, [(32, 32)]), 112, 672, 672), ((32, [(32, 32)]), 672, 112, 112),
    ((32, [(32, 32)]), 480, 80, 80), ((32, [(32, 32)]), 80, 480, 480), ((32, [(32, 32)]), 480, 112, 112),
    ((32, [(16, 16)]), 1152, 320, 320), ((32, [(16, 16)]), 1152, 192, 192), ((32, [(16, 16)]), 192, 1152, 1152),
    ((32, [(16, 16)]), 672, 192, 192), ((32, [(8, 8)]), 320, 64, 64),
]


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
    args = sys.argv[1:]
    slot, lazy = 0, "--lazy" in args
    if "--slot" in args:
        slot = int(args[args.index("--slot") + 1])
        del args[args.index("--slot"):args.index("--slot") + 2]
    modes = [int(m) for m in args if m != "--lazy"] or [0]
    if lazy:
        import numpy as np
        from gpu_util import LazyDesc, make_bn
        rng = np.random.default_rng(0)
    lib = L.lib()
    dev = getattr(lib.dll, "edet_dev_set", None)
    ensure_workspace(torch.device("cuda"))
    torch.manual_seed(0)
    tot = {m: 0.0 for m in modes}
    for (B, sizes), K, N, lddy in SHAPES:
        pyr = Pyr(B, sizes)
        M = pyr.rows
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        dy = torch.zeros(M, lddy, device="cuda", dtype=torch.bfloat16)
        dy[:, :N] = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        valid = torch.zeros(M, dtype=torch.bool, device="cuda")
        for sgi in range(pyr.nseg):
            valid[pyr.seg_slice(sgi)] = True
        ref_w = (dy[valid, :N].float().t() @ a[valid].float()).double()
        ref_b = dy[valid, :N].float().sum(0).double()
        if lazy:
            ld = LazyDesc(a, pyr, K, bn=make_bn(a, pyr, K, rng), act=1)
            lzp = ld.c
        else:
            lz = L.Lazy()
            lz.x, lz.gate, lz.ld, lz.act = a.data_ptr(), None, K, 0
            lzp = ctypes.byref(lz)
        algo = sum(pyr.seg_rows(i) for i in range(pyr.nseg)) * (K + N) * 2
        line = f"M={M:8d} K={K:5d} N={N:5d}"
        for m in modes:
            if dev is not None:
                dev(slot, m)
            dw = torch.zeros(N, K, device="cuda")
            db = torch.zeros(N, device="cuda")
            L.call("edet_conv1x1_wgrad", L.BF16, lzp, pyr.c, K, vp(dy), lddy, N, vp(dw), vp(db), stream())
            torch.cuda.synchronize()
            if lazy and m == modes[0]:
                ref_w, ref_b = dw.double().clone(), db.double().clone()
            ew = float((dw.double() - ref_w).norm() / ref_w.norm())
            eb = float((db.double() - ref_b).norm() / ref_b.norm())
            us = timeit(lambda: L.call("edet_conv1x1_wgrad", L.BF16, lzp, pyr.c, K, vp(dy), lddy, N,
                                       vp(dw), vp(db), stream()))
            tot[m] += us
            flag = "" if ew < 1e-4 and eb < 1e-4 else "  <<< WRONG"
            line += f" | m{m} {us:7.1f} us {algo / (us * 1e3):6.0f} GB/s err {ew:.1e}/{eb:.1e}{flag}"
        print(line, flush=True)
    print("total " + " ".join(f"m{m}={t:.1f}us" for m, t in tot.items()))
    if dev is not None:
        dev(slot, 0)


if __name__ == "__main__":
    main()
