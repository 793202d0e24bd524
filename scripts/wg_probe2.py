"""A/B of edet_conv1x1_wgrad plans through the development slots (edet_dev_set).

    python scripts/wg_probe2.py SPEC [SPEC ...]      SPEC = "slot=value,slot=value" ("-" = all 0)
Shapes and checking as scripts/wg_probe.py; prints us per launch and achieved GB/s per SPEC."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

from tf2mv_amd import _lib as L  # noqa: E402
from tf2mv_amd.runtime import Pyr, ensure_workspace, stream, vp  # noqa: E402
from wg_probe import SHAPES, timeit  # noqa: E402


def parse(spec):
    if spec == "-":
        return {}
    return {int(k): int(v) for k, v in (kv.split("=") for kv in spec.split(","))}


def main():
    specs = sys.argv[1:] or ["-"]
    lib = L.lib()
    dev = lib.fns["edet_dev_set"]
    ensure_workspace(torch.device("cuda"))
    torch.manual_seed(0)
    tot = {s: 0.0 for s in specs}
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
        lz = L.Lazy()
        lz.x, lz.gate, lz.ld, lz.act = a.data_ptr(), None, K, 0
        algo = sum(pyr.seg_rows(i) for i in range(pyr.nseg)) * (K + N) * 2
        line = f"M={M:8d} K={K:5d} N={N:5d}"
        for spec in specs:
            kv = parse(spec)
            for i in range(8):
                dev(i, kv.get(i, 0))
            dw = torch.zeros(N, K, device="cuda")
            db = torch.zeros(N, device="cuda")
            call = lambda: L.call("edet_conv1x1_wgrad", L.BF16, ctypes.byref(lz), pyr.c, K, vp(dy), lddy, N,  # noqa: E731
                                  vp(dw), vp(db), stream())
            call()
            torch.cuda.synchronize()
            ew = float((dw.double() - ref_w).norm() / ref_w.norm())
            eb = float((db.double() - ref_b).norm() / ref_b.norm())
            us = timeit(call)
            tot[spec] += us
            flag = "" if ew < 1e-4 and eb < 1e-4 else " WRONG"
            line += f" | {us:6.1f}us {algo / (us * 1e3):5.0f}{flag}"
        print(line, flush=True)
    for i in range(8):
        dev(i, 0)
    print("total " + " | ".join(f"[{s}] {t:.1f}us" for s, t in tot.items()))


if __name__ == "__main__":
    main()
