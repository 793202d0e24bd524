"""Run one libedet entry point at one shape a few times (for rocprofv3 counter passes).

    python tools/one_launch.py dwfwd  B H W C k s      (edet_dwconv_fwd, lazy BN+swish input)
    python tools/one_launch.py dwbwd  B H W C k        (edet_dwconv_bwd, stride 1, with the fold)
    python tools/one_launch.py gemm   M K N            (edet_conv1x1_fwd, lazy BN+swish A, stats)
    python tools/one_launch.py wgrad  M K N            (edet_conv1x1_wgrad, plain A)
REPS (default 5) launches, synchronised at the end.
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


def main():
    kind, dims = sys.argv[1], [int(v) for v in sys.argv[2:]]
    reps = int(os.environ.get("REPS", "5"))
    rng = np.random.default_rng(0)
    s = stream()
    bf = torch.bfloat16
    if kind in ("dwfwd", "dwbwd"):
        B, H, W, C, k = dims[:5]
        st = dims[5] if kind == "dwfwd" else 1
        pin = Pyr(B, [(H, W)])
        pout = pin.strided(st)
        x = torch.randn(pin.rows, C, device="cuda").to(bf)
        lz = LazyDesc(x, pin, C, bn=make_bn(x, pin, C, rng), act=1)
        w = torch.randn(k * k, C, device="cuda").to(bf)
        if kind == "dwfwd":
            y = torch.empty(pout.rows, C, device="cuda", dtype=bf)
            so = stat_out([(zeros64(C), zeros64(C))])
            f = lambda: L.call("edet_dwconv_fwd", L.BF16, lz.c, pin.c, C, k, st, vp(w), vp(y), pout.c, so, s)  # noqa: E731
        else:
            dy = torch.randn(pin.rows, C, device="cuda").to(bf)
            dx = torch.empty(pin.rows, C, device="cuda", dtype=bf)
            dw = torch.zeros(k * k, C, device="cuda")
            _, acc = bngrad64(1, C)
            f = lambda: L.call("edet_dwconv_bwd", L.BF16, lz.c, pin.c, C, k, 1, vp(dy), pin.c, vp(w), vp(dx), 0,  # noqa: E731
                               vp(dw), acc, s)
    else:
        M, K, N = dims[:3]
        pyr = Pyr(1, [(M, 1)])
        a = torch.randn(M, K, device="cuda").to(bf)
        if kind == "gemm":
            lz = LazyDesc(a, pyr, K, bn=make_bn(a, pyr, K, rng), act=1)
            wt = (torch.randn(N, K, device="cuda") * 0.1).to(bf)
            y = torch.empty(M, N, device="cuda", dtype=bf)
            so = stat_out([(zeros64(N), zeros64(N))])
            f = lambda: L.call("edet_conv1x1_fwd", L.BF16, lz.c, pyr.c, K, vp(wt), N, None, vp(y), N, 0, so, s)  # noqa: E731
        else:
            lz = LazyDesc(a, pyr, K)
            dy = torch.randn(M, N, device="cuda").to(bf)
            dw = torch.zeros(N, K, device="cuda")
            db = torch.zeros(N, device="cuda")
            f = lambda: L.call("edet_conv1x1_wgrad", L.BF16, lz.c, pyr.c, K, vp(dy), N, N, vp(dw), vp(db), s)  # noqa: E731
    from tf2mv_amd.runtime import ensure_workspace
    ensure_workspace("cuda")
    f()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        f()
    ev[1].record()
    torch.cuda.synchronize()
    print(f"{kind} {dims}: {ev[0].elapsed_time(ev[1]) * 1e3 / reps:.1f} us/launch")


if __name__ == "__main__":
    main()
