"""Isolated timing of the lazy BN-backward row kernels (reduce + apply) at one shape.

  python scripts/row_probe.py M C [gate]
EDET_ROW_PASSES overrides the rows-per-chunk heuristic (A/B only).
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
from gpu_util import LazyDesc, bngrad64, make_bn, seg_out  # noqa: E402


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
    M, C = int(sys.argv[1]), int(sys.argv[2])
    gate = len(sys.argv) > 3 and sys.argv[3] == "1"
    rng = np.random.default_rng(0)
    B = 32
    hw = M // B
    pyr = Pyr(B, [(hw, 1)])
    x = torch.randn(pyr.rows, C, device="cuda").to(torch.bfloat16)
    gt = (torch.rand(B, C, device="cuda") + 0.5) if gate else None
    lz = LazyDesc(x, pyr, C, bn=make_bn(x, pyr, C, rng), act=1, gate=gt)
    dv = torch.randn(pyr.rows, C, device="cuda").to(torch.bfloat16)
    dx = torch.empty_like(dv)
    grads = [(torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda"))]
    so = seg_out(grads)
    _, acc = bngrad64(1, C)
    s = stream()
    tr = timeit(lambda: L.call("edet_lazy_bwd_reduce", L.BF16, lz.c, pyr.c, C, vp(dv), None, None, acc, s))
    ta = timeit(lambda: L.call("edet_lazy_bwd_apply", L.BF16, lz.c, pyr.c, C, vp(dv), None, None, acc, so, vp(dx), 0, s))
    mb = M * C * 2 / 1e6
    print(f"M={M} C={C} gate={int(gate)} passes={os.environ.get('EDET_ROW_PASSES', 'auto')}: "
          f"reduce {tr:7.1f} us {2 * mb / tr * 1e-3:6.2f} TB/s   apply {ta:7.1f} us {3 * mb / ta * 1e-3:6.2f} TB/s")


if __name__ == "__main__":
    main()
