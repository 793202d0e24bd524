"""Where the D4 bench's gnorm (1044 in r01h, 197 in r01e) comes from: the per-step loss and
pre-clip gradient norm of the bench's own setup (same synthetic batch every step, the bench's
LR schedule), for D4 1024^2 B=8 in bf16 (twice, to show run-to-run spread) and fp32, and D0
512^2 B=32 bf16 for comparison.

    python scripts/d4_gnorm.py [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import synthetic_batch  # noqa: E402
from tf2mv_amd.anchors import Anchors  # noqa: E402
from tf2mv_amd.config import efficientnet_b0_blocks, get_efficientdet_config  # noqa: E402
from tf2mv_amd.model import EfficientDetNetTrain  # noqa: E402


def run(name, B, dtype, steps, tag):
    cfg = get_efficientdet_config(name)
    S = cfg.image_size
    anchors = Anchors(cfg.min_level, cfg.max_level, (S, S), cfg.num_scales, cfg.aspect_ratios, cfg.anchor_scale)
    m = EfficientDetNetTrain(efficientnet_b0_blocks(), cfg, anchors, dtype=dtype, seed=0,
                             lr_schedule={"warmup_steps": 100, "total_steps": 10000, "adjusted_lr": 0.08 * B / 64})
    x, t = synthetic_batch(anchors, B, S, 1000, "cuda", m.eng.tdtype)
    out = []
    top = {}
    for i in range(steps):
        r = m.train_step((x, t))
        out.append((float(r["loss"]), float(r["gnorm"])))
        if i in (0, steps - 1):
            g = {k: float((v.astype(np.float64) ** 2).sum()) for k, v in m.P.grads_dict().items()}
            tot = sum(g.values())
            top[i] = [(k, round(v / tot, 3)) for k, v in sorted(g.items(), key=lambda kv: -kv[1])[:6]]
    npos = float(t.mask.float().sum())
    print(f"{tag}: {name} B={B} {dtype} N+={npos:.0f}  " +
          "  ".join(f"{i}:{l:.3f}/{g:.1f}" for i, (l, g) in enumerate(out)), flush=True)
    for i, tp in top.items():
        print(f"{tag}: step {i} largest shares of gnorm^2: {tp}", flush=True)
    if hasattr(m, "scalars"):
        print(f"{tag}: scalars {m.scalars.cpu().tolist()}", flush=True)
    del m, x, t
    torch.cuda.empty_cache()


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    run("efficientdet-d0", 32, "bf16", steps, "d0")
    run("efficientdet-d4", 1, "f32", 2, "d4-b1")
    run("efficientdet-d4", 8, "bf16", steps, "d4-run1")
    run("efficientdet-d4", 8, "f32", steps, "d4-f32")


if __name__ == "__main__":
    main()
