"""Generate tests/golden/config_golden.json by importing the reference's TF-free helpers.

Run from the repo root in the build container (the reference is not on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
Imports (read-only, no bytecode written):
    efficientnet/utils/get_feat_sizes.py, utils/round_filters.py, utils/round_repeats.py,
    utils/block_args.py
and records their outputs over the D0..D7x parameter table so config.py is pinned to the
reference's own arithmetic.  The anchor/IoU known answers are hand-derived from
tests/test_anchors.py:10-15 and efficientnet/utils/iou.py:103-112 (see test_oracle_kat.py).
"""
import json
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference/AIServer"
sys.path.insert(0, REF)

from ai_api.ai_models.efficientnet.utils.get_feat_sizes import get_feat_sizes  # noqa: E402
from ai_api.ai_models.utils.round_filters import round_filters  # noqa: E402
from ai_api.ai_models.utils.round_repeats import round_repeats  # noqa: E402
from ai_api.ai_models.utils.block_args import EfficientDetBlockArgs  # noqa: E402

# (width, depth) per model name, as listed in utils/global_params.py:4-141 (restated: that
# module itself imports TensorFlow through config_class.py and cannot be imported here)
TABLE = {
    "efficientdet-d0": (1.0, 1.0, 512), "efficientdet-d1": (1.0, 1.1, 640), "efficientdet-d1-a": (0.8, 0.8, 640),
    "efficientdet-d2": (1.1, 1.2, 768), "efficientdet-d3": (1.2, 1.4, 896), "efficientdet-d4": (1.4, 1.8, 1024),
    "efficientdet-d5": (1.6, 2.2, 1280), "efficientdet-d6": (1.8, 2.6, 1280), "efficientdet-d7": (1.8, 2.6, 1536),
    "efficientdet-d7x": (2.0, 3.1, 1536),
}
BASE_FILTERS = [32, 16, 24, 40, 80, 112, 192, 320]
BASE_REPEATS = [1, 2, 2, 3, 3, 4, 1]

out = {"models": {}, "feat_sizes": {}, "block_args_fields": list(EfficientDetBlockArgs._fields),
       "block_args_defaults": list(EfficientDetBlockArgs.__new__.__defaults__)}
for name, (w, d, size) in TABLE.items():
    gp = types.SimpleNamespace(depth_coefficient=d)
    out["models"][name] = {
        "filters": [round_filters(f, w, 8) for f in BASE_FILTERS],
        "repeats": [round_repeats(r, gp) for r in BASE_REPEATS],
    }
    out["feat_sizes"][name] = [list(s) for s in get_feat_sizes((size, size), 8)]
for s in (10, 64, 100, 127, 513):
    out["feat_sizes"][f"square_{s}"] = [list(v) for v in get_feat_sizes((s, s + 3), 7)]

dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config_golden.json")
with open(dst, "w") as f:
    json.dump(out, f, indent=1)
print("wrote", dst)
