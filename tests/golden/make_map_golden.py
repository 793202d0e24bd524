"""Generate tests/golden/map_golden.json by running the reference's utils/mAP.py.

Run from the repo root in the build container (the reference is not on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_map_golden.py
The module imports only numpy.  It uses ``np.float``, which numpy 2.x removed (it was the
builtin float), so the alias is restored for the run.  Cases: the data of the module's own
main() (Get_mAP over two images) and seeded random single-image Get_mAP_one calls shaped
like test_step's (ground truth [y1,x1,y2,x2,class], predictions [..., class, score]).
"""
import json
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference/AIServer")
np.float = float  # removed alias (numpy >= 1.24); the reference was written against numpy 1.x
from ai_api.ai_models.utils import mAP as ref  # noqa: E402

cases = []
main_data = [
    {"image_path": "*.jpg", "groud_truth": [[1, 1, 2, 2, 1], [1, 1, 2, 2, 2], [1, 1.3, 2.4, 2, 1], [3, 1, 4, 2, 2]],
     "prediction": [[1.1, 1, 2.1, 2.2, 1, 0.8], [1.2, 1.2, 2.2, 2.2, 2, 0.7], [1.1, 1.3, 2.4, 2.1, 1, 0.6],
                    [1.1, 1.1, 2.1, 2.1, 1, 0.9]]},
    {"image_path": "*.jpg", "groud_truth": [[1, 1, 2, 2, 1], [1, 1, 2, 2, 2], [1, 1.3, 2.4, 2, 1], [3, 1, 4, 2, 2],
                                            [3, 1, 4, 2, 0]],
     "prediction": [[1.1, 1, 2.1, 2.2, 1, 0.8], [1.2, 1.2, 2.2, 2.2, 2, 0.7], [1.1, 1.3, 2.4, 2.1, 1, 0.7],
                    [1.1, 1.1, 2.1, 2.1, 1, 0.6]]},
]
cases.append({"kind": "get_map", "data": main_data, "class_num": 3, "thresh": 0.5,
              "value": float(ref.Get_mAP(main_data, class_num=3, thresh=0.5))})

rng = np.random.default_rng(7)
for k in range(12):
    nc = int(rng.integers(2, 6))
    ng, npred = int(rng.integers(1, 8)), int(rng.integers(1, 30))
    c = rng.uniform(0, 100, (ng, 2))
    s = rng.uniform(5, 40, (ng, 2))
    gt = np.concatenate([c - s / 2, c + s / 2, rng.integers(0, nc, (ng, 1))], 1)
    base = gt[rng.integers(0, ng, npred), :4] + rng.normal(0, 4, (npred, 4))
    pred = np.concatenate([base, rng.integers(0, nc, (npred, 1)), rng.uniform(0, 1, (npred, 1))], 1)
    gt, pred = np.round(gt, 3), np.round(pred, 3)
    v = float(ref.Get_mAP_one(gt.tolist(), pred.tolist(), nc, 0.5))
    cases.append({"kind": "get_map_one", "ground_truth": gt.tolist(), "prediction": pred.tolist(),
                  "class_num": nc, "thresh": 0.5, "value": v})

dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "map_golden.json")
with open(dst, "w") as f:
    json.dump(cases, f)
print("wrote", dst, len(cases), "cases")
