"""Host mAP of test_step (metrics.py) against the reference's own utils/mAP.py outputs.

tests/golden/map_golden.json was produced by tests/golden/make_map_golden.py, which runs the
reference module (the data of its main() and seeded single-image Get_mAP_one cases)."""
import json
import os

import numpy as np
import pytest

from tf2mv_amd import metrics

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "map_golden.json")))


@pytest.mark.parametrize("i", range(len(CASES)))
def test_map_matches_reference(i):
    c = CASES[i]
    if c["kind"] == "get_map":
        v = metrics.get_map(c["data"], c["class_num"], c["thresh"])
    else:
        v = metrics.get_map_one(c["ground_truth"], c["prediction"], c["class_num"], c["thresh"])
    assert v == c["value"]


def test_map_perfect_and_empty():
    gt = [[0, 0, 10, 10, 1], [20, 20, 30, 30, 2]]
    pred = [[0, 0, 10, 10, 1, 0.9], [20, 20, 30, 30, 2, 0.8]]
    # classes 1 and 2 perfect; class 0 has no ground truth and no predictions -> AP 0
    assert metrics.get_map_one(gt, pred, 3) == pytest.approx(2 / 3)
    assert metrics.get_map_one(gt, np.zeros((0, 6)), 3) == 0.0
