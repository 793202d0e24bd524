"""Known-answer tests pinning the CPU oracle (oracle/ref_anchors.py) — SURVEY §8(c)."""
import numpy as np

from oracle import ref_anchors as RA

f32 = np.float32


def test_iou_kat_from_iou_main():
    # efficientnet/utils/iou.py:103-112: [10,10,30,30] vs [20,20,40,40]
    b1, b2 = np.array([[10, 10, 30, 30]], f32), np.array([[20, 20, 40, 40]], f32)
    assert RA.iou(b1, b2)[0] == f32(100.0) / f32(700.0)
    np.testing.assert_allclose(RA.diou(b1, b2)[0], 100 / 700 - 200 / 1800, rtol=1e-6)


def test_anchors_kat_from_test_anchors():
    # tests/test_anchors.py:10-15: Anchors(0, 0, (10, 10), 3, [(1,1)], 3.0)
    lv = RA.generate_boxes(0, 0, (10, 10), 3, [(1.0, 1.0)], 3.0)
    assert len(lv) == 1 and lv[0].shape == (10, 10, 3, 4)
    b = lv[0]
    np.testing.assert_array_equal(b[0, :, 0, 1] + f32(1.5), np.arange(10, dtype=f32) + f32(0.5))  # centres .5..9.5
    halves = (b[..., 2] - b[..., 0]) / 2
    np.testing.assert_allclose(halves[0, 0], [1.5, 1.889882, 2.381102], rtol=1e-6)
    np.testing.assert_array_equal(b[4, 4, 0], np.array([3, 3, 6, 6], f32))  # exactly the first GT


def test_targets_kat_from_test_anchors():
    lv = RA.generate_boxes(0, 0, (10, 10), 3, [(1.0, 1.0)], 3.0)
    boxes = np.array([[3, 3, 6, 6], [5, 5, 9, 9]], f32)
    ob, oc, om, oi = RA.generate_targets(lv, boxes, [1, 2], 3)
    assert om[0][4, 4, 0, 0] and oi[0][4, 4, 0] == 1
    np.testing.assert_array_equal(ob[0][4, 4, 0], np.zeros(4, f32))  # IoU 1 -> encoded (0,0,0,0)
    assert oc[0].shape == (10, 10, 3, 3) and oc[0][4, 4, 0].tolist() == [0, 1, 0]
    assert not om[0][0, 0, 0, 0] and oc[0][0, 0, 0].tolist() == [1, 0, 0]  # BG is class 0
    # second GT: the 4x4 box centred at (7,7) matches an anchor at a centre 6.5/7.5
    assert oi[0].max() == 2


def test_encode_decode_roundtrip():
    rng = np.random.default_rng(0)
    a = np.sort(rng.uniform(0, 100, (64, 2, 2)).astype(f32), axis=1).transpose(0, 2, 1).reshape(64, 4)[:, [0, 2, 1, 3]]
    a = np.stack([a[:, 0], a[:, 1], a[:, 0] + 5 + a[:, 2] % 20, a[:, 1] + 5 + a[:, 3] % 20], -1).astype(f32)
    g = a + rng.uniform(-2, 2, a.shape).astype(f32)
    g[:, 2:] = np.maximum(g[:, 2:], g[:, :2] + 1)
    np.testing.assert_allclose(RA.decode(a, RA.encode(a, g)), g, rtol=0, atol=1e-3)


def test_nms_oracle_greedy_diou():
    # three overlapping boxes around (10,10), one far away; scores are logits
    boxes = np.array([[0, 0, 10, 10], [1, 1, 11, 11], [30, 30, 40, 40], [0, 0, 10, 10.5]], f32)
    scores = np.array([0.5, 0.9, 0.7, 0.9], f32)
    # order by score desc, ties by index: 1, 3, 2, 0.  Box 1 suppresses 3 (DIoU >= 0.5) and 0.
    assert RA.diou(boxes[1:2], boxes[3:4])[0] >= 0.5 and RA.diou(boxes[1:2], boxes[0:1])[0] >= 0.5
    np.testing.assert_array_equal(RA.get_nms(boxes, scores, 200, 0.5, 1e-4), [1, 2])
    np.testing.assert_array_equal(RA.get_nms(boxes, scores, 1, 0.5, 1e-4), [1])
    # score threshold on the logits: nothing at or above 1.0
    assert RA.get_nms(boxes, scores, 200, 0.5, 1.0).size == 0


def test_convert_outputs_one_drops_background():
    boxes = [np.arange(2 * 2 * 1 * 4, dtype=f32).reshape(2, 2, 1, 4) * f32(10)]
    lg = np.full((2, 2, 1, 3), -5, f32)
    lg[0, 0, 0] = [3, 1, 0]     # background wins: dropped
    lg[0, 1, 0] = [0, 2, 1]     # class 1, logit 2
    lg[1, 1, 0] = [0, 1, 1]     # tie between classes 1 and 2: first max (1)
    b, c, s = RA.convert_outputs_one(boxes, [lg])
    np.testing.assert_array_equal(c, [1, 1])
    np.testing.assert_allclose(s, 1 / (1 + np.exp(-np.array([2.0, 1.0]))), rtol=1e-6)
