"""Input pipeline and checkpoint naming, CPU.

Known answers for the reference's label format (datasets/coco_dataset_one.py:29-72) on the
committed sample tests/golden/data/{classes,labels}.txt, the proportional-resize geometry
(utils/image_helper.py:293-358) including its (y, x) field quirk, the class-balanced sample
loop (:156-212) and the Keras name/layout map (checkpoint.py).  Pixel values of the INTER_AREA
restatement are parity-unpinned (cv2 absent); only exact cases are asserted for them.
"""
import os

import numpy as np
import pytest

from tf2mv_amd import checkpoint as CK
from tf2mv_amd import data as D

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "data")


def _images(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    Image.fromarray(rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)).save(tmp_path / "img_a.png")  # W 640, H 480
    Image.fromarray(rng.integers(0, 256, (640, 480, 3), dtype=np.uint8)).save(tmp_path / "img_b.png")  # W 480, H 640
    Image.fromarray(np.zeros((32, 32, 3), np.uint8)).save(tmp_path / "img_c.png")
    return str(tmp_path)


def test_load_classes_and_labels():
    classes = D.load_classes(os.path.join(FIX, "classes.txt"))
    assert classes == ["BG", "cat", "dog", "person"]
    logged = []
    labels = D.load_labels(os.path.join(FIX, "labels.txt"), "/imgs", classes, log=lambda *a: logged.append(a))
    assert [os.path.basename(l["image_path"]) for l in labels] == ["img_a.png", "img_b.png", "img_c.png"]
    assert labels[0]["classes"] == [1, 2] and labels[0]["boxes"] == [[200.0, 100.0, 400.0, 300.0], [20.0, 10.0, 90.0, 60.0]]
    # empty field skipped, unknown class reported and skipped
    assert labels[1]["classes"] == [3, 1] and labels[1]["boxes"] == [[0.0, 0.0, 479.0, 639.0], [10.0, 600.0, 30.0, 700.0]]
    assert len(logged) == 1 and logged[0][1] == "horse"
    assert labels[2]["classes"] == [] and labels[2]["boxes"] == []


def test_prepare_known_answers(tmp_path):
    root = _images(tmp_path)
    classes = D.load_classes(os.path.join(FIX, "classes.txt"))
    labels = D.load_labels(os.path.join(FIX, "labels.txt"), root, classes, log=lambda *a: None)
    # 640x480 -> 512x512: resized 512x384, top 64; fields (f1, f2) land on (y, x)
    img, boxes, cls = D.prepare(labels[0], (512, 512))
    assert img.shape == (512, 512, 3) and img.dtype == np.float32 and 0 <= img.min() and img.max() <= 1
    np.testing.assert_array_equal(boxes, np.float32([[144, 160, 304, 320], [72, 16, 112, 72]]))
    np.testing.assert_array_equal(cls, [1, 2])
    assert np.all(img[:64] == np.float32(128) / 255) and np.all(img[448:] == np.float32(128) / 255)
    # 480x640 -> 512x512: resized 384x512, left 64; the last box is clipped at the bottom edge
    img, boxes, cls = D.prepare(labels[1], (512, 512))
    np.testing.assert_allclose(boxes, [[0, 64, 511.2, 447.2], [480, 72, 512, 88]], rtol=0, atol=1e-4)
    np.testing.assert_array_equal(cls, [3, 1])
    assert np.all(img[:, :64] == np.float32(128) / 255)


def test_prepare_drops_degenerate_boxes():
    lab = {"image_path": "", "classes": [1, 2, 3], "boxes": [[10, 10, 11, 50], [-30, -30, -10, -5], [5, 5, 40, 40]]}
    _, boxes, cls = D.prepare(lab, (64, 64), image=np.zeros((64, 64, 3), np.uint8))
    # box 0 is 1 px wide, box 1 clips to zero extent: only box 2 survives
    np.testing.assert_array_equal(cls, [3])
    np.testing.assert_array_equal(boxes, np.float32([[5, 5, 40, 40]]))


def test_point_geometry_float32():
    # identity perspective is float32 arithmetic, not an exact no-op (image_helper.py:183-186)
    p = D.identity_perspective_points((640, 480), [[123.4, 56.7]])
    c = np.float32([320, 240])
    want_x = np.float32(np.float32(np.float32(np.float32(123.4) - c[0]) * np.float32(640)) / np.float32(640)) + c[0]
    assert p[0, 0] == want_x and p.dtype == np.float32
    pts, pad = D.proportional_resize_points((640, 480), (512, 512), [[640, 480]])
    assert pad == (64, 64, 0, 0)
    np.testing.assert_array_equal(pts, np.float32([[512, 448]]))


def test_resize_area_exact_cases():
    a = np.arange(4 * 4 * 3, dtype=np.uint8).reshape(4, 4, 3) * 4
    out = D.resize_area(a, 2, 2)
    want = a.reshape(2, 2, 2, 2, 3).astype(np.float64).mean(axis=(1, 3))
    np.testing.assert_array_equal(out, np.rint(want).astype(np.uint8))
    const = np.full((7, 9, 3), 77, np.uint8)
    np.testing.assert_array_equal(D.resize_area(const, 5, 3), np.full((3, 5, 3), 77, np.uint8))
    np.testing.assert_array_equal(D.resize_area(const, 13, 11), np.full((11, 13, 3), 77, np.uint8))


def test_generator_balances_classes_and_skips_empty(tmp_path):
    root = _images(tmp_path)

    class _A:
        image_size = (512, 512)
        device = "cpu"
    gen = D.DataGenerator(root, os.path.join(FIX, "labels.txt"), os.path.join(FIX, "classes.txt"), _A(), True, seed=3)
    it = gen.generate()
    seen = [next(it) for _ in range(6)]
    # class_list = [1, 2, 3]; the k-th yielded image holds class class_list[k % 3] (img_c, with
    # no boxes, is never yielded)
    for k, (img, boxes, cls) in enumerate(seen):
        assert img.shape == (512, 512, 3) and len(cls) > 0
        assert [1, 2, 3][k % 3] in set(cls.tolist())
    x, gb, gc, n = D.collate(seen[:2])
    assert x.shape == (2, 512, 512, 3) and gb.shape[0] == 2 and n.tolist() == [len(seen[0][2]), len(seen[1][2])]


def test_keras_layout_roundtrip():
    from oracle.ref_model import param_specs
    from tf2mv_amd.config import get_efficientdet_config
    cfg = get_efficientdet_config("efficientdet-d0", {"image_size": 128, "num_classes": 5})
    rng = np.random.default_rng(0)
    sd = {n: rng.standard_normal(shape).astype(np.float32) for n, (shape, _) in param_specs(cfg).items()}
    kr = CK.keras_state_dict(sd)
    assert all(k.endswith(":0") for k in kr)
    # Keras conventions: 1x1 conv and pointwise [1,1,Cin,Cout], depthwise [k,k,C,1], stem [3,3,3,32]
    assert kr["efficientnet-b0/blocks_0/conv2d/kernel:0"].shape == (1, 1, 32, 16)
    assert kr["efficientnet-b0/blocks_0/depthwise_conv2d/depthwise_kernel:0"].shape == (3, 3, 32, 1)
    assert kr["efficientnet-b0/blocks_0/se/conv2d/kernel:0"].shape == (1, 1, 32, 8)
    assert kr["class_net/class-predict/pointwise_kernel:0"].shape == (1, 1, 64, 45)
    assert kr["efficientnet-b0/stem/conv2d/kernel:0"].shape == (3, 3, 3, 32)
    assert kr["bi_fpn/bi_fpn_node/WSM_0:0"].shape == ()  # scalars (bifpn.py:45-54)
    # the transposition really moves elements (not a reshape)
    w = sd["efficientnet-b0/blocks_0/conv2d/kernel"]
    assert kr["efficientnet-b0/blocks_0/conv2d/kernel:0"][0, 0, 3, 5] == w[5, 3]
    d = sd["efficientnet-b0/blocks_0/depthwise_conv2d/depthwise_kernel"]
    assert kr["efficientnet-b0/blocks_0/depthwise_conv2d/depthwise_kernel:0"][1, 2, 7, 0] == d[1 * 3 + 2, 7]
    class _M:
        def state_dict(self):
            return {k: np.zeros_like(v) for k, v in sd.items()}

        def load_state_dict(self, d):
            self.d = d
    m = _M()
    CK.load_keras_state_dict(m, kr, strict=True)
    assert m.d.keys() == sd.keys()
    for k in sd:
        np.testing.assert_array_equal(m.d[k], sd[k])


def test_load_keras_state_dict_strictness():
    class _M:
        def __init__(self):
            self.sd = {"a/conv2d/kernel": np.zeros((4, 3), np.float32), "a/bn/gamma": np.ones(4, np.float32)}

        def state_dict(self):
            return dict(self.sd)

        def load_state_dict(self, sd):
            self.sd = sd
    m = _M()
    w = {"a/conv2d/kernel:0": np.arange(12, dtype=np.float32).reshape(1, 1, 3, 4), "a/bn/gamma:0": np.full(4, 2.0)}
    CK.load_keras_state_dict(m, w)
    np.testing.assert_array_equal(m.sd["a/conv2d/kernel"], np.arange(12, dtype=np.float32).reshape(3, 4).T)
    with pytest.raises(KeyError):
        CK.load_keras_state_dict(m, {"a/bn/gamma:0": np.ones(4), "b/x:0": np.ones(1)})
    with pytest.raises(ImportError):
        CK.read_h5_weights("/nonexistent.h5")
