"""Training augmentation on the GPU (edet_augment_image, csrc/augment.hip; SURVEY §8(f) row 4,
coco_dataset_one.py:99-135) against the CPU restatements of the OpenCV operations
(oracle/ref_augment.py, data.resize_area).  Parity-unpinned (cv2 absent): blur and warp must
equal the restatement bit for bit, the resize within one uint8 level (the host's einsum sums in
another order), the noise is checked as a distribution.
"""
import os
import random

import numpy as np
import pytest
import torch

from oracle import ref_augment as R
from tf2mv_amd import _lib as L
from tf2mv_amd import augment as A
from tf2mv_amd import data as D
from tf2mv_amd.runtime import stream, vp

pytestmark = pytest.mark.gpu


def _run(img, p, oh, ow, dtype=L.F32, out_raw=True):
    h, w = img.shape[:2]
    src = torch.from_numpy(img).cuda()
    scratch = torch.empty(2 * h * w * 3, dtype=torch.uint8, device="cuda")
    p.out_raw = 1 if out_raw else 0
    out = torch.empty((oh, ow, 3), dtype=torch.uint8 if out_raw else (torch.float32 if dtype == L.F32 else torch.bfloat16),
                      device="cuda")
    L.call("edet_augment_image", dtype, vp(src), h, w, p, vp(scratch), vp(out), oh, ow, stream())
    torch.cuda.synchronize()
    return out.cpu().numpy() if out_raw else out.float().cpu().numpy()


def _params(h, w, blur=0, inv=None, noise=False, border=0, bg=(0, 0, 0), place=None, pad_border=0, pad_bg=(0, 0, 0)):
    p = L.AugParams()
    m = np.eye(3) if inv is None else inv
    for i in range(9):
        p.warp[i] = float(np.asarray(m).reshape(-1)[i])
    p.blur, p.noise, p.noise_seed, p.warp_border, p.pad_border = blur, int(noise), 12345, border, pad_border
    p.rw, p.rh, p.top, p.left = place if place is not None else (w, h, 0, 0)
    for c in range(3):
        p.warp_bg[c], p.pad_bg[c] = bg[c], pad_bg[c]
    return p


@pytest.mark.parametrize("k", [2, 3, 4])
@pytest.mark.parametrize("h,w", [(37, 53), (1, 9), (64, 64)])
def test_blur_equals_restatement(k, h, w):
    img = np.random.default_rng(k + h).integers(0, 256, (h, w, 3), dtype=np.uint8)
    out = _run(img, _params(h, w, blur=k), h, w)
    np.testing.assert_array_equal(out, R.box_blur(img, k))


@pytest.mark.parametrize("border", [0, 1])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_warp_equals_restatement(border, seed):
    """A reference-style draw's warp (scale 0.5..2, offset +-45 px) on a 150 x 211 image."""
    rng = random.Random(seed)
    d = A.draw(rng)
    h, w = 150, 211
    img = np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    inv, _, _ = A.augment_geometry(w, h, d, np.zeros((0, 2)), (w, h))
    bg = (17, 200, 99)
    out = _run(img, _params(h, w, inv=inv, border=border, bg=bg), h, w)
    ref = R.warp_perspective(img, inv, bool(border), bg)
    np.testing.assert_array_equal(out, ref)
    # a projective map too
    org = np.float32([[0, 0], [w, 0], [0, h], [w, h]])
    hm = A.perspective_transform(org, np.float32([[10, -7], [w - 3, 12], [-9, h + 4], [w + 15, h - 20]]))
    inv2 = np.linalg.inv(hm)
    np.testing.assert_array_equal(_run(img, _params(h, w, inv=inv2, border=border, bg=bg), h, w),
                                  R.warp_perspective(img, inv2, bool(border), bg))


def test_identity_chain_copies_and_noise_distribution():
    h, w = 97, 131
    img = np.random.default_rng(3).integers(0, 256, (h, w, 3), dtype=np.uint8)
    np.testing.assert_array_equal(_run(img, _params(h, w), h, w), img)
    mid = np.full((300, 300, 3), 128, np.uint8)  # no clipping: noise = out - 128 in [-20, 19]
    n = _run(mid, _params(300, 300, noise=True), 300, 300).astype(np.int64) - 128
    assert n.min() == -20 and n.max() == 19
    counts = np.bincount((n + 20).ravel(), minlength=40)
    assert counts.min() > 0.8 * n.size / 40 and counts.max() < 1.2 * n.size / 40
    assert abs(n.mean() + 0.5) < 0.05
    edge = np.zeros((50, 50, 3), np.uint8)
    e = _run(edge, _params(50, 50, noise=True), 50, 50)
    assert e.max() <= 19 and e.min() == 0  # clipped at 0


@pytest.mark.parametrize("h,w,size", [(480, 640, (512, 512)), (640, 480, (512, 512)), (100, 77, (128, 128)),
                                      (300, 300, (512, 512))])
@pytest.mark.parametrize("pad_border", [0, 1])
def test_resize_and_border(h, w, size, pad_border):
    """The proportional resize into the frame (data.resize_area within one level), the border
    constant or replicated, and the /255 float output."""
    img = np.random.default_rng(h + w).integers(0, 256, (h, w, 3), dtype=np.uint8)
    rw, rh, top, _, left, _ = D._resize_dims(w, h, size)
    bg = (5, 6, 7)
    p = _params(h, w, place=(rw, rh, top, left), pad_border=pad_border, pad_bg=bg)
    out = _run(img, p, size[1], size[0])
    small = D.resize_area(img, rw, rh)
    inner = out[top:top + rh, left:left + rw].astype(np.int64)
    assert np.abs(inner - small).max() <= 1
    if pad_border == 0:
        frame = out.copy()
        frame[top:top + rh, left:left + rw] = bg
        assert (frame == np.uint8(bg)).all()
    else:
        ys = np.clip(np.arange(size[1]) - top, 0, rh - 1)
        xs = np.clip(np.arange(size[0]) - left, 0, rw - 1)
        np.testing.assert_array_equal(out, out[top:top + rh, left:left + rw][ys][:, xs])
    p2 = _params(h, w, place=(rw, rh, top, left), pad_border=pad_border, pad_bg=bg)
    f = _run(img, p2, size[1], size[0], out_raw=False)
    np.testing.assert_array_equal(f, out.astype(np.float32) / 255)


def test_augment_batch_on_the_label_sample(tmp_path):
    """The pipeline on the committed label sample: a seeded draw per image, pixels written into
    the batch tensor, boxes from the host geometry after the clip / 2-px filter; the identity
    chain reproduces data.prepare (boxes bit for bit, pixels within one level)."""
    from PIL import Image
    here = os.path.dirname(os.path.abspath(__file__))
    rng = np.random.default_rng(0)
    Image.fromarray(rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)).save(tmp_path / "img_a.png")
    Image.fromarray(rng.integers(0, 256, (640, 480, 3), dtype=np.uint8)).save(tmp_path / "img_b.png")
    classes = D.load_classes(os.path.join(here, "golden", "data", "classes.txt"))
    labels = D.load_labels(os.path.join(here, "golden", "data", "labels.txt"), str(tmp_path), classes,
                           log=lambda *a: None)[:2]
    imgs = [D.read_image(l["image_path"]) for l in labels]
    out = torch.empty((2, 512, 512, 3), dtype=torch.float32, device="cuda")
    res = A.augment_batch(imgs, labels, random.Random(0), (512, 512), out, L.F32, identity=True)
    torch.cuda.synchronize()
    for b, lab in enumerate(labels):
        ref_img, ref_boxes, ref_cls = D.prepare(lab, (512, 512), image=imgs[b])
        np.testing.assert_array_equal(res[b][0], ref_boxes)
        np.testing.assert_array_equal(res[b][1], ref_cls)
        assert np.abs(out[b].cpu().numpy() - ref_img).max() <= 1 / 255 + 1e-6
    res = A.augment_batch(imgs, labels, random.Random(7), (512, 512), out, L.F32)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert np.isfinite(o).all() and o.min() >= 0 and o.max() <= 1
    for boxes, cls in res:
        assert boxes.shape[1] == 4 and len(boxes) == len(cls)
        assert (boxes[:, 2] - boxes[:, 0] >= 2).all() and (boxes[:, 3] - boxes[:, 1] >= 2).all()
        assert (boxes >= 0).all() and (boxes <= 512).all()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_getdataset_augment_end_to_end(tmp_path, dtype):
    """GetDataSet(augment=True) (coco_dataset_one.py:214-246 with get_random_data's chain): a
    batch pulled from the generator has the batch shape and storage dtype, pixels in [0, 1],
    and targets equal to generate_targets_batched of the draws' own boxes -- the augmented
    boxes are recomputed here from the same seeded streams through augment_geometry."""
    from PIL import Image
    from tf2mv_amd.anchors import Anchors
    here = os.path.dirname(os.path.abspath(__file__))
    rng = np.random.default_rng(0)
    Image.fromarray(rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)).save(tmp_path / "img_a.png")
    Image.fromarray(rng.integers(0, 256, (640, 480, 3), dtype=np.uint8)).save(tmp_path / "img_b.png")
    S = 128
    anchors = Anchors(3, 7, (S, S), 3, [(1.0, 1.0), (1.4, 0.7), (0.7, 1.4)], 4.0, device="cuda")
    it, gen = D.GetDataSet(str(tmp_path), os.path.join(here, "golden", "data", "labels.txt"),
                           os.path.join(here, "golden", "data", "classes.txt"), 3, anchors, is_train=True,
                           seed=11, augment=True, dtype=dtype)
    x, t = next(it)
    torch.cuda.synchronize()
    assert x.shape == (3, S, S, 3) and x.is_cuda
    assert x.dtype == (torch.float32 if dtype == "f32" else torch.bfloat16)
    xf = x.float().cpu().numpy()
    assert np.isfinite(xf).all() and xf.min() >= 0 and xf.max() <= 1 and xf.std() > 0.05
    # replay the generator's streams on the host: same label order, same draws, same geometry
    ref_gen = D.DataGenerator(str(tmp_path), os.path.join(here, "golden", "data", "labels.txt"),
                              os.path.join(here, "golden", "data", "classes.txt"), anchors, True, 11)
    labs = ref_gen.generate_labels()
    samples = []
    while len(samples) < 3:
        lab = next(labs)
        img = D.read_image(lab["image_path"])
        d = A.draw(ref_gen.rng, ref_gen.np_rng)
        h, w = img.shape[:2]
        _, pts, _ = A.augment_geometry(w, h, d, np.array(lab["boxes"], np.float64).reshape(-1, 2), (S, S))
        bx = pts.reshape(-1, 4)
        bx[:, 0][bx[:, 0] < 0] = 0
        bx[:, 1][bx[:, 1] < 0] = 0
        bx[:, 2][bx[:, 2] > S] = S
        bx[:, 3][bx[:, 3] > S] = S
        keep = np.logical_and(bx[:, 2] - bx[:, 0] >= 2, bx[:, 3] - bx[:, 1] >= 2)
        if keep.any():
            samples.append((None, bx[keep][:, [1, 0, 3, 2]], np.array(lab["classes"], np.int32)[keep]))
    _, gb, gc, n = D.collate([(np.zeros((1,)), b, c) for _, b, c in samples])
    ref = anchors.generate_targets_batched(gb, gc, n)
    for f in ("cls", "mask"):
        np.testing.assert_array_equal(getattr(t, f).cpu().numpy(), getattr(ref, f).cpu().numpy())
    np.testing.assert_array_equal(t.box.cpu().numpy(), ref.box.cpu().numpy())
