"""Training augmentation of the input pipeline: the random chain of
``datasets/coco_dataset_one.py:get_random_data`` (:74-154) with its pixel work on the GPU.

Reference chain (all OpenCV, cv2 is not in this image):
  1. blur          ksize = random.randint(0, 4); cv2.blur(img, (k, k)) when k > 0   (:99-101)
  2. perspective   offset = (U*90 - 45, U*90 - 45), scale = (U*1.5 + 0.5, U*1.5 + 0.5), angles 0
                   (:105-117) -> ImageHelper.opencvPerspective (image_helper.py:110-197): a
                   float32 4x4 transform, the box corners mapped through it and projected,
                   the image warped by cv2.getPerspectiveTransform(corners) with a random
                   border colour and mode (image_helper.py:200-217)
  3. noise         ImageHelper.opencvNoise (image_helper.py:245-257)
  4. resize        ImageHelper.opencvProportionalResize with a random border (image_helper.py:
                   293-330), then BGR->RGB and /255
  5. boxes         clip to the frame, drop < 2 px, reorder (coco_dataset_one.py:138-151)

Here the draws (Python ``random``, exactly the reference's calls in its order; the noise seed from
a separate numpy stream, as the reference's noise comes from numpy's global RNG and consumes
nothing from ``random``), the transform matrices and the
box-corner geometry run on the host in numpy float32 / float64, op for op as the reference
computes them (bit-exact against that restatement: tests/test_augment.py), and the pixel work
-- blur, warp, noise, resize + border + normalisation -- is one ``edet_augment_image`` call
per image (csrc/augment.hip) that writes the image straight into the batch tensor.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

from . import data as D

__all__ = ["AugmentDraw", "draw", "perspective_matrix", "project_points", "perspective_transform",
           "augment_geometry", "aug_params"]


@dataclass
class AugmentDraw:
    """One image's random draws, in the reference's order of calls on its ``random`` module."""
    ksize: int
    offset: Tuple[float, float]
    scale: Tuple[float, float]
    warp_bg: Tuple[int, int, int]      # getRandomColor() of opencvPerspectiveP, BGR
    warp_replicate: bool               # random.random() >= 0.5 -> BORDER_REPLICATE
    noise_seed: int                    # the noise stream (numpy's global RNG in the reference)
    pad_bg: Tuple[int, int, int]       # getRandomColor() of opencvProportionalResize, BGR
    pad_replicate: bool

    @staticmethod
    def identity(pad_bg=(128, 128, 128)) -> "AugmentDraw":
        """No augmentation: the deterministic chain of data.prepare."""
        return AugmentDraw(0, (0.0, 0.0), (1.0, 1.0), (0, 0, 0), False, 0, tuple(pad_bg), False)


def draw(rng: random.Random, np_rng: Optional[np.random.Generator] = None) -> AugmentDraw:
    """coco_dataset_one.py:99-126 / image_helper.py:207-214, 312-318: the same calls on the
    Python ``random`` stream in the same order (randint(0, 4); four random(); getRandomColor +
    random() in the warp; getRandomColor + random() in the resize). The noise
    (image_helper.py:249) draws from numpy's RNG, not from ``random``: its seed comes from
    ``np_rng`` (default: numpy's global RNG, as the reference), so the ``random`` sequence --
    and with it the next image's draws and the generator's shuffle -- is the reference's."""
    ksize = rng.randint(0, 4)
    ox = rng.random() * 90 - 45
    oy = rng.random() * 90 - 45
    sx = rng.random() * 1.5 + 0.5
    sy = rng.random() * 1.5 + 0.5
    wbg = (rng.randint(0, 255), rng.randint(0, 255), rng.randint(0, 255))
    wrep = rng.random() >= 0.5
    seed = (int(np_rng.integers(0, 2**63, dtype=np.int64)) if np_rng is not None
            else int(np.random.randint(0, 2**63, dtype=np.int64)))
    pbg = (rng.randint(0, 255), rng.randint(0, 255), rng.randint(0, 255))
    prep = rng.random() >= 0.5
    return AugmentDraw(ksize, (ox, oy), (sx, sy), wbg, wrep, seed, pbg, prep)


def perspective_matrix(offset=(0.0, 0.0, 0.0), angle=(0.0, 0.0, 0.0), scale=(1.0, 1.0, 1.0)) -> np.ndarray:
    """image_helper.py:121-165: the float32 4x4 row-vector transform, built as the reference
    builds it -- identity, then right-multiplied (np.matmul, float32) by the translation, the
    x / y / z rotations and the scale."""
    f32 = np.float32
    r = np.radians(angle)
    cx, sx_ = math.cos(r[0]), math.sin(r[0])
    cy, sy_ = math.cos(r[1]), math.sin(r[1])
    cz, sz_ = math.cos(r[2]), math.sin(r[2])
    steps = [
        [[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [offset[0], offset[1], offset[2], 1]],
        [[1, 0, 0, 0], [0, cx, -sx_, 0], [0, -sx_, cx, 0], [0, 0, 0, 1]],
        [[cy, 0, sy_, 0], [0, 1, 0, 0], [-sy_, 0, cy, 0], [0, 0, 0, 1]],
        [[cz, sz_, 0, 0], [-sz_, cz, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]],
        [[scale[0], 0, 0, 0], [0, scale[1], 0, 0], [0, 0, scale[2], 0], [0, 0, 0, 1]],
    ]
    m = f32(np.eye(4))
    for s in steps:
        m = np.matmul(m, f32(s))
    return m


def project_points(width: int, height: int, m: np.ndarray, points) -> np.ndarray:
    """image_helper.py:180-188: each point -> (p - centre) @ M, projected onto the image plane
    (x * w / (w + z) + cx), all in float32 as the reference's numpy scalars compute it."""
    centre = np.float32([width / 2, height / 2, 0, 0])
    out = []
    for p in points:
        t = np.matmul(np.float32([p[0], p[1], 0, 1]) - centre, m)
        out.append([t[0] * width / (width + t[2]) + centre[0], t[1] * height / (height + t[2]) + centre[1]])
    return np.float32(out)


def perspective_transform(org: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """cv2.getPerspectiveTransform(org, dst): the 3x3 homography with m22 = 1 mapping the four
    org points onto dst, from the 8x8 linear system in float64 (OpenCV's published system)."""
    a = np.zeros((8, 8), np.float64)
    b = np.zeros(8, np.float64)
    for i in range(4):
        x, y = float(org[i][0]), float(org[i][1])
        u, v = float(dst[i][0]), float(dst[i][1])
        a[i] = [x, y, 1, 0, 0, 0, -x * u, -y * u]
        a[i + 4] = [0, 0, 0, x, y, 1, -x * v, -y * v]
        b[i], b[i + 4] = u, v
    h = np.linalg.solve(a, b)
    return np.append(h, 1.0).reshape(3, 3)


def augment_geometry(width: int, height: int, d: AugmentDraw, boxes_xy, size: Tuple[int, int]):
    """The host half of get_random_data for one image of ``width`` x ``height``: the warp's
    destination -> source map (for edet_augment_image), the box points through the perspective
    and the proportional resize (float32, as the reference), and the resize placement.

    boxes_xy: the label's boxes as stored by load_labels, reshaped (-1, 2) (float64).
    Returns (inverse 3x3 float64, points float32 [n, 2], (rw, rh, top, left))."""
    m = perspective_matrix((d.offset[0], d.offset[1], 0), (0, 0, 0), (d.scale[0], d.scale[1], 1))
    pts = project_points(width, height, m, np.asarray(boxes_xy, np.float64).reshape(-1, 2))
    corners = np.float32([[0, 0], [width, 0], [0, height], [width, height]])
    dst = project_points(width, height, m, corners)
    hmat = perspective_transform(corners, dst)
    inv = np.linalg.inv(hmat)  # warpPerspective maps each destination pixel back (invert, LU)
    rw, rh, top, _, left, _ = D._resize_dims(width, height, size)
    pts, _ = D.proportional_resize_points((width, height), size, pts)
    return inv, pts, (rw, rh, top, left)


def aug_params(d: AugmentDraw, inv: Optional[np.ndarray], placement, L, out_raw: bool = False):
    """edet_aug_params for edet_augment_image (RGB images: the BGR border colours reversed)."""
    p = L.AugParams()
    m = np.eye(3) if inv is None else np.asarray(inv, np.float64)
    for i in range(9):
        p.warp[i] = float(m.reshape(-1)[i])
    p.noise_seed = int(d.noise_seed) & 0xFFFFFFFFFFFFFFFF
    p.blur = int(d.ksize)
    p.warp_border = 1 if d.warp_replicate else 0
    p.noise = 1 if inv is not None else 0
    p.rw, p.rh, p.top, p.left = (int(v) for v in placement)
    p.pad_border = 1 if d.pad_replicate else 0
    p.out_raw = 1 if out_raw else 0
    for c in range(3):
        p.warp_bg[c] = int(d.warp_bg[2 - c])
        p.pad_bg[c] = int(d.pad_bg[2 - c])
    return p


def augment_one(img: np.ndarray, lab: dict, d: AugmentDraw, size: Tuple[int, int], out_b, dtype_code: int,
                identity: bool = False):
    """One image of get_random_data: the host geometry, then (when any box survives the clip /
    2-px filter, else nothing is launched and None returned -- the reference's generator skips
    such samples, coco_dataset_one.py:200-201) one edet_augment_image call writing the pixels into
    ``out_b`` ([size[1], size[0], 3] device tensor in the compute dtype).
    Returns (boxes float32 [n, 4] in generate_targets order, classes int32 [n]) or None."""
    import torch

    from . import _lib as L
    from .runtime import stream, vp
    h, w = img.shape[:2]
    boxes = np.array(lab["boxes"], dtype=np.float64).reshape((-1, 2))
    inv, pts, place = augment_geometry(w, h, d, boxes, size)
    if identity:  # the deterministic chain: data.prepare's geometry, no warp, no noise
        pts = D.identity_perspective_points((w, h), boxes)
        pts, _ = D.proportional_resize_points((w, h), size, pts)
        inv = None
    bx = pts.reshape((-1, 4))
    bx[:, 0][bx[:, 0] < 0] = 0
    bx[:, 1][bx[:, 1] < 0] = 0
    bx[:, 2][bx[:, 2] > size[0]] = size[0]
    bx[:, 3][bx[:, 3] > size[1]] = size[1]
    keep = np.logical_and(bx[:, 2] - bx[:, 0] >= 2, bx[:, 3] - bx[:, 1] >= 2)
    classes = np.array(lab["classes"], dtype=np.int32)[keep]
    if len(classes) == 0:
        return None
    dev = out_b.device
    src = torch.from_numpy(np.array(img, dtype=np.uint8, order="C", copy=True)).to(dev)
    scratch = torch.empty(2 * h * w * 3, dtype=torch.uint8, device=dev)
    p = aug_params(d, inv, place, L)
    L.call("edet_augment_image", dtype_code, vp(src), h, w, p, vp(scratch), vp(out_b), size[1], size[0], stream())
    return bx[keep][:, [1, 0, 3, 2]], classes


def augment_batch(images: Sequence[np.ndarray], labels: Sequence[dict], rng: random.Random, size: Tuple[int, int],
                  out, dtype_code: int, identity: bool = False, np_rng: Optional[np.random.Generator] = None):
    """augment_one over a batch, one draw per image (identity: the deterministic chain).
    Samples left without boxes give None and leave their slot of ``out`` unwritten."""
    return [augment_one(img, lab, AugmentDraw.identity() if identity else draw(rng, np_rng), size, out[b],
                        dtype_code, identity) for b, (img, lab) in enumerate(zip(images, labels))]
