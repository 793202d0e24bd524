"""Input pipeline: label files, classes, the deterministic preprocessing chain and batching into
``Anchors.generate_targets_batched`` (the host side feeding the hot path).

Mirrors ``datasets/coco_dataset_one.py`` (``DataGenerator``: ``LoadClasses`` :29-37,
``LoadLabels`` :39-72, ``get_random_data`` :74-154, ``generate`` :156-212, ``GetDataSet``
:214-246) and the geometry of ``utils/image_helper.py`` (``opencvProportionalResize`` :293-330,
``opencvProportionalResizePoint`` :333-358).

Formats:
  classes file   one class name per line; index 0 is the prepended 'BG'.
  label file     ``<relative image path>|<class>,<f1>,<f2>,<f3>,<f4>|...`` one image per line;
                 empty fields are skipped, unknown class names are reported and skipped.

Reference quirk kept on purpose: ``LoadLabels`` stores a box as ``[f2, f1, f4, f3]`` and the
point helpers read every pair as (x, y), so f1/f3 go through the *vertical* resize and f2/f4
through the *horizontal* one; the final ``[:, [1, 0, 3, 2]]`` (coco_dataset_one.py:151) then
yields ``[T_y(f1), T_x(f2), T_y(f3), T_x(f4)]`` -- the label fields are (y1, x1, y2, x2) in
effect, whatever the loader's variable names say.

Augmentation: the reference applies random blur, perspective, noise and a random border in
both its train and eval generators (:94-131).  ``prepare`` runs the chain with every random
draw at its identity (blur size 0, offset 0, scale 1, no noise), i.e. the perspective step maps
every point to itself and only the proportional resize remains; ``GetDataSet(augment=True)``
runs the random chain with its pixel work on the GPU (augment.py, csrc/augment.hip).
``cv2.resize(INTER_AREA)`` is restated below (exact area averaging when shrinking, bilinear
when enlarging); with cv2 absent its pixel values are parity-unpinned, the box geometry is
pinned by the known-answer tests in tests/test_data.py.
"""
from __future__ import annotations

import os
import random
import sys
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

__all__ = ["load_classes", "load_labels", "proportional_resize_points", "identity_perspective_points", "resize_area",
           "proportional_resize", "prepare", "DataGenerator", "collate", "GetDataSet"]


def load_classes(classes_path: str) -> List[str]:
    """coco_dataset_one.py:29-37: ['BG'] + the stripped lines of the classes file."""
    with open(classes_path, "r", encoding="utf-8") as f:
        names = f.readlines()
    return ["BG"] + [c.strip() for c in names]


def load_labels(label_path: str, image_path: str, classes: Sequence[str], log=None) -> List[Dict]:
    """coco_dataset_one.py:39-72: one dict per line with image_path, classes (indices into
    ``classes``) and boxes [[f2, f1, f4, f3], ...] as floats (the reference's storage order)."""
    log = log or (lambda *a: print(*a, file=sys.stderr))
    labels = []
    with open(label_path, "r", encoding="utf-8") as f:
        for line in f.readlines():
            parts = line.strip().split("|")
            full = os.path.join(image_path, parts[0])
            cls, boxes = [], []
            for field in parts[1:]:
                if field == "":
                    continue
                info = field.split(",")
                if info[0] not in classes:
                    log("label error:", info[0], full)
                    continue
                cls.append(list(classes).index(info[0]))
                f1, f2, f3, f4 = (float(v) for v in info[1:5])
                boxes.append([f2, f1, f4, f3])
            labels.append({"image_path": full, "classes": cls, "boxes": boxes})
    return labels


def _resize_dims(width: int, height: int, size: Tuple[int, int]) -> Tuple[int, int, int, int, int, int]:
    """image_helper.py:296-310: long side to the target, padding split floor/ceil."""
    new_w, new_h = size[0], size[1]
    if width / height > new_w / new_h:
        rw = new_w
        rh = int((height / width) * rw)
    else:
        rh = new_h
        rw = int((width / height) * rh)
    top = (new_h - rh) // 2
    bottom = new_h - rh - top
    left = (new_w - rw) // 2
    right = new_w - rw - left
    return rw, rh, top, bottom, left, right


def proportional_resize_points(img_size: Tuple[int, int], size: Tuple[int, int], points) -> Tuple[np.ndarray, Tuple]:
    """image_helper.py:322-329 / 333-358: img_size = (width, height); every point p ->
    (p0 * rw / width + left, p1 * rh / height + top).  The reference's points are a float32
    array, so each operation rounds to float32 (a float32 scalar with a Python int stays
    float32); restated op by op."""
    width, height = img_size
    rw, rh, top, bottom, left, right = _resize_dims(width, height, size)
    f = np.float32
    out = []
    for p in (np.asarray(points, np.float32) if points is not None else []):
        x = f(f(f(p[0]) * f(rw)) / f(width)) + f(left)
        y = f(f(f(p[1]) * f(rh)) / f(height)) + f(top)
        out.append([x, y])
    return np.float32(out), (top, bottom, left, right)


def identity_perspective_points(img_size: Tuple[int, int], points) -> np.ndarray:
    """image_helper.py:120,180-188 at offset 0, angles 0, scale 1 (M = I): each point goes
    through (p - c) @ I, then x * w / (w + 0) + c in float32 -- the identity up to float32
    rounding, kept so boxes match the reference bit for bit."""
    width, height = img_size
    f = np.float32
    c = np.float32([width / 2, height / 2, 0, 0])
    out = []
    for p in np.asarray(points, np.float64):
        t = np.float32([p[0], p[1], 0, 1]) - c
        x = f(f(t[0] * f(width)) / f(f(width) + t[2])) + c[0]
        y = f(f(t[1] * f(height)) / f(f(height) + t[2])) + c[1]
        out.append([x, y])
    return np.float32(out)


def _area_weights(src: int, dst: int) -> np.ndarray:
    """[dst, src] weights of cv2 INTER_AREA along one axis: exact footprint averaging when
    shrinking; bilinear with half-pixel centres (clamped) when enlarging."""
    w = np.zeros((dst, src), np.float64)
    if dst <= src:
        scale = src / dst
        for d in range(dst):
            a, b = d * scale, (d + 1) * scale
            i0, i1 = int(np.floor(a)), min(int(np.ceil(b)), src)
            for i in range(i0, i1):
                w[d, i] = min(b, i + 1) - max(a, i)
            w[d] /= scale
    else:
        scale = src / dst
        for d in range(dst):
            x = (d + 0.5) * scale - 0.5
            x0 = int(np.floor(x))
            t = x - x0
            i0, i1 = min(max(x0, 0), src - 1), min(max(x0 + 1, 0), src - 1)
            w[d, i0] += 1 - t
            w[d, i1] += t
    return w


def resize_area(img: np.ndarray, width: int, height: int) -> np.ndarray:
    """cv2.resize(img, (width, height), interpolation=INTER_AREA) restated for uint8 HWC
    images (separable weights, round to nearest, saturate).  Parity-unpinned: cv2 absent."""
    h, w = img.shape[:2]
    wy, wx = _area_weights(h, height), _area_weights(w, width)
    x = img.astype(np.float64)
    x = x if x.ndim == 3 else x[..., None]
    out = np.einsum("yh,hwc->ywc", wy, x, optimize=True)        # rows, then columns
    out = np.einsum("ywc,xw->yxc", out, wx, optimize=True)
    out = np.clip(np.rint(out), 0, 255).astype(np.uint8)
    return out if img.ndim == 3 else out[..., 0]


def proportional_resize(img: np.ndarray, size: Tuple[int, int], points=None, bg_color=(128, 128, 128)):
    """image_helper.py:293-330 with a constant border: resized image padded to ``size``
    (width, height), the points mapped as in ``proportional_resize_points``, and the padding
    (top, bottom, left, right).  ``img`` is HWC uint8 RGB; ``bg_color`` is given in the
    reference's BGR order."""
    height, width = img.shape[:2]
    rw, rh, top, bottom, left, right = _resize_dims(width, height, size)
    small = resize_area(img, rw, rh)
    out = np.empty((size[1], size[0], img.shape[2]), np.uint8)
    out[...] = np.asarray(bg_color[::-1], np.uint8)
    out[top:top + rh, left:left + rw] = small
    pts, pad = proportional_resize_points((width, height), size, points)
    return out, pts, pad


def read_image(path: str) -> np.ndarray:
    """HWC uint8 RGB (the reference decodes BGR with cv2.imdecode and converts to RGB at
    coco_dataset_one.py:133; PIL decodes to RGB directly)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), np.uint8)


def prepare(label: Dict, image_size: Tuple[int, int], image: Optional[np.ndarray] = None,
            bg_color=(128, 128, 128)):
    """coco_dataset_one.py:74-154 with every augmentation draw at its identity.

    Returns (image float32 [h, w, 3] RGB in [0, 1], boxes float32 [n, 4] in generate_targets
    order, classes int32 [n]).  Boxes are clipped to the image and those under 2 px in either
    extent are dropped, exactly as the reference does after its resize."""
    img = read_image(label["image_path"]) if image is None else image
    pts = np.array(label["boxes"], dtype=np.float64).reshape((-1, 2))
    pts = identity_perspective_points((img.shape[1], img.shape[0]), pts)
    img, pts, _ = proportional_resize(img, image_size, pts, bg_color=bg_color)
    out = img.astype(np.float32) / 255
    boxes = pts.reshape((-1, 4))
    boxes[:, 0][boxes[:, 0] < 0] = 0
    boxes[:, 1][boxes[:, 1] < 0] = 0
    boxes[:, 2][boxes[:, 2] > image_size[0]] = image_size[0]
    boxes[:, 3][boxes[:, 3] > image_size[1]] = image_size[1]
    keep = np.logical_and(boxes[:, 2] - boxes[:, 0] >= 2, boxes[:, 3] - boxes[:, 1] >= 2)
    boxes = boxes[keep][:, [1, 0, 3, 2]]
    classes = np.array(label["classes"], dtype=np.int32)[keep]
    return out, boxes, classes


class DataGenerator:
    """coco_dataset_one.py:14-212 (the sample loop and class balancing; see module docstring
    for augmentation)."""

    def __init__(self, image_path: str, label_path: str, classes_path: str, anchors, is_train: bool = True,
                 seed: Optional[int] = None):
        self.image_path, self.label_path, self.classes_path = image_path, label_path, classes_path
        self.anchors = anchors
        self.image_size = tuple(anchors.image_size)
        self.is_train = is_train
        self.rng = random.Random(seed)
        # the augmentation noise's stream (numpy's RNG in the reference, image_helper.py:249):
        # seeded alongside rng for reproducible runs, numpy's global RNG otherwise
        self.np_rng = np.random.default_rng(seed) if seed is not None else None
        self.LoadClasses()
        self.LoadLabels()

    def LoadClasses(self):
        self.classes = load_classes(self.classes_path)
        self.classes_num = len(self.classes)

    def LoadLabels(self):
        self.labels = load_labels(self.label_path, self.image_path, self.classes)
        self.labels_num = len(self.labels)

    def get_random_data(self, label):
        return prepare(label, self.image_size)

    def generate(self) -> Iterator[Tuple[np.ndarray, np.ndarray, np.ndarray]]:
        """coco_dataset_one.py:156-212: shuffle at the start of every pass; when training,
        take images round-robin over the classes present (an image is used only when it holds
        the class whose turn it is); skip samples left without boxes."""
        yield from self._sample_order(skip_empty=True)

    def generate_labels(self) -> Iterator[Dict]:
        """The labels in generate()'s order, before get_random_data (the augmenting GetDataSet
        runs the chain itself and skips samples whose boxes vanish)."""
        return self._sample_order(skip_empty=False)

    def _sample_order(self, skip_empty: bool):
        class_list, image_classes = [], {}
        if self.is_train:
            seen = set()
            for lab in self.labels:
                s = set(lab["classes"])
                image_classes[lab["image_path"]] = list(s)
                seen |= s
            class_list = list(seen)
        n = len(self.labels)
        i, class_index = 0, 0
        order = self.labels.copy()
        while True:
            if i == 0:
                self.rng.shuffle(order)
            lab = order[i]
            if class_list and self.is_train:
                if class_list[class_index] not in image_classes[lab["image_path"]]:
                    i = (i + 1) % n
                    continue
                class_index = class_index + 1 if class_index < len(class_list) - 1 else 0
            i = (i + 1) % n
            if not skip_empty:
                yield lab
                continue
            image, boxes, classes = self.get_random_data(lab)
            if len(classes) == 0:
                continue
            yield image, boxes, classes


def collate(samples: Sequence[Tuple[np.ndarray, np.ndarray, np.ndarray]], device=None):
    """Stack a batch for ``train_step``: images [B, H, W, 3] float32 (on ``device``) and
    padded gt tensors (boxes [B, G, 4], classes [B, G], counts [B]) for
    ``Anchors.generate_targets_batched`` -- the batched form of GetDataSet's per-image
    ``anchors.generate_targets`` map (coco_dataset_one.py:229-233)."""
    B = len(samples)
    G = max(1, max(len(s[2]) for s in samples))
    gb = torch.zeros(B, G, 4, dtype=torch.float32)
    gc = torch.zeros(B, G, dtype=torch.int32)
    n = torch.zeros(B, dtype=torch.int32)
    for b, (_, boxes, cls) in enumerate(samples):
        k = len(cls)
        gb[b, :k] = torch.from_numpy(np.asarray(boxes, np.float32).reshape(-1, 4))
        gc[b, :k] = torch.from_numpy(np.asarray(cls, np.int32))
        n[b] = k
    x = torch.from_numpy(np.stack([s[0] for s in samples]))
    if device is not None:
        x = x.to(device)
    return x, gb, gc, n


def GetDataSet(image_path: str, label_path: str, classes_path: str, batch_size: int, anchors,
               is_train: bool = True, seed: Optional[int] = None, augment: bool = False, dtype: str = "f32"):
    """coco_dataset_one.py:214-246: (iterator of (images, Targets) batches, generator).

    augment=True runs the reference's random chain (blur, perspective, noise, random borders;
    augment.py + edet_augment_image on the GPU) instead of the identity chain: images are
    decoded on the host, augmented on the device straight into the batch tensor (``dtype``
    storage), and samples whose boxes all vanish are skipped as the reference skips them."""
    gen = DataGenerator(image_path, label_path, classes_path, anchors, is_train, seed)

    def batches():
        it = gen.generate()
        while True:
            samples = [next(it) for _ in range(batch_size)]
            x, gb, gc, n = collate(samples, anchors.device)
            yield x, anchors.generate_targets_batched(gb, gc, n)

    def augmented():
        from . import _lib as L
        from . import augment as AUG
        it = gen.generate_labels()
        W, H = gen.image_size
        tdt = torch.float32 if dtype == "f32" else torch.bfloat16
        while True:
            x = torch.empty((batch_size, H, W, 3), dtype=tdt, device=anchors.device)
            samples = []
            while len(samples) < batch_size:
                lab = next(it)
                r = AUG.augment_one(read_image(lab["image_path"]), lab, AUG.draw(gen.rng, gen.np_rng), (W, H), x[len(samples)],
                                    L.F32 if dtype == "f32" else L.BF16)
                if r is not None:
                    samples.append((None, r[0], r[1]))
            B = len(samples)
            G = max(1, max(len(s[2]) for s in samples))
            gb = torch.zeros(B, G, 4, dtype=torch.float32)
            gc = torch.zeros(B, G, dtype=torch.int32)
            n = torch.zeros(B, dtype=torch.int32)
            for b, (_, bx, cl) in enumerate(samples):
                gb[b, :len(cl)] = torch.from_numpy(bx)
                gc[b, :len(cl)] = torch.from_numpy(cl)
                n[b] = len(cl)
            yield x, anchors.generate_targets_batched(gb, gc, n)

    return (augmented() if augment else batches()), gen
