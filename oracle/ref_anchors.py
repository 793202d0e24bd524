"""numpy fp32 restatement of efficientnet/utils/anchors.py + iou.py (TEST INFRASTRUCTURE ONLY).

Each function follows the reference op sequence in float32 (numpy performs IEEE fp32 ops
without FMA contraction, like TF's CPU kernels):
  generate_boxes   anchors.py:47-84    (tf.range: fp32 accumulation start, start+delta, ...)
  iou              iou.py:27-69        ('iou' type, divide_no_nan)
  diou             iou.py:85-95
  generate_targets anchors.py:91-138   (argmax first-max, >= threshold, encode, one-hot)
  encode           anchors.py:219-243
  decode           anchors.py:245-274
  get_nms          nms.py:5-61         (sort + boolean_mask greedy loop, DIoU)
  convert_outputs_one anchors.py:161-202
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
EPSILON = f32(1e-8)


def feat_sizes(image_size, max_level):
    """get_feat_sizes.py:4-21."""
    h, w = image_size
    out = [(h, w)]
    for _ in range(max_level):
        h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        out.append((h, w))
    return out


def tf_range_f32(start, limit, delta):
    start, limit, delta = f32(start), f32(limit), f32(delta)
    n = int(np.ceil(np.abs((limit - start) / delta)))
    out = np.empty(n, f32)
    v = start
    for i in range(n):
        out[i] = v
        v = f32(v + delta)
    return out


def generate_boxes(min_level, max_level, image_size, num_scales, aspect_ratios, anchor_scale):
    fs = feat_sizes(image_size, max_level)
    scales = anchor_scale if isinstance(anchor_scale, (list, tuple)) else [anchor_scale] * (max_level - min_level + 1)
    out = []
    for level in range(min_level, max_level + 1):
        per = []
        for octave in range(num_scales):
            for aspect in aspect_ratios:
                stride = (fs[0][0] / float(fs[level][0]), fs[0][1] / float(fs[level][1]))
                octave_scale = octave / float(num_scales)
                sc = scales[level - min_level]
                bx = sc * stride[1] * 2 ** octave_scale
                by = sc * stride[0] * 2 ** octave_scale
                hx = f32(bx * aspect[1] / 2.0)
                hy = f32(by * aspect[0] / 2.0)
                x = tf_range_f32(stride[1] / 2, image_size[1], stride[1])
                y = tf_range_f32(stride[0] / 2, image_size[0], stride[0])
                xv, yv = np.meshgrid(x, y)
                b = np.stack([yv - hy, xv - hx, yv + hy, xv + hx], -1).astype(f32)
                per.append(b[:, :, None, :])
        out.append(np.concatenate(per, axis=-2))
    return out


def iou(b1, b2):
    b1 = np.asarray(b1, f32)
    b2 = np.asarray(b2, f32)
    zero = f32(0)
    b1_w = np.maximum(zero, b1[..., 3] - b1[..., 1])
    b1_h = np.maximum(zero, b1[..., 2] - b1[..., 0])
    b2_w = np.maximum(zero, b2[..., 3] - b2[..., 1])
    b2_h = np.maximum(zero, b2[..., 2] - b2[..., 0])
    a1 = b1_w * b1_h
    a2 = b2_w * b2_h
    iy1 = np.maximum(b1[..., 0], b2[..., 0])
    ix1 = np.maximum(b1[..., 1], b2[..., 1])
    iy2 = np.minimum(b1[..., 2], b2[..., 2])
    ix2 = np.minimum(b1[..., 3], b2[..., 3])
    inter = np.maximum(zero, ix2 - ix1) * np.maximum(zero, iy2 - iy1)
    union = a1 + a2 - inter
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(union == 0, zero, inter / np.where(union == 0, f32(1), union))
    return r.astype(f32)


def diou(b1, b2):
    b1 = np.asarray(b1, f32)
    b2 = np.asarray(b2, f32)
    v = iou(b1, b2)
    ey1 = np.minimum(b1[..., 0], b2[..., 0]); ex1 = np.minimum(b1[..., 1], b2[..., 1])
    ey2 = np.maximum(b1[..., 2], b2[..., 2]); ex2 = np.maximum(b1[..., 3], b2[..., 3])
    c1 = np.stack([(b1[..., 0] + b1[..., 2]) / f32(2), (b1[..., 1] + b1[..., 3]) / f32(2)], -1)
    c2 = np.stack([(b2[..., 0] + b2[..., 2]) / f32(2), (b2[..., 1] + b2[..., 3]) / f32(2)], -1)
    # iou.py:91-96: tf.linalg.norm = sqrt(sum of squares), then **2
    e = np.sqrt(np.sum((c2 - c1) * (c2 - c1), -1, dtype=f32))
    diag = np.stack([ey2 - ey1, ex2 - ex1], -1)
    d = np.sqrt(np.sum(diag * diag, -1, dtype=f32))
    e2, d2 = e * e, d * d
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(d2 == 0, f32(0), e2 / np.where(d2 == 0, f32(1), d2))
    return (v - r).astype(f32)


def _center_size(b):
    yc = (b[..., 2] + b[..., 0]) / f32(2.0)
    xc = (b[..., 3] + b[..., 1]) / f32(2.0)
    h = b[..., 2] - b[..., 0]
    w = b[..., 3] - b[..., 1]
    return yc, xc, h, w


def encode(anchors, boxes):
    ya, xa, ha, wa = _center_size(np.asarray(anchors, f32))
    y, x, h, w = _center_size(np.asarray(boxes, f32))
    ha, wa, h, w = (np.maximum(EPSILON, t) for t in (ha, wa, h, w))
    tx = (x - xa) / wa
    ty = (y - ya) / ha
    tw = np.log(w / wa)
    th = np.log(h / ha)
    return np.stack([ty, tx, th, tw], -1).astype(f32)


def decode(anchors, rel):
    ya, xa, ha, wa = _center_size(np.asarray(anchors, f32))
    rel = np.asarray(rel, f32)
    ty, tx, th, tw = rel[..., 0], rel[..., 1], rel[..., 2], rel[..., 3]
    w = np.exp(tw) * wa
    h = np.exp(th) * ha
    yc = ty * ha + ya
    xc = tx * wa + xa
    return np.stack([yc - h / f32(2), xc - w / f32(2), yc + h / f32(2), xc + w / f32(2)], -1).astype(f32)


def generate_targets(anchor_levels, boxes, classes, classes_num, iou_threshold=0.5):
    """Per image: returns per level (boxes [H,W,A,4], one-hot [H,W,A,C], mask [H,W,A,1], class idx)."""
    boxes = np.asarray(boxes, f32).reshape(-1, 4)
    classes = np.asarray(classes).reshape(-1)
    ob, oc, om, oi = [], [], [], []
    for anc in anchor_levels:
        H, W, A, _ = anc.shape
        if boxes.shape[0] == 0:
            mask = np.zeros((H, W, A), bool)
            idx = np.zeros((H, W, A), np.int64)
        else:
            v = iou(anc[:, :, :, None, :], boxes[None, None, None, :, :])  # [H,W,A,N]
            idx = np.argmax(v, -1)  # first max
            mask = np.max(v, -1) >= f32(iou_threshold)
        if boxes.shape[0]:
            enc = encode(anc, boxes[idx])
            cls = classes[idx]
        else:
            enc = np.zeros((H, W, A, 4), f32)
            cls = np.zeros((H, W, A), np.int64)
        enc = np.where(mask[..., None], enc, f32(0)).astype(f32)
        cls = np.where(mask, cls, 0).astype(np.int64)
        ob.append(enc)
        oc.append(np.eye(classes_num, dtype=f32)[cls])
        om.append(mask[..., None])
        oi.append(cls.astype(np.int32))
    return ob, oc, om, oi


def get_nms(boxes, scores, max_output_size, iou_threshold=0.5, score_threshold=float("-inf")):
    """nms.py:5-61, literally: indices sorted by descending score (tf.argsort DESCENDING: ties
    keep the lower index first), then repeatedly keep the head and drop the rest whose DIoU
    with it is >= iou_threshold; stop at max_output_size, an empty list or a head score below
    score_threshold."""
    boxes = np.asarray(boxes, f32)
    scores = np.asarray(scores, f32)
    order = np.argsort(-scores, kind="stable")
    boxes_sort, idxs = boxes[order], order
    result = []
    while True:
        if len(result) >= max_output_size or len(idxs) == 0:
            break
        top = idxs[0]
        if scores[top] < f32(score_threshold):
            break
        result.append(int(top))
        if len(idxs) == 1:
            break
        keep = diou(boxes_sort[0:1], boxes_sort[1:]) < f32(iou_threshold)
        boxes_sort, idxs = boxes_sort[1:][keep], idxs[1:][keep]
    return np.asarray(result, np.int64)


def convert_outputs_one(level_boxes, level_logits, max_output_size=200, iou_threshold=0.5,
                        score_threshold=0.0001):
    """anchors.py:161-202 for one image: per level argmax class / max logit over [H,W,A],
    drop class 0, concatenate levels, DIoU-NMS on the logits, sigmoid of the kept scores.
    level_boxes: decoded [H,W,A,4]; level_logits: [H,W,A,NC]."""
    nb, nc, ns = [], [], []
    for b, lg in zip(level_boxes, level_logits):
        lg = np.asarray(lg, f32).reshape(-1, np.shape(lg)[-1])
        cid = np.argmax(lg, -1)
        sc = np.max(lg, -1)
        m = cid != 0
        nb.append(np.asarray(b, f32).reshape(-1, 4)[m])
        nc.append(cid[m])
        ns.append(sc[m])
    nb, nc, ns = np.concatenate(nb), np.concatenate(nc), np.concatenate(ns)
    idx = get_nms(nb, ns, max_output_size, iou_threshold, score_threshold)
    s = ns[idx]
    return nb[idx], nc[idx], (f32(1) / (f32(1) + np.exp(-s))).astype(f32)
