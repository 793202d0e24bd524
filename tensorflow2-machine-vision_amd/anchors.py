"""Anchors: generation, training targets and decoding on the GPU.

Mirrors ``efficientnet/utils/anchors.py:12`` (``Anchors``): same constructor arguments, same
per-level box tensors ``[H, W, A, 4]`` in (y1, x1, y2, x2) pixels, anchor index
``octave * len(aspect_ratios) + aspect``.  The heavy per-anchor work runs in
libedet (csrc/anchors.hip) and is bit-exact with the reference's fp32 op sequence.

Training targets are produced in the compact pyramid layout the loss kernel consumes
(``Targets``); ``Targets.from_reference`` converts the reference's per-level
(boxes, one-hot classes, masks) tuples.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple, Union

import numpy as np
import torch

from . import _lib as L
from .config import get_feat_sizes
from .runtime import Pyr, memcpy, memset0, stream, vp


def anchor_half_sizes(image_size, feat_sizes, level, num_scales, aspect_ratios, anchor_scale):
    """(half_y, half_x) per anchor in python float64 exactly as anchors.py:58-67 computes them,
    rounded to fp32 where the reference hands them to TF."""
    stride = (feat_sizes[0][0] / float(feat_sizes[level][0]), feat_sizes[0][1] / float(feat_sizes[level][1]))
    halves = []
    for octave in range(num_scales):
        for aspect in aspect_ratios:
            octave_scale = octave / float(num_scales)
            base_x = anchor_scale * stride[1] * 2 ** octave_scale
            base_y = anchor_scale * stride[0] * 2 ** octave_scale
            halves.append((base_y * aspect[0] / 2.0, base_x * aspect[1] / 2.0))
    return stride, np.asarray(halves, np.float32)


def _pyramid_base(levels, pyr: Pyr):
    """(base pointer, row stride in elements, dtype code) of per-level [B,H,W,A,k] views that
    share one pyramid buffer [rows][ld] (what EfficientDetNet.call and convert_outputs_boxes
    return)."""
    lv = levels[0]
    # row stride from the first dimension of size > 1 (torch reports nominal strides for
    # size-1 dimensions, e.g. the 1x1 top level)
    ld = lv.stride(2) if lv.shape[2] > 1 else lv.stride(1) if lv.shape[1] > 1 else lv.stride(0)
    for s, v in enumerate(levels):  # the views must really be segments of one buffer
        assert v.untyped_storage().data_ptr() == lv.untyped_storage().data_ptr()
        assert v.storage_offset() - lv.storage_offset() == (pyr.row_off[s] - pyr.row_off[0]) * ld
    base = lv.untyped_storage().data_ptr()
    ptr = base + (lv.storage_offset() - pyr.row_off[0] * ld) * lv.element_size()
    return ptr, ld, (L.BF16 if lv.dtype == torch.bfloat16 else L.F32)


class Targets:
    """Compact training targets in pyramid row layout (rows = the heads' pyramid rows)."""

    def __init__(self, pyr: Pyr, A: int, device):
        self.pyr, self.A = pyr, A
        self.box = torch.empty((pyr.rows, A, 4), dtype=torch.float32, device=device)
        self.cls = torch.empty((pyr.rows, A), dtype=torch.int32, device=device)
        self.mask = torch.empty((pyr.rows, A), dtype=torch.uint8, device=device)

    @staticmethod
    def from_reference(y_true_boxes, y_true_classes, y_true_masks, pyr: Pyr, A: int, device) -> "Targets":
        """Convert (boxes [B,H,W,A,4], one-hot classes [B,H,W,A,C], masks [B,H,W,A,1]) per level."""
        t = Targets(pyr, A, device)
        for s in range(pyr.nseg):
            sl = pyr.seg_slice(s)
            b = y_true_boxes[s].to(device=device, dtype=torch.float32).contiguous()
            c = y_true_classes[s].to(device=device, dtype=torch.float32).contiguous()
            m = y_true_masks[s].to(device=device).contiguous()
            if m.dtype != torch.uint8 and m.dtype != torch.bool:
                m = (m != 0)
            memcpy(t.box[sl], b)
            memcpy(t.mask[sl], m.view(torch.uint8) if m.dtype == torch.bool else m)
            n = pyr.seg_rows(s) * A
            L.call("edet_onehot_to_index", vp(c), n, c.shape[-1], vp(t.cls[sl]), stream())
        return t


class Anchors:
    def __init__(self, min_level: int, max_level: int, image_size: Tuple[int, int], num_scales: int,
                 aspect_ratios: Sequence[Tuple[float, float]], anchor_scale: Union[float, List[float]],
                 device="cuda"):
        self.min_level, self.max_level = min_level, max_level
        self.image_size = tuple(image_size)
        self.num_scales = num_scales
        self.aspect_ratios = list(aspect_ratios)
        self.anchor_scale = anchor_scale
        if isinstance(anchor_scale, (list, tuple)):
            assert len(anchor_scale) == max_level - min_level + 1
            self.anchor_scales = list(anchor_scale)
        else:
            self.anchor_scales = [anchor_scale] * (max_level - min_level + 1)
        self.device = torch.device(device)
        self.feat_sizes = get_feat_sizes(self.image_size, self.max_level)
        self.boxes = self._generate_boxes()
        self.flat = torch.cat([b.reshape(-1, 4) for b in self.boxes], 0) if len(self.boxes) > 1 else self.boxes[0].reshape(-1, 4)

    def get_anchors_per_location(self) -> int:
        return self.num_scales * len(self.aspect_ratios)

    @property
    def level_sizes(self):
        return [self.feat_sizes[l] for l in range(self.min_level, self.max_level + 1)]

    def _generate_boxes(self) -> List[torch.Tensor]:
        A = self.get_anchors_per_location()
        out = []
        for level in range(self.min_level, self.max_level + 1):
            stride, halves = anchor_half_sizes(self.image_size, self.feat_sizes, level, self.num_scales,
                                               self.aspect_ratios, self.anchor_scales[level - self.min_level])
            fh, fw = self.feat_sizes[level]
            # tf.range(stride/2, size, stride): the start/delta are converted to fp32
            sy, dy = np.float32(stride[0] / 2), np.float32(stride[0])
            sx, dx = np.float32(stride[1] / 2), np.float32(stride[1])
            ny = int(np.ceil(np.abs((np.float32(self.image_size[0]) - sy) / dy)))
            nx = int(np.ceil(np.abs((np.float32(self.image_size[1]) - sx) / dx)))
            assert (ny, nx) == (fh, fw), f"tf.range length {ny}x{nx} != feature size {fh}x{fw}"
            half = torch.from_numpy(halves).to(self.device)
            boxes = torch.empty((fh, fw, A, 4), dtype=torch.float32, device=self.device)
            L.call("edet_anchor_boxes", fh, fw, float(sy), float(dy), float(sx), float(dx), A, vp(half), vp(boxes),
                   stream())
            out.append(boxes)  # `half` is released stream-ordered by the caching allocator
        return out

    def pyramid(self, batch: int) -> Pyr:
        return Pyr(batch, self.level_sizes)

    def generate_targets_batched(self, gt_boxes: torch.Tensor, gt_classes: torch.Tensor, n_gt: torch.Tensor,
                                 iou_threshold: float = 0.5, pyr: Pyr = None) -> Targets:
        """gt_boxes [B, G, 4] (y1,x1,y2,x2 pixels), gt_classes [B, G] int, n_gt [B] valid counts."""
        B, G = gt_boxes.shape[0], gt_boxes.shape[1]
        pyr = pyr or self.pyramid(B)
        A = self.get_anchors_per_location()
        t = Targets(pyr, A, self.device)
        if pyr.rows != sum(pyr.seg_rows(s) for s in range(pyr.nseg)):
            memset0(t.box); memset0(t.cls); memset0(t.mask)  # padding rows between levels
        gb = gt_boxes.to(self.device, torch.float32).contiguous()
        gc = gt_classes.to(self.device, torch.int32).contiguous()
        ng = n_gt.to(self.device, torch.int32).contiguous()
        L.call("edet_generate_targets", vp(self.flat), pyr.c, A, vp(gb), vp(gc), vp(ng), max(G, 1),
               float(iou_threshold), vp(t.box), vp(t.cls), vp(t.mask), stream())
        return t

    def generate_targets(self, boxes: torch.Tensor, classes: torch.Tensor, classes_num: int, iou_threshold=0.5):
        """Per-image form of anchors.py:91-138: returns per-level (boxes [H,W,A,4],
        one-hot classes [H,W,A,classes_num], masks [H,W,A,1] bool)."""
        boxes = torch.as_tensor(boxes, dtype=torch.float32, device=self.device).reshape(-1, 4)
        classes = torch.as_tensor(classes, device=self.device).reshape(-1)
        n = boxes.shape[0]
        t = self.generate_targets_batched(boxes[None], classes[None].to(torch.int32),
                                          torch.tensor([n], dtype=torch.int32), iou_threshold)
        A = t.A
        ob, oc, om = [], [], []
        for s, (fh, fw) in enumerate(self.level_sizes):
            sl = t.pyr.seg_slice(s)
            ob.append(t.box[sl].reshape(fh, fw, A, 4))
            # one-hot expansion is a data-format conversion for API compatibility (not hot path)
            oc.append(torch.nn.functional.one_hot(t.cls[sl].long(), classes_num).float().reshape(fh, fw, A, classes_num))
            om.append(t.mask[sl].bool().reshape(fh, fw, A, 1))
        return tuple(ob), tuple(oc), tuple(om)

    def convert_outputs_boxes(self, outputs_boxes, pyr: Pyr = None, ld: int = None, dtype=None):
        """Decode [ty, tx, th, tw] per level to (y1, x1, y2, x2) (anchors.py:141-158, :245-274).

        ``outputs_boxes`` is either a tuple of per-level [B,H,W,A,4] tensors sharing one
        pyramid buffer (as returned by EfficientDetNet.call) or a raw [rows, ld] buffer."""
        A = self.get_anchors_per_location()
        if isinstance(outputs_boxes, (tuple, list)):
            pyr = pyr or self.pyramid(outputs_boxes[0].shape[0])
            raw_ptr, ld, dt = _pyramid_base(outputs_boxes, pyr)
        else:
            raw_ptr = outputs_boxes.data_ptr()
            dt = L.BF16 if outputs_boxes.dtype == torch.bfloat16 else L.F32
        out = torch.empty((pyr.rows, A, 4), dtype=torch.float32, device=self.device)
        L.call("edet_decode_boxes", dt, vp(self.flat), pyr.c, A, raw_ptr, ld, vp(out), stream())
        res = []
        for s, (fh, fw) in enumerate(self.level_sizes):
            res.append(out[pyr.seg_slice(s)].view(pyr.batch, fh, fw, A, 4))
        return tuple(res)

    def detect(self, outputs_boxes, outputs_classes, max_output_size: int = 200, iou_threshold: float = 0.5,
               score_threshold: float = 0.0001):
        """convert_outputs_one (anchors.py:161-202 + nms.py:5-61) for every image of the batch,
        one GPU launch: first-argmax class != 0, DIoU-NMS on the logits, sigmoid scores.

        outputs_boxes: decoded per-level boxes (convert_outputs_boxes); outputs_classes:
        per-level logits [B,H,W,A,NC] as returned by EfficientDetNet.call.  Returns
        (boxes [B,max,4], class ids [B,max], scores [B,max], counts [B]); rows past counts[b]
        are unspecified."""
        B = outputs_classes[0].shape[0]
        NC = outputs_classes[0].shape[-1]
        A = self.get_anchors_per_location()
        pyr = self.pyramid(B)
        bptr, bld, bdt = _pyramid_base(outputs_boxes, pyr)
        assert bdt == L.F32 and bld == 4 * A, "outputs_boxes must be decoded fp32 boxes"
        cptr, cld, cdt = _pyramid_base(outputs_classes, pyr)
        N = sum(h * w for h, w in self.level_sizes) * A
        dev = self.device
        scratch = torch.empty(2 * B * N, dtype=torch.float32, device=dev)
        ob = torch.empty((B, max_output_size, 4), dtype=torch.float32, device=dev)
        oc = torch.empty((B, max_output_size), dtype=torch.int32, device=dev)
        os_ = torch.empty((B, max_output_size), dtype=torch.float32, device=dev)
        cnt = torch.empty(B, dtype=torch.int32, device=dev)
        L.call("edet_detect_nms", cdt, bptr, cptr, cld, pyr.c, A, NC, max_output_size, float(iou_threshold),
               float(score_threshold), vp(scratch), vp(ob), vp(oc), vp(os_), vp(cnt), stream())
        return ob, oc, os_, cnt

    def convert_outputs_one(self, batch_index: int, outputs_boxes, outputs_classes):
        """anchors.py:161-202 signature: (boxes [k,4], class ids [k], scores [k]) of one image."""
        ob, oc, os_, cnt = self.detect(outputs_boxes, outputs_classes)
        k = int(cnt[batch_index])
        return ob[batch_index, :k], oc[batch_index, :k].long(), os_[batch_index, :k]
