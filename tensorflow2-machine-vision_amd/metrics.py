"""Per-image mAP of the reference's evaluation step (host numpy, like the reference).

Restates ``AIServer/ai_api/ai_models/utils/mAP.py`` (``Get_TPFP`` :3-64, ``Get_AP`` :66-101,
``Get_mAP`` :103-110, ``Get_mAP_one`` :114-126), which ``EfficientDetNetTrain.test_step``
(efficientdet_net_train.py:160-167) calls through ``tf.numpy_function`` once per image.  The
arithmetic and its quirks are kept so the metric matches the reference number for number:

  * one TP per ground truth: the prediction with the highest IoU for that ground truth
    (np.argmax, first maximum) becomes TP if that IoU >= thresh;
  * rows sorted by score with ``np.argsort(...)[::-1]`` (ties: reverse of argsort order);
  * the precision list goes into ``mrec`` and the recall list into ``mpre`` (the reference's
    variable names are swapped; the envelope and the area are computed on them as written);
  * every class id in [0, class_num) is averaged, the background class 0 included.

``np.float`` in the reference is the builtin float (float64).
"""
from __future__ import annotations

import numpy as np


def get_tpfp(data, class_id, thresh=0.5):
    tp = []
    gt_num = 0
    for d in data:
        gt = np.array(d["groud_truth"], dtype=np.float64).reshape(-1, 5)
        gt = gt[gt[..., 4] == class_id]
        gt = np.expand_dims(gt, axis=0)
        gt_num += gt.shape[1]
        pred = np.array(d["prediction"], dtype=np.float64).reshape(-1, 6)
        pred = pred[pred[..., 4] == class_id]
        pred = np.expand_dims(pred, axis=1)
        if gt.shape[1] == 0 or pred.shape[0] == 0:
            continue
        gt_min, gt_max = gt[..., 0:2], gt[..., 2:4]
        gt_wh = gt_max - gt_min
        p_min, p_max = pred[..., 0:2], pred[..., 2:4]
        p_wh = p_max - p_min
        i_wh = np.maximum(np.minimum(gt_max, p_max) - np.maximum(gt_min, p_min), 0.0)
        inter = i_wh[..., 0] * i_wh[..., 1]
        iou = inter / (gt_wh[..., 0] * gt_wh[..., 1] + p_wh[..., 0] * p_wh[..., 1] - inter)
        tp_one = np.zeros((pred.shape[0],))
        best = np.argmax(iou, axis=0)
        for i in range(best.shape[0]):
            if iou[best[i], i] >= thresh:
                tp_one[best[i]] = 1
        tp.append(np.concatenate([tp_one[:, None], pred[:, 0, 5:6]], axis=-1))
    tp = np.concatenate(tp, 0) if tp else np.zeros((0, 2))
    tp = tp[np.argsort(tp[:, 1])[::-1], :]
    return tp, gt_num


def get_ap(data, class_id, thresh=0.5):
    tp, gt_num = get_tpfp(data, class_id, thresh)
    precision, recall = [], []
    tp_sum = 0.0
    for i in range(tp.shape[0]):
        if tp[i][0] == 1:
            tp_sum += 1.0
        precision.append(tp_sum / (i + 1))
        recall.append(tp_sum / gt_num)
    mrec = np.concatenate(([0.0], precision, [1.0]))
    mpre = np.concatenate(([0.0], recall, [0.0]))
    for i in range(mpre.size - 1, 0, -1):
        mpre[i - 1] = np.maximum(mpre[i - 1], mpre[i])
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return float(np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1]))


def get_map(data, class_num, thresh=0.5):
    return sum(get_ap(data, c, thresh) for c in range(class_num)) / class_num


def get_map_one(ground_truth, prediction, class_num, thresh=0.5):
    """ground_truth [[y1, x1, y2, x2, class]], prediction [[y1, x1, y2, x2, class, score]]."""
    return get_map([{"image_path": "*.jpg", "groud_truth": ground_truth, "prediction": prediction}], class_num, thresh)
