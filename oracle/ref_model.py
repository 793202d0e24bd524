"""torch-CPU restatement of the reference EfficientDet forward / loss / train step.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Runs in float64 by default (float32 for
the timed CPU baseline).  Layout NHWC at the interface, NCHW internally.  Parameters come as
a dict keyed by the build's parameter names (same values the GPU model holds), in the build's
storage layouts: stem [3][3][3][Co] (HWIO), 1x1 kernels [out][in], depthwise [k*k][C],
SE kernels [R][C] / [C][R].

TF semantics restated:
  SAME padding   pad_before = floor(total/2), extra at bottom/right           (A1)
  BN training    biased batch variance over N,H,W, eps 1e-3                  (A2)
  swish          x * sigmoid(x)                                              (A3)
  resize nearest half-pixel centres: src = min(floor((o+.5)*in/out), in-1)  (A4)
  SeparableConv  depthwise then pointwise, bias after pointwise              (A5)
  sigmoid CE     max(x,0) - x z + log(1 + exp(-|x|))                         (A6)
  Huber          0.5 e^2 if |e|<=d else 0.5 d^2 + d(|e|-d)                   (A7)
  Keras mean     SUM_OVER_BATCH_SIZE = sum / #elements                        (A8)
  l2_loss        sum(t^2)/2; clip_by_global_norm; SGD momentum; EMA          (A9,A10)
Reference file:line for each block is cited in the function docstrings.
"""
from __future__ import annotations

import math
import re
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as Fn


def same_pad(n, k, s):
    out = (n + s - 1) // s
    tot = max((out - 1) * s + k - n, 0)
    return tot // 2, tot - tot // 2


def conv_same(x, w, stride, groups=1):
    """x NCHW, w [Co, Ci/g, k, k]."""
    k = w.shape[-1]
    pt, pb = same_pad(x.shape[2], k, stride)
    pl, pr = same_pad(x.shape[3], k, stride)
    x = Fn.pad(x, (pl, pr, pt, pb))
    return Fn.conv2d(x, w, stride=stride, groups=groups)


def swish(x):
    return x * torch.sigmoid(x)


class BNState:
    def __init__(self):
        self.batch = {}  # name -> (mean, var_biased, count)


def batch_norm(x, p, name, training, eps, bnstate: Optional[BNState]):
    """Keras BatchNormalization on NCHW x (axis = channels)."""
    g, b = p[name + "/gamma"], p[name + "/beta"]
    if training:
        mean = x.mean(dim=(0, 2, 3))
        var = ((x - mean[None, :, None, None]) ** 2).mean(dim=(0, 2, 3))
        if bnstate is not None:
            bnstate.batch[name] = (mean.detach(), var.detach(), x.shape[0] * x.shape[2] * x.shape[3])
    else:
        mean, var = p[name + "/moving_mean"], p[name + "/moving_variance"]
    inv = 1.0 / torch.sqrt(var + eps)
    return (x - mean[None, :, None, None]) * (inv * g)[None, :, None, None] + b[None, :, None, None]


def maxpool_same(x):
    """MaxPooling2D 3x3 s2 'SAME' (resample_feature_map.py:35-38): padded cells ignored."""
    pt, pb = same_pad(x.shape[2], 3, 2)
    pl, pr = same_pad(x.shape[3], 3, 2)
    x = Fn.pad(x, (pl, pr, pt, pb), value=-math.inf)
    return Fn.max_pool2d(x, 3, 2)


def resize_nearest(x, H, W):
    """tf.image.resize(method='nearest') (resample_feature_map.py:41): half-pixel centres."""
    h, w = x.shape[2], x.shape[3]
    sy, sx = np.float32(h) / np.float32(H), np.float32(w) / np.float32(W)
    iy = [min(int(np.floor((np.float32(o) + np.float32(0.5)) * sy)), h - 1) for o in range(H)]
    ix = [min(int(np.floor((np.float32(o) + np.float32(0.5)) * sx)), w - 1) for o in range(W)]
    return x[:, :, iy][:, :, :, ix]


class RefEfficientDet:
    """Restatement of EfficientDetNet (efficientdet_net.py:10-95) + EfficientDetNetTrain."""

    def __init__(self, model_desc, params: Dict[str, np.ndarray], dtype=torch.float64):
        """model_desc: the GPU model object (used only for its *structure*: block specs,
        level sizes, BiFPN topology, head repeats — all derived from config.py, which is
        itself pinned against reference fixtures)."""
        self.m = model_desc
        self.cfg = model_desc.cfg
        self.dtype = dtype
        self.p = {k: torch.tensor(np.asarray(v), dtype=dtype) for k, v in params.items()}
        self.eps = self.cfg.batch_norm_epsilon

    # ---- parameter helpers (build layouts -> torch conv weights)
    def w1x1(self, name):  # [out][in] -> [out, in, 1, 1]
        w = self.p[name]
        return w[:, :, None, None]

    def wdw(self, name, k):  # [k*k][C] -> [C, 1, k, k]
        w = self.p[name]
        return w.t().reshape(-1, 1, k, k)

    def bn(self, x, name, training, st):
        return batch_norm(x, self.p, name, training, self.eps, st)

    # ---- layers
    def stem(self, x, training, st):
        """layers/stem.py:37-38."""
        bb = self.m.bb
        w = self.p[f"{bb}/stem/conv2d/kernel"].permute(3, 2, 0, 1)  # HWIO -> OIHW
        return swish(self.bn(conv_same(x, w, 2), f"{bb}/stem/tpu_batch_normalization", training, st))

    def mbconv(self, x, i, training, st):
        """layers/mb_conv_block.py:127-160 (no skip, no drop-connect)."""
        sp = self.m.specs[i]
        b = self.m.block_bns[i]
        pre = f"{self.m.bb}/blocks_{i}"
        if sp.expand_ratio != 1:
            x = swish(self.bn(Fn.conv2d(x, self.w1x1(b["expand_w"])), b["bn0"].name, training, st))
        k = sp.kernel_size
        x = conv_same(x, self.wdw(f"{pre}/depthwise_conv2d/depthwise_kernel", k), sp.stride, groups=x.shape[1])
        x = swish(self.bn(x, b["bn1"].name, training, st))
        # SE (layers/se.py:35-39)
        s = x.mean(dim=(2, 3), keepdim=True)
        s = Fn.conv2d(s, self.w1x1(f"{pre}/se/conv2d/kernel"), self.p[f"{pre}/se/conv2d/bias"])
        s = Fn.conv2d(swish(s), self.w1x1(f"{pre}/se/conv2d_1/kernel"), self.p[f"{pre}/se/conv2d_1/bias"])
        x = torch.sigmoid(s) * x
        return self.bn(Fn.conv2d(x, self.w1x1(b["project_w"])), b["bn2"].name, training, st)

    def resample(self, x, rr, H, training, st):
        """ResampleFeatureMap.call (resample_feature_map.py:43-52)."""
        if rr is not None and rr["conv"] is not None:
            pre = rr["conv"]
            x = Fn.conv2d(x, self.w1x1(f"{pre}/conv2d/kernel"), self.p[f"{pre}/conv2d/bias"])
            x = self.bn(x, rr["bn"].name, training, st)
        if x.shape[2] > H:
            x = maxpool_same(x)
        elif x.shape[2] < H:
            x = resize_nearest(x, H, H)
        return x

    def sepconv(self, x, pre, dwname, pwname, bname):
        x = conv_same(x, self.wdw(f"{pre}/{dwname}", 3), 1, groups=x.shape[1])
        return Fn.conv2d(x, self.w1x1(f"{pre}/{pwname}"), self.p[f"{pre}/{bname}"])

    def bifpn_cell(self, c, feats, training, st):
        """BiFPNNode.call / BiFPN.call (bifpn.py:59-67, 89-117)."""
        nodes = list(feats)
        nl = len(self.m.levels)
        outs = {}
        for j, node in enumerate(self.m.cells[c]):
            lvl = node["level"]
            H = self.m.level_hw[lvl][0]
            pre = node["prefix"]
            w = self.p[f"{pre}/WSM"]
            wsum = w.sum()
            acc = None
            for k, src in enumerate(node["inputs"]):
                r = self.resample(nodes[src], node["resample"][k], H, training, st) * w[k] / (wsum + 0.0001)
                acc = r if acc is None else acc + r
            op = f"{pre}/op_after_combine"
            y = self.sepconv(swish(acc), op, "separable_conv2d/depthwise_kernel", "separable_conv2d/pointwise_kernel",
                             "separable_conv2d/bias")
            y = self.bn(y, node["bn"].name, training, st)
            nodes.append(y)
            if j >= nl - 2:
                outs[lvl] = y
        return [outs[l] for l in self.m.levels]

    def head(self, net, feats, training, st, masks=None):
        """ClassNet.call / BoxNet.call (class_net.py:79-103, box_net.py:81-102)."""
        h = self.m.heads[net]
        surv = self.cfg.survival_prob
        out = []
        for li, lvl in enumerate(self.m.levels):
            image = feats[li]
            for i, pre in enumerate(h["convs"]):
                orig = image
                image = self.sepconv(image, pre, "depthwise_kernel", "pointwise_kernel", "bias")
                image = swish(self.bn(image, h["bns"][i][li].name, training, st))
                if i > 0 and surv:
                    if training:
                        m = masks[net][i - 1][li] if masks is not None else None
                        if m is not None:
                            image = image * torch.as_tensor(m, dtype=self.dtype)[:, None, None, None]
                    image = image + orig
            pre = h["predict"]
            c = self.sepconv(image, pre, "depthwise_kernel", "pointwise_kernel", "bias")
            B, _, H, W = c.shape
            last = h["nout"] // self.m.A
            out.append(c.permute(0, 2, 3, 1).reshape(B, H, W, self.m.A, last))
        return out

    def backbone(self, x_nhwc, training, st: Optional[BNState] = None):
        """BackboneModel.call (backbone_model.py:96-148): [features, reduction_1..5], NHWC."""
        x = torch.as_tensor(np.asarray(x_nhwc), dtype=self.dtype).permute(0, 3, 1, 2)
        x = self.stem(x, training, st)
        reds = []
        for i in range(len(self.m.specs)):
            x = self.mbconv(x, i, training, st)
            if i in self.m.red_idx:
                reds.append(x)
        return [t.permute(0, 2, 3, 1) for t in [x] + reds]

    def forward(self, x_nhwc, training, masks=None, st: Optional[BNState] = None):
        """EfficientDetNet.call: returns (boxes list, classes list) NHWC [B,H,W,A,*]."""
        x = torch.as_tensor(np.asarray(x_nhwc), dtype=self.dtype).permute(0, 3, 1, 2)
        x = self.stem(x, training, st)
        reds = []
        for i in range(len(self.m.specs)):
            x = self.mbconv(x, i, training, st)
            if i in self.m.red_idx:
                reds.append(x)
        all_feats = [x] + reds
        feats = [all_feats[l] for l in self.m.levels if l < len(all_feats)]
        for l in self.m.levels:
            if l < len(all_feats):
                continue
            feats.append(self.resample(feats[-1], self.m.resample_extra[l], self.m.level_hw[l][0], training, st))
        for c in range(self.cfg.fpn_cell_repeats):
            feats = self.bifpn_cell(c, feats, training, st)
        self.fpn_out = feats
        cls = self.head("class_net", feats, training, st, masks)
        box = self.head("box_net", feats, training, st, masks)
        return box, cls

    # ---- loss (efficientdet_net_train.py:21-52, losses/*.py)
    def l2_loss(self, weight_decay=4e-5):
        pat = re.compile(r".*(kernel|weight)$")
        return weight_decay * sum((v ** 2).sum() / 2 for k, v in self.p.items() if pat.match(k))

    def detection_loss(self, box_pred, cls_pred, y_box, y_cls_onehot, y_mask, alpha=0.25, gamma=1.5,
                       with_l2=True, npos_sum=None, count_scale=1.0):
        """_get_loss (efficientdet_net_train.py:41-52).  Data-parallel form (not in the
        reference, which trains on one device): ``npos_sum`` = the all-reduced mask count and
        ``count_scale`` = world size, so the replicas' losses sum to the global-batch loss."""
        if npos_sum is None:
            npos_sum = sum(torch.as_tensor(np.asarray(m), dtype=self.dtype).sum() for m in y_mask)
        npos = torch.as_tensor(npos_sum, dtype=self.dtype) + 1.0
        loss = self.l2_loss() if with_l2 else torch.zeros((), dtype=self.dtype)
        parts = []
        for l in range(len(box_pred)):
            yb = torch.as_tensor(np.asarray(y_box[l]), dtype=self.dtype)
            yc = torch.as_tensor(np.asarray(y_cls_onehot[l]), dtype=self.dtype)
            # BoxLoss (box_loss.py:21-30)
            mask = (yb != 0).to(self.dtype)
            e = box_pred[l] - yb
            ae = e.abs()
            hub = torch.where(ae <= 0.1, 0.5 * e ** 2, 0.5 * 0.1 ** 2 + 0.1 * (ae - 0.1))
            lb = (hub * mask).sum() / (npos * 4.0)
            # FocalLoss (focal_loss.py:26-52) + Keras SUM_OVER_BATCH_SIZE
            x = cls_pred[l]
            p = torch.sigmoid(x)
            pt = yc * p + (1 - yc) * (1 - p)
            at = yc * alpha + (1 - yc) * (1 - alpha)
            mod = (1.0 - pt) ** gamma
            ce = torch.clamp(x, min=0) - x * yc + torch.log1p(torch.exp(-x.abs()))
            lf = (at * mod * ce / npos).sum() / (x.numel() * count_scale)
            parts.append((lf.detach(), lb.detach()))
            loss = loss + lb * 50.0 + lf
        return loss, parts


def ref_train_step(ref: RefEfficientDet, x, y_box, y_cls, y_mask, masks=None, lr=0.01, momentum=0.9, clip=10.0,
                   ema_decay=0.9998, mom_state=None, ema_state=None, bn_momentum=0.99):
    """train_step_normal (efficientdet_net_train.py:112-132) + SGD momentum + EMA + BN moving
    update.  Returns (loss, gnorm, new_params dict, grads dict, bnstate)."""
    for v in ref.p.values():
        v.requires_grad_(False)
    train_keys = [k for k in ref.p if not (k.endswith("/moving_mean") or k.endswith("/moving_variance"))]
    for k in train_keys:
        ref.p[k].requires_grad_(True)
    st = BNState()
    box, cls = ref.forward(x, True, masks, st)
    loss, parts = ref.detection_loss(box, cls, y_box, y_cls, y_mask)
    grads = torch.autograd.grad(loss, [ref.p[k] for k in train_keys], allow_unused=True)
    grads = {k: (g if g is not None else torch.zeros_like(ref.p[k])) for k, g in zip(train_keys, grads)}
    gnorm = torch.sqrt(sum((g ** 2).sum() for g in grads.values()))
    scale = clip / max(float(gnorm), clip)
    new = {}
    mom_state = mom_state if mom_state is not None else {k: torch.zeros_like(ref.p[k]) for k in train_keys}
    for k in train_keys:
        g = grads[k] * scale
        v = momentum * mom_state[k] - lr * g
        new[k] = (ref.p[k].detach() + v)
        mom_state[k] = v
    for name, (mean, var, cnt) in st.batch.items():
        unb = var * cnt / max(cnt - 1, 1)
        mm, mv = ref.p[name + "/moving_mean"], ref.p[name + "/moving_variance"]
        new[name + "/moving_mean"] = mm - (mm - mean) * (1 - bn_momentum)
        new[name + "/moving_variance"] = mv - (mv - unb) * (1 - bn_momentum)
    return loss.detach(), gnorm.detach(), new, {k: g.detach() for k, g in grads.items()}, st, parts
