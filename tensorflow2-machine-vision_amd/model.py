"""EfficientDet on MI355X: drop-in for the reference's call()/train_step() surface.

Reference (AIServer/ai_api/ai_models/):
  efficientnet/backbone_model.py:12-148     BackboneModel            -> _backbone()
  layers/stem.py, layers/mb_conv_block.py, layers/se.py             -> _stem(), _mbconv()
  layers/resample_feature_map.py, layers/bifpn.py                   -> _resample(), _bifpn_cell()
  layers/class_net.py, layers/box_net.py                            -> _head()
  efficientnet/efficientdet_net.py:10-95    EfficientDetNet.call     -> EfficientDetNet.call
  efficientnet/efficientdet_net_train.py    EfficientDetNetTrain     -> EfficientDetNetTrain
      _reg_l2_loss :21-28, _get_loss :41-52, train_step_normal :112-132

Surface kept: ``EfficientDetNet(blocks_args, global_params)``, ``call(inputs, training)``
returning ``(boxes, classes)`` — boxes first — as per-level tuples of
``[B, H_l, W_l, A, 4]`` / ``[B, H_l, W_l, A, num_classes]`` views (compute dtype), anchor-major
channel packing; ``backbone(inputs, training)`` returning ``[features, r1..r5]``-style
feature list; ``EfficientDetNetTrain(blocks_args, global_params, anchors).train_step(data)``
with ``data = (x, y_true_boxes[5], y_true_classes[5], y_true_masks[5])`` (or
``(x, Targets)``) returning ``{'loss': f32[], 'gnorm': f32[]}`` (device scalars).
Inputs are NHWC torch tensors on the GPU, values in [0, 1] like the reference's /255 data.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L
from . import ops
from .anchors import Anchors, Targets
from .config import (BlockSpec, Config, efficientnet_b0_blocks, expand_blocks, get_efficientdet_config,
                     get_feat_sizes, round_filters)
from .runtime import Act, BNParam, Engine, ParamStore, Pyr, Tape, memset0, memset0_many, round_up, stream, vp

CLS_LD_PAD = 8  # class / box logits row stride padded to a multiple of 8 in training



# the SE-gated depthwise output is materialised for project convs of at least this many output
# channels (0 = all); narrower ones read it lazily (EDET_MATERIALIZE_SE_MIN_N, same-box A/B)
MATERIALIZE_SE_MIN_N = int(os.environ.get("EDET_MATERIALIZE_SE_MIN_N", "0"))

class EfficientDetNet:
    def __init__(self, blocks_args=None, global_params: Optional[Config] = None, name: str = "",
                 dtype: str = "bf16", device="cuda", seed: int = 0):
        self.cfg = global_params if global_params is not None else get_efficientdet_config("efficientdet-d0")
        self.blocks_args = blocks_args if blocks_args is not None else efficientnet_b0_blocks()
        if not isinstance(self.blocks_args, list):
            raise ValueError("blocks_args should be a list.")
        self.name = name
        self.eng = Engine(dtype, device)
        self.P = ParamStore()
        cfg = self.cfg
        self.A = len(cfg.aspect_ratios) * cfg.num_scales
        self.NC = cfg.num_classes
        self.F = cfg.fpn_num_filters
        self.levels = list(range(cfg.min_level, cfg.max_level + 1))
        self.specs: List[BlockSpec] = expand_blocks(self.blocks_args, cfg)
        self._register()
        self.P.finalize(self.eng.device, self.eng.tdtype, seed)
        self._count_batch = None
        self.last_outputs = None
        # SE-gated depthwise outputs written once before the project conv (ops.materialize)
        self.materialize_se = True
        # inference: SE squeeze in the depthwise epilogue (edet_dwconv_fwd_squeeze)
        self.fused_squeeze = True

    # ------------------------------------------------------------------ parameters
    def _register(self):
        cfg, P = self.cfg, self.P
        mom, eps = cfg.batch_norm_momentum, cfg.batch_norm_epsilon
        S = cfg.image_size
        sizes = get_feat_sizes((S, S), cfg.max_level)
        bb = cfg.backbone_name or "backbone"
        self.bb = bb
        cs = round_filters(self.blocks_args[0].input_filters, cfg.width_coefficient, cfg.depth_divisor)
        self.stem_c = cs
        P.add(f"{bb}/stem/conv2d/kernel", (3, 3, 3, cs), ("normal", math.sqrt(2.0 / (9 * cs))), True)
        self.stem_bn = P.add_bn(f"{bb}/stem/tpu_batch_normalization", cs, mom, eps)
        self.stem_bn.hw = sizes[1][0] * sizes[1][1]
        # blocks
        self.block_bns = []
        hw = sizes[1]
        for sp in self.specs:
            pre = f"{bb}/blocks_{sp.index}"
            bns = {}
            bn_id = iter(["tpu_batch_normalization", "tpu_batch_normalization_1", "tpu_batch_normalization_2"])
            conv_id = iter(["conv2d", "conv2d_1"])
            e = sp.expanded_filters
            if sp.expand_ratio != 1:
                n = next(conv_id)
                P.add(f"{pre}/{n}/kernel", (e, sp.input_filters), ("normal", math.sqrt(2.0 / e)), True, pw=True)
                bns["expand_w"] = f"{pre}/{n}/kernel"
                bns["bn0"] = P.add_bn(f"{pre}/{next(bn_id)}", e, mom, eps)
                bns["bn0"].hw = hw[0] * hw[1]
            k = sp.kernel_size
            P.add(f"{pre}/depthwise_conv2d/depthwise_kernel", (k * k, e), ("normal", math.sqrt(2.0 / (k * k))), True)
            hw = ((hw[0] + sp.stride - 1) // sp.stride, (hw[1] + sp.stride - 1) // sp.stride)
            bns["bn1"] = P.add_bn(f"{pre}/{next(bn_id)}", e, mom, eps)
            bns["bn1"].hw = hw[0] * hw[1]
            R = sp.se_filters
            P.add(f"{pre}/se/conv2d/kernel", (R, e), ("normal", math.sqrt(2.0 / R)), True)
            P.add(f"{pre}/se/conv2d/bias", (R,), ("const", 0.0), False)
            P.add(f"{pre}/se/conv2d_1/kernel", (e, R), ("normal", math.sqrt(2.0 / e)), True)
            P.add(f"{pre}/se/conv2d_1/bias", (e,), ("const", 0.0), False)
            n = next(conv_id)
            P.add(f"{pre}/{n}/kernel", (sp.output_filters, e), ("normal", math.sqrt(2.0 / sp.output_filters)), True,
                  pw=True)
            bns["project_w"] = f"{pre}/{n}/kernel"
            bns["bn2"] = P.add_bn(f"{pre}/{next(bn_id)}", sp.output_filters, mom, eps)
            bns["bn2"].hw = hw[0] * hw[1]
            bns["out_hw"] = hw
            self.block_bns.append(bns)
        # reductions (backbone_model.py:119-139)
        self.red_idx = []
        for i, sp in enumerate(self.specs):
            if i == len(self.specs) - 1 or self.specs[i + 1].stride > 1:
                self.red_idx.append(i)
        # feats P_min..P5 from the backbone; extra levels by ResampleFeatureMap
        bb_levels = [l for l in self.levels if l < len(self.red_idx) + 1]
        self.feat_channels = {}
        for l in bb_levels:
            self.feat_channels[l] = self.specs[self.red_idx[l - 1]].output_filters
        F = self.F
        self.level_hw = {l: sizes[l] for l in self.levels}
        self.level_hw_input = sizes[0]
        self.resample_extra = {}
        prev_c = self.feat_channels[bb_levels[-1]]
        for l in self.levels:
            if l in self.feat_channels:
                continue
            pre = f"resample_p{l}"
            rec = {"conv": None}
            if prev_c != F:
                P.add(f"{pre}/conv2d/kernel", (F, prev_c), ("glorot", prev_c, F), True, pw=True)
                P.add(f"{pre}/conv2d/bias", (F,), ("const", 0.0), False)
                rec["conv"] = pre
                rec["bn"] = P.add_bn(f"{pre}/bn", F, mom, eps)
                rec["bn"].hw = sizes[l - 1][0] * sizes[l - 1][1]
            self.resample_extra[l] = rec
            prev_c = F
        # BiFPN cells (bifpn.py:69-117)
        nl = len(self.levels)
        self.node_defs = []  # (level index into self.levels, [input node ids])
        for i in range(nl - 2, 0, -1):   # top-down: P6'..P4'
            self.node_defs.append(i)
        for i in range(nl):              # bottom-up: P3''..P7''
            self.node_defs.append(i)
        self.cells = []
        chans = {l: (self.feat_channels[l] if l in self.feat_channels else F) for l in self.levels}
        for c in range(cfg.fpn_cell_repeats):
            cell = []
            ins = self._node_inputs(nl)
            for j, li in enumerate(self.node_defs):
                pre = f"fpn_cell_{c}/node_{j}"
                lvl = self.levels[li]
                node = {"level": lvl, "inputs": ins[j], "resample": []}
                n_in = len(ins[j])
                P.add(f"{pre}/WSM", (n_in,), ("const", 1.0), False)
                for k, src in enumerate(ins[j]):
                    src_level, src_c = self._src_level_channels(src, c, chans)
                    rr = {"conv": None}
                    if src_c != F:
                        rp = f"{pre}/resample_{k}"
                        P.add(f"{rp}/conv2d/kernel", (F, src_c), ("glorot", src_c, F), True, pw=True)
                        P.add(f"{rp}/conv2d/bias", (F,), ("const", 0.0), False)
                        rr["conv"] = rp
                        rr["bn"] = P.add_bn(f"{rp}/bn", F, mom, eps)
                        rr["bn"].hw = sizes[src_level][0] * sizes[src_level][1]
                    node["resample"].append(rr)
                op = f"{pre}/op_after_combine"
                P.add(f"{op}/separable_conv2d/depthwise_kernel", (9, F), ("glorot", 9 * F, 9), True)
                P.add(f"{op}/separable_conv2d/pointwise_kernel", (F, F), ("glorot", F, F), True, pw=True)
                P.add(f"{op}/separable_conv2d/bias", (F,), ("const", 0.0), False)
                node["bn"] = P.add_bn(f"{op}/batch_normalization", F, mom, eps)
                node["bn"].hw = sizes[lvl][0] * sizes[lvl][1]
                node["prefix"] = pre
                cell.append(node)
            self.cells.append(cell)
        # heads
        self.heads = {}
        for net, nout, bias0 in (("class_net", self.A * self.NC, -math.log((1 - 0.01) / 0.01)),
                                 ("box_net", self.A * 4, 0.0)):
            tag = "class" if net == "class_net" else "box"
            h = {"convs": [], "bns": []}
            for i in range(cfg.box_class_repeats):
                pre = f"{net}/{tag}-{i}"
                P.add(f"{pre}/depthwise_kernel", (9, F), ("vs_fan_in", 9 * F), True)
                P.add(f"{pre}/pointwise_kernel", (F, F), ("vs_fan_in", F), True, pw=True)
                P.add(f"{pre}/bias", (F,), ("const", 0.0), False)
                h["convs"].append(pre)
                lv_bns = []
                for l in self.levels:
                    b = P.add_bn(f"{net}/{tag}-{i}-bn-{l}", F, mom, eps)
                    b.hw = sizes[l][0] * sizes[l][1]
                    lv_bns.append(b)
                h["bns"].append(lv_bns)
            pre = f"{net}/{tag}-predict"
            P.add(f"{pre}/depthwise_kernel", (9, F), ("vs_fan_in", 9 * F), True)
            P.add(f"{pre}/pointwise_kernel", (nout, F), ("vs_fan_in", F), True, pw=True)
            P.add(f"{pre}/bias", (nout,), ("const", bias0), False)
            h["predict"] = pre
            h["nout"] = nout
            self.heads[net] = h

    def _node_inputs(self, nl):
        """Input node ids per BiFPN node: ids 0..nl-1 are the cell inputs, nl.. the nodes."""
        td = list(range(nl - 2, 0, -1))
        ins = []
        prev = nl - 1  # top input (P7)
        # top-down: node j at level li takes (input li, previous top-down node or P_top)
        for j, li in enumerate(td):
            ins.append([li, prev])
            prev = nl + j
        # bottom-up P3'': (P3, last top-down node)
        ins.append([0, prev])
        last = nl + len(td)
        for li in range(1, nl):
            j_node = nl + len(td) + li  # id of this node
            if li < nl - 1:
                td_id = nl + td.index(li)
                ins.append([li, td_id, last])
            else:
                ins.append([li, last])
            last = j_node
        return ins

    def _src_level_channels(self, src, cell, chans):
        nl = len(self.levels)
        if src < nl:
            lvl = self.levels[src]
            c = chans[lvl] if cell == 0 else self.F
            return lvl, c
        return self.levels[self.node_defs[src - nl]], self.F

    # ------------------------------------------------------------------ helpers
    def _set_counts(self, B: int):
        if self._count_batch == B:
            return
        host = np.ones(max(self.P.n_bn, 1), np.float32)
        for bn in self.P.bns:
            host[bn.coff:bn.coff + bn.C] = float(B * bn.hw)
        self.P.bn_count.copy_(torch.from_numpy(host))
        self._count_batch = B

    def _prepare_input(self, inputs) -> torch.Tensor:
        x = inputs
        if not isinstance(x, torch.Tensor):
            x = torch.as_tensor(np.asarray(x))
        x = x.to(self.eng.device)
        assert x.dim() == 4 and x.shape[-1] == 3, "inputs must be NHWC [B, H, W, 3]"
        if x.dtype != self.eng.tdtype:
            x32 = x.float().contiguous() if x.dtype != torch.float32 else x.contiguous()
            xc = torch.empty(x.shape, dtype=self.eng.tdtype, device=self.eng.device)
            L.call("edet_cast_f32", self.eng.dt, vp(x32), vp(xc), x32.numel(), stream())
            return xc
        return x.contiguous()

    # ------------------------------------------------------------------ forward pieces
    def _mbconv(self, x: Act, i: int) -> Act:
        sp, b = self.specs[i], self.block_bns[i]
        eng, P = self.eng, self.P
        pre = f"{self.bb}/blocks_{i}"
        if sp.expand_ratio != 1:
            x = ops.conv1x1(eng, P, x, b["expand_w"], sp.expanded_filters, bns=[b["bn0"]], act=L.ACT_SWISH,
                            name=f"{pre}/expand")
        # inference: the SE squeeze rides in the depthwise epilogue (BN affine from moving
        # statistics); training needs the batch statistics of the whole output first
        svec = None if eng.training or not self.fused_squeeze else eng.zeros64(x.pyr.batch, x.C)
        d = ops.dwconv(eng, P, x, f"{pre}/depthwise_conv2d/depthwise_kernel", sp.kernel_size, sp.stride,
                       bns=[b["bn1"]], act=L.ACT_SWISH, name=f"{pre}/dw", squeeze=svec)
        ops.squeeze_excite(eng, P, d, f"{pre}/se", sp.se_filters, svec=svec)
        # the gated value is written once: the project conv's forward GEMM (and in training its
        # weight gradient) read it plain.  Also in inference, where BN + swish + gate could ride in
        # the GEMM's A staging: that lengthened the GEMMs' latency-bound K loops more than the
        # pass costs (config 2: 40.5k -> 31.2k images/s, r04k)
        if self.materialize_se and (MATERIALIZE_SE_MIN_N <= 0 or sp.output_filters >= MATERIALIZE_SE_MIN_N):
            d = ops.materialize(eng, d, name=f"{pre}/se_out")
        return ops.conv1x1(eng, P, d, b["project_w"], sp.output_filters, bns=[b["bn2"]], name=f"{pre}/project")

    def backbone(self, inputs, training: bool = False) -> List[torch.Tensor]:
        """BackboneModel.call (backbone_model.py:96-148): [features, reduction_1..5] as
        [B, H, W, C] tensors in the compute dtype (the normalised, activated block outputs)."""
        if training:
            memset0(self.P.bn_tstats)
        self.eng.tape = None
        x = self._prepare_input(inputs)
        B = x.shape[0]
        self._set_counts(B)
        self.eng.begin_scratch()
        self.eng.training = training
        if not training:
            L.call("edet_bn_inference_stats", self.P.n_bn, vp(self.P.bn_mm), vp(self.P.bn_mv), vp(self.P.bn_count),
                   vp(self.P.bn_istats[0]), vp(self.P.bn_istats[1]), stream())
        acts = self._backbone_acts(x, training)
        outs = []
        for a in acts:
            y = ops.materialize(self.eng, a).raw
            outs.append(y[: a.pyr.rows].view(B, a.pyr.H, a.pyr.W, a.C))
        self.eng.training = False
        return outs

    def _backbone_acts(self, x: torch.Tensor, training: bool) -> List[Act]:
        """Backbone as lazy activations: [features, reduction_1, ..., reduction_5]."""
        eng = self.eng
        out = ops.stem(eng, self.P, x, f"{self.bb}/stem/conv2d/kernel", self.stem_bn)
        reds = []
        for i in range(len(self.specs)):
            out = self._mbconv(out, i)
            if i in self.red_idx:
                reds.append(out)
        return [out] + reds

    def _resample_conv(self, x: Act, rr) -> Act:
        if rr["conv"] is None:
            return x
        return ops.conv1x1(self.eng, self.P, x, f"{rr['conv']}/conv2d/kernel", self.F, f"{rr['conv']}/conv2d/bias",
                           bns=[rr["bn"]], name=rr["conv"])

    def _bifpn_cell(self, c: int, feats: List[Act], pyr_out: Optional[Tuple[torch.Tensor, Pyr]]) -> List[Act]:
        eng, P, F = self.eng, self.P, self.F
        nl = len(self.levels)
        nodes: List[Act] = list(feats)
        outs_by_level = {}
        for j, node in enumerate(self.cells[c]):
            lvl = node["level"]
            H, W = self.level_hw[lvl]
            ins = []
            for k, src in enumerate(node["inputs"]):
                a = self._resample_conv(nodes[src], node["resample"][k])
                h = a.pyr.H
                mode = L.MODE_SAME if h == H else (L.MODE_MAXPOOL if h > H else L.MODE_UPSAMPLE)
                ins.append((a, mode))
            pre = node["prefix"]
            fused = ops.bifpn_fuse(eng, P, ins, [f"{pre}/WSM"], H, W, name=f"{pre}/fuse")
            op = f"{pre}/op_after_combine/separable_conv2d"
            d = ops.dwconv(eng, P, fused, f"{op}/depthwise_kernel", 3, 1, name=f"{pre}/dw")
            out_buf = None
            if pyr_out is not None and j >= nl - 2:
                buf, pyr = pyr_out
                s = self.levels.index(lvl)
                out_buf = buf[pyr.seg_slice(s)]
            o = ops.conv1x1(eng, P, d, f"{op}/pointwise_kernel", F, f"{op}/bias", bns=[node["bn"]],
                            out_buf=out_buf, name=f"{pre}/pw")
            nodes.append(o)
            if j >= nl - 2:
                outs_by_level[lvl] = o
        return [outs_by_level[l] for l in self.levels]

    def _head(self, net: str, image: Act, masks: Optional[torch.Tensor], training: bool) -> Act:
        eng, P, F = self.eng, self.P, self.F
        h = self.heads[net]
        surv = self.cfg.survival_prob
        for i, pre in enumerate(h["convs"]):
            orig = image
            d = ops.dwconv(eng, P, image, f"{pre}/depthwise_kernel", 3, 1, name=f"{pre}/dw")
            r = ops.conv1x1(eng, P, d, f"{pre}/pointwise_kernel", F, f"{pre}/bias", bns=h["bns"][i],
                            act=L.ACT_SWISH, name=f"{pre}/pw")
            if i > 0 and surv:
                scale = masks[i - 1] if (training and masks is not None) else None
                image = ops.residual(eng, r, orig, scale, name=f"{pre}/residual")
            else:
                image = r
        pre = h["predict"]
        d = ops.dwconv(eng, P, image, f"{pre}/depthwise_kernel", 3, 1, name=f"{pre}/dw")
        nout = h["nout"]
        ld = round_up(nout, CLS_LD_PAD) if training else nout
        return ops.conv1x1(eng, P, d, f"{pre}/pointwise_kernel", nout, f"{pre}/bias", ldy=ld, name=f"{pre}/pw")

    def _forward(self, inputs, training: bool, masks: Optional[Dict[str, torch.Tensor]] = None):
        eng, P = self.eng, self.P
        if eng.device.type != "cuda":
            raise RuntimeError("this model was built host-only (structure and parameters); the "
                               "EfficientDet compute path runs only on the GPU through libedet")
        x = self._prepare_input(inputs)
        B = x.shape[0]
        assert (x.shape[1], x.shape[2]) == self.level_hw_input, "input size must match the config image_size"
        self._set_counts(B)
        eng.begin_scratch()
        eng.training = training
        if not training:
            L.call("edet_bn_inference_stats", P.n_bn, vp(P.bn_mm), vp(P.bn_mv), vp(P.bn_count),
                   vp(P.bn_istats[0]), vp(P.bn_istats[1]), stream())
        all_feats = self._backbone_acts(x, training)
        feats = [all_feats[l] for l in self.levels if l < len(all_feats)]
        for l in self.levels:
            if l < len(all_feats):
                continue
            rec = self.resample_extra[l]
            a = self._resample_conv(feats[-1], rec)
            feats.append(ops.maxpool(eng, a, name=f"resample_p{l}"))
        pyr = Pyr(B, [self.level_hw[l] for l in self.levels])
        buf = eng.empty(pyr.rows, self.F)
        for c in range(self.cfg.fpn_cell_repeats):
            last = c == self.cfg.fpn_cell_repeats - 1
            feats = self._bifpn_cell(c, feats, (buf, pyr) if last else None)
        last_bns = [feats[s].bns[0] for s in range(len(self.levels))]
        image = ops.assemble_pyramid(eng, buf, pyr, feats, last_bns, name="fpn_out")
        cls = self._head("class_net", image, masks.get("class_net") if masks else None, training)
        box = self._head("box_net", image, masks.get("box_net") if masks else None, training)
        return cls, box, pyr

    def _views(self, act: Act, pyr: Pyr, last: int):
        out = []
        for s, l in enumerate(self.levels):
            H, W = self.level_hw[l]
            out.append(act.raw[pyr.seg_slice(s), : self.A * last].view(pyr.batch, H, W, self.A, last))
        return tuple(out)

    def call(self, inputs, training: bool = False, masks: Optional[Dict[str, torch.Tensor]] = None):
        """EfficientDetNet.call (efficientdet_net.py:76-95): returns (boxes, classes).

        training=True normalises with batch statistics (BN training mode) and applies the
        drop-connect scales in ``masks`` ({'class_net'|'box_net': [repeats-1, levels, B]},
        1/0 survival divided by survival_prob); no gradients are recorded here — use
        EfficientDetNetTrain.train_step for training."""
        if training:
            memset0(self.P.bn_tstats)
        self.eng.tape = None
        cls, box, pyr = self._forward(inputs, training, masks)
        self.eng.training = False
        self.last_outputs = (cls, box, pyr)
        return self._views(box, pyr, 4), self._views(cls, pyr, self.NC)

    __call__ = call

    # ------------------------------------------------------------------ checkpoints
    def state_dict(self):
        return self.P.state_dict()

    def load_state_dict(self, sd):
        self.P.load_state_dict(sd)

    def save_weights(self, path: str):
        from safetensors.numpy import save_file
        save_file({k: np.ascontiguousarray(v) for k, v in self.state_dict().items()}, path)

    def load_weights(self, path: str):
        from safetensors.numpy import load_file
        self.load_state_dict(load_file(path))


class EfficientDetNetTrain(EfficientDetNet):
    """EfficientDetNetTrain (efficientdet_net_train.py:11-132): fused loss + optimizer."""

    def __init__(self, blocks_args=None, global_params: Optional[Config] = None, anchors: Optional[Anchors] = None,
                 name: str = "", min_lr: float = 1e-6, dtype: str = "bf16", device="cuda", seed: int = 0,
                 lr_schedule: Optional[Dict] = None, world_size: int = 1, grad_allreduce=None,
                 npos_allreduce=None, drop_seed: int = 1234, rank: int = 0, skip_nonfinite: bool = False):
        super().__init__(blocks_args, global_params, name, dtype, device, seed)
        cfg = self.cfg
        self.anchors = anchors
        self.min_lr = min_lr
        self.world_size = world_size
        self.grad_allreduce = grad_allreduce
        self.npos_allreduce = npos_allreduce
        # each data-parallel replica draws its own drop-connect masks (MirroredStrategy replicas
        # draw tf.random.uniform independently, drop_connect.py:13): fold the rank into the seed
        self.rank = rank
        self.drop_seed = drop_seed ^ (0x9E3779B97F4A7C15 * rank & 0xFFFFFFFFFFFFFFFF) if rank else drop_seed
        dev = self.eng.device
        self.scalars = torch.zeros(8, dtype=torch.float32, device=dev)
        self.norm_partials = torch.zeros(2 * L.OPT_NORM_BLOCKS, dtype=torch.float64, device=dev)
        self.level_parts = torch.zeros(2 * L.MAX_SEG, dtype=torch.float32, device=dev)
        self.step_counter = torch.zeros(1, dtype=torch.int32, device=dev)
        s = lr_schedule or {}
        sc = L.Sched()
        sc.adjusted_lr = s.get("adjusted_lr", 0.08 * 2 / 64)
        sc.warmup_init = s.get("warmup_init", 0.008)
        sc.warmup_steps = s.get("warmup_steps", 1000)
        sc.total_steps = s.get("total_steps", 300000)
        sc.momentum = s.get("momentum", 0.9)
        sc.ema_decay = s.get("ema_decay", 0.9998)
        sc.clip_norm = s.get("clip_norm", 10.0)
        sc.l2_weight = s.get("l2_weight", 4e-5)
        sc.fixed_lr = s.get("fixed_lr", 0.0)
        # SURVEY §5 failure detection: a step with a NaN / Inf gradient norm leaves the weights,
        # optimizer slots and step counter unchanged and reports it in scalars[6] (off by default:
        # the reference applies every step, efficientdet_net_train.py:129-130)
        sc.skip_nonfinite = int(bool(skip_nonfinite))
        self.sched = sc
        self.drop_masks = None
        self.steps_run = 0  # compute_step calls (graphed_train_step needs one eager warm-up)
        self.last_step_signature = None  # shape_signature of the last compute_step's data
        self.fixed_masks = None  # test hook: {'class_net': [rep-1, nseg, B], 'box_net': ...}

    # ------------------------------------------------------------------ data
    def _targets(self, data, pyr: Pyr) -> Targets:
        if len(data) == 2 and isinstance(data[1], Targets):
            t = data[1]
            assert t.pyr.rows == pyr.rows and t.pyr.sizes == pyr.sizes
            return t
        _, yb, yc, ym = data
        return Targets.from_reference(yb, yc, ym, pyr, self.A, self.eng.device)

    def _make_masks(self, B: int):
        cfg = self.cfg
        reps = cfg.box_class_repeats - 1
        if not cfg.survival_prob or reps <= 0:
            return None
        if self.fixed_masks is not None:
            return self.fixed_masks
        nseg = len(self.levels)
        n = 2 * reps * nseg * B
        if self.drop_masks is None or self.drop_masks.numel() != n:
            self.drop_masks = torch.empty(n, dtype=torch.float32, device=self.eng.device)
        L.call("edet_dropmask", vp(self.drop_masks), n, float(cfg.survival_prob), self.drop_seed,
               vp(self.step_counter), stream())
        m = self.drop_masks.view(2, reps, nseg, B)
        return {"class_net": m[0], "box_net": m[1]}

    # ------------------------------------------------------------------ step
    def prepare_step(self, data):
        """Zero the per-step accumulators, build the targets and count this replica's positive
        anchors into scalars[5].  Split from the compute so a data-parallel step can all-reduce
        N+ between the two (and capture each half in its own graph)."""
        P = self.P
        x = data[0]
        B = x.shape[0]
        s = stream()
        memset0_many([P.g, P.bn_tstats, self.scalars, self.level_parts])
        pyr = Pyr(B, [self.level_hw[l] for l in self.levels])
        t = self._targets(data, pyr)
        # N+ = sum(masks) + 1 (the +1 is added by the loss kernel); padding rows are never read
        self._count_positives(t, pyr, self.scalars[5:6], s)
        return t, pyr

    def _count_positives(self, t, pyr, out, s):
        if pyr.rows == sum(pyr.seg_rows(seg) for seg in range(pyr.nseg)):
            # levels back to back (every level a multiple of 128 rows, D0 at 512 included): one launch
            L.call("edet_count_positives", vp(t.mask), pyr.rows * self.A, vp(out), s)
            return
        for seg in range(pyr.nseg):
            sl = pyr.seg_slice(seg)
            L.call("edet_count_positives", vp(t.mask[sl]), pyr.seg_rows(seg) * self.A, vp(out), s)

    def compute_step(self, data, t, pyr):
        """Forward, fused loss (fwd+bwd) and backward with N+ already global in scalars[5]."""
        eng = self.eng
        x = data[0]
        s = stream()
        masks = self._make_masks(x.shape[0])
        eng.tape = Tape(eng, getattr(self, "grad_trace", None))
        cls, box, pyr2 = self._forward(x, True, masks)
        # fused focal + Huber loss: gradients are written in place over the logits.  The focal
        # mean runs over this replica's elements, so it is scaled by world_size to make the
        # replicas' sum the global-batch mean.
        L.call("edet_detection_loss", eng.dt, vp(cls.raw), cls.ld, vp(box.raw), box.ld, pyr.c, self.A, self.NC,
               vp(t.cls), vp(t.box), vp(self.scalars[5:6]), float(self.cfg.alpha), float(self.cfg.gamma), 0.1, 50.0,
               float(self.world_size), vp(cls.raw), vp(box.raw), vp(self.scalars[0:1]), vp(self.level_parts), s)
        eng.tape.alias(cls, cls.raw, cls.ld)
        eng.tape.alias(box, box.raw, box.ld)
        eng.tape.backward()
        eng.tape = None
        eng.training = False
        self.steps_run += 1
        self.last_step_signature = self.shape_signature(data)
        return t

    @staticmethod
    def shape_signature(data):
        """(shape, dtype) of the step's input image batch: the persistent buffers of an eager step
        are sized by it (dist.graphed_train_step checks its warm-up ran on the same shapes)."""
        x = data[0]
        return (tuple(x.shape), str(x.dtype))

    def forward_backward(self, data):
        """Zero accumulators, targets, N+ (all-reduced when data-parallel), forward, loss,
        backward.  No optimizer."""
        t, pyr = self.prepare_step(data)
        if self.npos_allreduce is not None:
            self.npos_allreduce(self.scalars[5:6])
        return self.compute_step(data, t, pyr)

    def apply_gradients(self):
        P = self.P
        s = stream()
        L.call("edet_opt_norm", vp(P.w), vp(P.g), P.numel, P.n_l2, self.sched, vp(self.scalars),
               vp(self.norm_partials), vp(self.step_counter), s)
        L.call("edet_opt_apply", vp(P.w), vp(P.g), vp(P.v), vp(P.ema), P.numel, P.n_l2, self.sched, vp(self.scalars),
               vp(self.norm_partials), self.eng.dt, vp(P.wc) if P.wc is not P.w else None, vp(self.step_counter), s)
        P.refresh_compute_copy(cast=False)  # transposed 1x1 copies for the next dgrad
        cfg = self.cfg
        # a skipped non-finite step (skip_nonfinite) leaves the moving statistics alone as well
        skip = vp(self.scalars[6:7]) if self.sched.skip_nonfinite else None
        L.call("edet_bn_update_moving", P.n_bn, vp(P.bn_tstats[0]), vp(P.bn_tstats[1]), vp(P.bn_count),
               float(cfg.batch_norm_momentum), skip, vp(P.bn_mm), vp(P.bn_mv), s)

    def load_state_dict(self, sd):
        """Weights (and BN moving statistics) from a checkpoint, with fresh optimizer state:
        zero momentum, EMA = the loaded weights, step counter 0 -- the reference restarts the
        same way from its weights-only h5 (train.py:127-129, 150)."""
        super().load_state_dict(sd)
        memset0(self.P.v)
        memset0(self.step_counter)

    def test_step(self, data):
        """test_step (efficientdet_net_train.py:135-169): inference-mode forward, the same loss
        (forward only), decode + DIoU-NMS per image on the GPU, and the reference's per-image
        mAP (host numpy, metrics.py) averaged over the batch.

        data = (x, gt_boxes [B,G,4], gt_classes [B,G], y_true_boxes[5], y_true_classes[5],
        y_true_masks[5]); each image's G ground-truth rows are scored as given, like the
        reference's numpy_function call."""
        from . import metrics
        x, real_boxes, real_classes, yb, yc, ym = data
        boxes_out, classes_out = self.call(x, training=False)
        cls, box, pyr = self.last_outputs
        t = Targets.from_reference(yb, yc, ym, pyr, self.A, self.eng.device)
        s = stream()
        sc = torch.zeros(8, dtype=torch.float32, device=self.eng.device)
        parts = torch.zeros(2 * L.MAX_SEG, dtype=torch.float32, device=self.eng.device)
        self._count_positives(t, pyr, sc[5:6], s)
        L.call("edet_detection_loss", self.eng.dt, vp(cls.raw), cls.ld, vp(box.raw), box.ld, pyr.c, self.A, self.NC,
               vp(t.cls), vp(t.box), vp(sc[5:6]), float(self.cfg.alpha), float(self.cfg.gamma), 0.1, 50.0, 1.0,
               None, None, vp(sc[0:1]), vp(parts), s)
        P = self.P  # _reg_l2_loss (efficientdet_net_train.py:21-28): the L2 prefix of the flat weights
        l2 = 4e-5 * 0.5 * float((P.w[: P.n_l2].double() ** 2).sum())
        loss = float(sc[0]) + l2
        ob, oc, os_, cnt = self.anchors.detect(self.anchors.convert_outputs_boxes(boxes_out), classes_out)
        ob, oc, os_, cnt = ob.cpu().numpy(), oc.cpu().numpy(), os_.cpu().numpy(), cnt.cpu().numpy()
        rb = np.asarray(real_boxes.cpu() if isinstance(real_boxes, torch.Tensor) else real_boxes, np.float64)
        rc = np.asarray(real_classes.cpu() if isinstance(real_classes, torch.Tensor) else real_classes, np.float64)
        m = 0.0
        for b in range(x.shape[0]):
            k = int(cnt[b])
            pred = np.concatenate([ob[b, :k], oc[b, :k, None], os_[b, :k, None]], -1)
            gt = np.concatenate([rb[b], rc[b][:, None]], -1)
            m += metrics.get_map_one(gt, pred, self.NC, 0.5)
        return {"loss": loss, "mAP": m / x.shape[0]}

    def train_step(self, data):
        """train_step_normal (efficientdet_net_train.py:112-132)."""
        self.forward_backward(data)
        if self.grad_allreduce is not None:
            self.grad_allreduce(self.P.g)
        self.apply_gradients()
        out = {"loss": self.scalars[0], "gnorm": self.scalars[3]}
        if self.sched.skip_nonfinite:
            out["skipped"] = self.scalars[6]
        return out
