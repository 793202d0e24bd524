"""torch-CPU restatement of the reference EfficientDet forward / loss / train step.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Runs in float64 by default (float32 for
the timed CPU baseline).  Layout NHWC at the interface, NCHW internally.

Structure is derived HERE, from the config and the reference's own construction rules, never
from the product's model object:
  * block list        efficientnet/backbone_model.py:59-93 (first block of a stage takes the
                      stage stride and input width, repeats s=1 / C_in = C_out) with
                      utils/round_filters.py:2-12, utils/round_repeats.py:3-6
  * block layers      layers/mb_conv_block.py:41-124 (conv2d / tpu_batch_normalization name
                      counters :45-51, SE width max(1, int(C_in * se_ratio)) :98-101)
  * reductions        backbone_model.py:119-139 (last block, or block before a stride-2 one)
  * feature levels    efficientdet_net.py:80-85 (all_feats[min:max+1] + resample_p6/p7)
  * resampling        layers/resample_feature_map.py:14-41: conv1x1+bias+BN iff the input's
                      channel count differs from the target, max-pool iff taller than the
                      level size, nearest resize iff shorter -- decided from the tensor that
                      actually arrives, exactly like Keras' lazy build
  * BiFPN topology    layers/bifpn.py:108-116 (the eight explicit node calls)
  * heads             layers/class_net.py:54-103, layers/box_net.py:52-102 (shared convs,
                      per-level BN 'class-%d-bn-%d', residual iff i > 0 and survival_prob)
Parameters are created on first use, like Keras layers: ``param_specs(cfg)`` runs the forward
on a 'meta' tensor and records every (name, shape, initialiser) in creation order.  A test
checks that list against the product's parameter table, so a product that wires a BiFPN edge,
a head BN or an endpoint differently from the reference rules cannot agree with this oracle.

Naming and storage layouts (the build's checkpoint contract): 1x1 kernels
[out][in]; depthwise kernels [k*k][C]; stem kernel HWIO [3][3][3][Co]; BN variables
'<bn>/gamma', '/beta', '/moving_mean', '/moving_variance'; BiFPN fusion weights one vector
'<node>/WSM' of the node's n_in scalars (the reference's WSM_0..WSM_{n-1}, bifpn.py:47-54).

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
"""
from __future__ import annotations

import math
import re
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as Fn

# efficientnet/train.py:81-89 -- (num_repeat, kernel_size, strides, expand_ratio,
# input_filters, output_filters, se_ratio), the EfficientDetBlockArgs field order
B0_BLOCKS = [
    (1, 3, (1, 1), 1, 32, 16, 0.25), (2, 3, (2, 2), 6, 16, 24, 0.25), (2, 5, (2, 2), 6, 24, 40, 0.25),
    (3, 3, (2, 2), 6, 40, 80, 0.25), (3, 5, (1, 1), 6, 80, 112, 0.25), (4, 5, (2, 2), 6, 112, 192, 0.25),
    (1, 3, (1, 1), 6, 192, 320, 0.25),
]


def round_filters(filters, width, divisor):
    """utils/round_filters.py:2-12."""
    filters = filters * width
    new = max(divisor, int(filters + divisor / 2) // divisor * divisor)
    if new < 0.9 * filters:
        new += divisor
    return int(new)


def round_repeats(repeats, depth):
    """utils/round_repeats.py:3-6."""
    return int(math.ceil(depth * repeats))


def _args(b):
    """EfficientDetBlockArgs-like record (namedtuple or plain tuple) -> tuple of 7 fields."""
    if hasattr(b, "num_repeat"):
        return (b.num_repeat, b.kernel_size, tuple(b.strides), b.expand_ratio, b.input_filters, b.output_filters,
                b.se_ratio)
    return tuple(b)


def block_list(cfg, blocks_args=None):
    """BackboneModel._build (backbone_model.py:40-93): one record per MBConvBlock."""
    blocks = []
    for a in (blocks_args if blocks_args is not None else B0_BLOCKS):
        rep, k, strides, e, cin, cout, se = _args(a)
        cin = round_filters(cin, cfg.width_coefficient, cfg.depth_divisor)
        cout = round_filters(cout, cfg.width_coefficient, cfg.depth_divisor)
        rep = round_repeats(rep, cfg.depth_coefficient)
        blocks.append(dict(k=k, s=strides[0], e=e, cin=cin, cout=cout, se=se))
        for _ in range(rep - 1):
            blocks.append(dict(k=k, s=1, e=e, cin=cout, cout=cout, se=se))
    return blocks


def _keras_counter_names(base):
    """mb_conv_block.py:45-51: '', '_1', '_2', ... via the double-next counter."""
    c = iter(range(1 << 30))

    def nxt():
        return base + ("" if not next(c) else "_" + str(next(c) // 2))
    return nxt


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


def maxpool_same(x, route=None, stats=None):
    """MaxPooling2D 3x3 s2 'SAME' (resample_feature_map.py:35-38): padded cells ignored.

    ``route`` (optional, same shape as x): choose each window's argmax on these values instead
    of x's own (first maximum in row-major order, like TF's MaxPoolGrad and torch) and take x
    at that position.  Parity tests pass the product's own fp32 values here so that windows
    whose top two entries lie within fp32 rounding of each other -- where fp32 and fp64
    legitimately pick different winners and the gradient is routed to a different pixel --
    are decided the same way on both sides; ``stats['rerouted']`` counts the windows whose
    decision that changed.  The forward value changes by at most that near-tie gap."""
    pt, pb = same_pad(x.shape[2], 3, 2)
    pl, pr = same_pad(x.shape[3], 3, 2)
    xp = Fn.pad(x, (pl, pr, pt, pb), value=-math.inf)
    if route is None:
        return Fn.max_pool2d(xp, 3, 2)
    rp = Fn.pad(torch.as_tensor(route, dtype=x.dtype), (pl, pr, pt, pb), value=-math.inf)
    _, idx = Fn.max_pool2d(rp, 3, 2, return_indices=True)
    N, C, Ho, Wo = idx.shape
    out = xp.reshape(N, C, -1).gather(2, idx.reshape(N, C, -1)).reshape(N, C, Ho, Wo)
    if stats is not None:
        ownv, own = Fn.max_pool2d(xp.detach(), 3, 2, return_indices=True)
        moved = own != idx
        stats["rerouted"] = stats.get("rerouted", 0) + int(moved.sum())
        stats["windows"] = stats.get("windows", 0) + idx.numel()
        # the tie gap: how far below its own window maximum the routed value lies, relative
        # to the tensor's largest magnitude (0 when nothing moved)
        if bool(moved.any()):
            gap = float((ownv - out.detach())[moved].max()) / max(float(x.detach().abs().max()), 1e-30)
            stats["max_gap_rel"] = max(stats.get("max_gap_rel", 0.0), gap)
    return out


def resize_nearest(x, H, W):
    """tf.image.resize(method='nearest') (resample_feature_map.py:41): half-pixel centres."""
    h, w = x.shape[2], x.shape[3]
    sy, sx = np.float32(h) / np.float32(H), np.float32(w) / np.float32(W)
    iy = [min(int(np.floor((np.float32(o) + np.float32(0.5)) * sy)), h - 1) for o in range(H)]
    ix = [min(int(np.floor((np.float32(o) + np.float32(0.5)) * sx)), w - 1) for o in range(W)]
    return x[:, :, iy][:, :, :, ix]


# Keras initialisers, as (kind, *args) records:
#   ('normal', std)        utils/conv_kernel_initializer.py:4-25  N(0, sqrt(2 / (kh*kw*out)))
#   ('glorot', fan_in, fan_out)   keras default glorot_uniform, U(+-sqrt(6/(fi+fo)))
#   ('vs_fan_in', fan_in)  tf.initializers.VarianceScaling(): truncated normal, scale 1, fan_in
#   ('const', v)           zeros / ones / constant initialisers
def _cki(kh, kw, out):
    return ("normal", math.sqrt(2.0 / (kh * kw * out)))


def bf16_store(t):
    """bf16 storage of a tensor the product keeps in HBM, both directions: the value is rounded
    on the forward, and (through .to's autograd) the incoming gradient on the backward."""
    return t.to(torch.bfloat16).to(t.dtype)


class _GradBF16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def _dither_round(t, gen, frac):
    """bf16 round-to-nearest-even of t plus a uniform dither of +-frac/2 bf16 ulp: the same
    rounding error magnitude (x 1.01 in RMS at frac = 1/4), different rounding decisions per
    seed -- one member of an ensemble of bf16-storage emulations."""
    if gen is None:
        return t.to(torch.bfloat16).to(t.dtype)
    _, e = torch.frexp(t)
    u = torch.rand(t.shape, generator=gen, dtype=t.dtype, device=t.device) - 0.5
    d = torch.where(t != 0, u * frac * torch.ldexp(torch.ones_like(t), e - 8), torch.zeros_like(t))  # 0 stays 0
    return (t + d).to(torch.bfloat16).to(t.dtype)


class _StoreDither(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gen, frac, both):
        ctx.gen, ctx.frac = gen, frac
        return _dither_round(x, gen, frac) if both else x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return _dither_round(g, ctx.gen, ctx.frac), None, None, None


class _OperandDither(torch.autograd.Function):
    """Forward rounding only: a matrix-core operand the product rounds to bf16 while staging it
    (gradient untouched -- the gradient of that value is rounded where it is stored)."""

    @staticmethod
    def forward(ctx, x, gen, frac):
        return _dither_round(x, gen, frac)

    @staticmethod
    def backward(ctx, g):
        return g, None, None


def bf16_dither_hooks(seed, frac=0.25):
    """(store, gstore, ostore) for RefEfficientDet: bf16 storage emulated in both directions with a
    seeded sub-ulp dither before each rounding (see _dither_round), and the bf16 rounding of the
    1x1 convolutions' lazily transformed A operands (ostore, forward only)."""
    gen = None if seed is None else torch.Generator().manual_seed(seed)
    return (lambda t: _StoreDither.apply(t, gen, frac, True), lambda t: _StoreDither.apply(t, gen, frac, False),
            lambda t: _OperandDither.apply(t, gen, frac))


def bf16_grad(t):
    """Identity forward, bf16 rounding of the gradient: a value the product never stores (a lazy
    BN / swish output) whose gradient its consumer's dgrad writes in bf16."""
    return _GradBF16.apply(t)


class RefEfficientDet:
    """Restatement of EfficientDetNet (efficientdet_net.py:10-95) + EfficientDetNetTrain."""

    def __init__(self, cfg, params: Optional[Dict[str, np.ndarray]] = None, dtype=torch.float64, blocks_args=None):
        self.cfg = cfg
        self.dtype = dtype
        self.blocks = block_list(cfg, blocks_args)
        first = _args((blocks_args if blocks_args is not None else B0_BLOCKS)[0])
        self.stem_filters = round_filters(first[4], cfg.width_coefficient, cfg.depth_divisor)
        self.eps = cfg.batch_norm_epsilon
        self.F = cfg.fpn_num_filters
        self.A = cfg.num_scales * len(cfg.aspect_ratios)
        self.NC = cfg.num_classes
        self.levels = list(range(cfg.min_level, cfg.max_level + 1))
        ls = [cfg.image_size]  # global_params.py:206-208
        for _ in range(cfg.max_level):
            ls.append((ls[-1] + 1) // 2)
        self.levels_size = ls
        self.bb = cfg.backbone_name or "backbone"
        n = len(self.blocks)
        self.red_idx = [i for i in range(n) if i == n - 1 or self.blocks[i + 1]["s"] > 1]
        self.recording = None
        self.trace = None  # debug: name -> intermediate tensor (the product's activation names)
        self.routes = None  # name -> values deciding max-pool winners (see maxpool_same)
        self.route_stats = {}
        self.store = None  # storage rounding of every tensor the product keeps in HBM (bf16 emulation)
        self.gstore = None  # gradient rounding at every conv / resample input (the stored dv)
        # forward rounding of a 1x1 conv's A operand that the product transforms lazily (BN /
        # swish applied while staging) and rounds to bf16 for the matrix cores
        self.ostore = None
        self._names = {}
        self.p = {}
        if params is not None:
            self.p = {k: torch.tensor(np.asarray(v), dtype=dtype) for k, v in params.items()}

    def _t(self, name, x):
        """Name an intermediate with the product's activation name (tracing / pool routing)."""
        if self.recording is None:
            if self.trace is not None:
                if x.requires_grad:
                    x.retain_grad()
                self.trace[name] = x
            if self.routes is not None:
                self._names[id(x)] = name
        return x

    def _st(self, x):
        """A tensor the product stores (conv outputs, SE output, fusion sums, residual sums,
        pooled values): rounded by ``store`` when emulating a storage precision."""
        return x if self.store is None or self.recording is not None else self.store(x)

    def _gin(self, x):
        """A conv or resample input: its gradient is what the product's dgrad / fusion backward
        stores, rounded by ``gstore`` when emulating a storage precision."""
        if self.gstore is None or self.recording is not None:
            return x
        y = self.gstore(x)
        if id(x) in self._names:  # keep the pool routing's name on the wrapped value
            self._names[id(y)] = self._names[id(x)]
        return y

    def _op(self, x):
        """The A operand of a 1x1 conv (expand, resample): the product stages bf16(v(x)) for the
        MFMA, so its value is rounded by ``ostore`` when emulating bf16 (a stored operand -- the
        SE output, a depthwise output -- is already rounded and not wrapped)."""
        return x if self.ostore is None or self.recording is not None else self.ostore(x)

    def _pool(self, x, stored):
        route = None
        if self.routes is not None:
            route = self.routes.get(self._names.get(id(x)))
        y = maxpool_same(x, route, self.route_stats)
        # resample_p6/p7 are stored; a BiFPN input is pooled inside the fusion kernel
        return self._st(y) if stored else y

    # ---- parameters, created on first use (Keras lazy build)
    def w(self, name, shape, init):
        if self.recording is not None:
            if name not in self.recording:
                self.recording[name] = (tuple(shape), init)
            else:
                assert self.recording[name][0] == tuple(shape), (name, shape, self.recording[name])
            return torch.zeros(shape, dtype=self.dtype, device="meta")
        t = self.p[name]
        assert tuple(t.shape) == tuple(shape), (name, tuple(t.shape), shape)
        return t

    def w1x1(self, name, out, cin, init):  # [out][in] -> [out, in, 1, 1]
        return self.w(name, (out, cin), init)[:, :, None, None]

    def wdw(self, name, k, C, init):  # [k*k][C] -> [C, 1, k, k]
        return self.w(name, (k * k, C), init).t().reshape(C, 1, k, k)

    def bn(self, x, name, training, st):
        """Keras BatchNormalization (momentum 0.99, eps 1e-3) on NCHW x."""
        C = x.shape[1]
        g = self.w(name + "/gamma", (C,), ("const", 1.0))
        b = self.w(name + "/beta", (C,), ("const", 0.0))
        if self.recording is not None:
            self.recording.setdefault("__bn__", []).append(name)
        if training:
            mean = x.mean(dim=(0, 2, 3))
            var = ((x - mean[None, :, None, None]) ** 2).mean(dim=(0, 2, 3))
            if st is not None:
                st.batch[name] = (mean.detach(), var.detach(), x.shape[0] * x.shape[2] * x.shape[3])
        elif self.recording is not None:
            mean = var = torch.zeros(C, dtype=self.dtype, device="meta")
        else:
            mean, var = self.p[name + "/moving_mean"], self.p[name + "/moving_variance"]
        inv = 1.0 / torch.sqrt(var + self.eps)
        return (x - mean[None, :, None, None]) * (inv * g)[None, :, None, None] + b[None, :, None, None]

    # ---- layers
    def stem(self, x, training, st):
        """layers/stem.py:37-38 (conv 3x3 s2 SAME, no bias -> BN -> swish)."""
        cs = self.stem_filters  # round_filters(blocks_args[0].input_filters) (stem.py:15-16)
        w = self.w(f"{self.bb}/stem/conv2d/kernel", (3, 3, 3, cs), _cki(3, 3, cs)).permute(3, 2, 0, 1)
        return self._t("stem", swish(self.bn(self._st(conv_same(x, w, 2)), f"{self.bb}/stem/tpu_batch_normalization",
                                             training, st)))

    def mbconv(self, x, i, training, st):
        """layers/mb_conv_block.py:127-160 (no skip, no drop-connect)."""
        b = self.blocks[i]
        pre = f"{self.bb}/blocks_{i}"
        bn_name = _keras_counter_names("tpu_batch_normalization")
        conv_name = _keras_counter_names("conv2d")
        cin, e = b["cin"], b["cin"] * b["e"]
        if b["e"] != 1:
            n = conv_name()
            x = self._st(Fn.conv2d(self._op(self._gin(x)), self.w1x1(f"{pre}/{n}/kernel", e, cin, _cki(1, 1, e))))
            x = self._t(f"{pre}/expand", swish(self.bn(x, f"{pre}/{bn_name()}", training, st)))
        k = b["k"]
        x = self._st(conv_same(self._gin(x), self.wdw(f"{pre}/depthwise_conv2d/depthwise_kernel", k, e, _cki(k, k, 1)), b["s"],
                               groups=e))
        x = swish(self.bn(x, f"{pre}/{bn_name()}", training, st))
        # SE (layers/se.py:35-39), width mb_conv_block.py:98-101
        R = max(1, int(cin * b["se"]))
        s = x.mean(dim=(2, 3), keepdim=True)
        s = Fn.conv2d(s, self.w1x1(f"{pre}/se/conv2d/kernel", R, e, _cki(1, 1, R)),
                      self.w(f"{pre}/se/conv2d/bias", (R,), ("const", 0.0)))
        s = Fn.conv2d(swish(s), self.w1x1(f"{pre}/se/conv2d_1/kernel", e, R, _cki(1, 1, e)),
                      self.w(f"{pre}/se/conv2d_1/bias", (e,), ("const", 0.0)))
        x = self._t(f"{pre}/se_out", self._st(torch.sigmoid(s) * x))
        n = conv_name()
        x = self._st(Fn.conv2d(self._gin(x), self.w1x1(f"{pre}/{n}/kernel", b["cout"], e, _cki(1, 1, b["cout"]))))
        return self._t(f"{pre}/project", self.bn(x, f"{pre}/{bn_name()}", training, st))

    def resample(self, x, prefix, level_size, training, st):
        """ResampleFeatureMap (resample_feature_map.py:14-52): decisions from the arriving
        tensor's channels and height, as its lazy build() makes them."""
        F = self.F
        C = x.shape[1]
        x = self._gin(x)
        if C != F:
            x = self._st(Fn.conv2d(self._op(x), self.w1x1(f"{prefix}/conv2d/kernel", F, C, ("glorot", C, F)),
                                   self.w(f"{prefix}/conv2d/bias", (F,), ("const", 0.0))))
            x = self._t(prefix, self.bn(x, f"{prefix}/bn", training, st))
        if x.shape[2] > level_size:
            x = self._t(prefix + "/pool", self._pool(x, stored=prefix.startswith("resample_p")))
        elif x.shape[2] < level_size:
            x = resize_nearest(x, level_size, level_size)
        return x

    def sepconv(self, x, pre, dwname, pwname, bname, nout, dw_init, pw_init, b_init):
        C = x.shape[1]
        x = self._st(conv_same(self._gin(x), self.wdw(f"{pre}/{dwname}", 3, C, dw_init), 1, groups=C))
        return self._st(Fn.conv2d(self._gin(x), self.w1x1(f"{pre}/{pwname}", nout, C, pw_init),
                                  self.w(f"{pre}/{bname}", (nout,), b_init)))

    # bifpn.py:108-116: (level, input node ids); ids 0..4 = P3..P7 inputs, 5.. = nodes
    BIFPN_NODES = [(6, [3, 4]), (5, [2, 5]), (4, [1, 6]), (3, [0, 7]), (4, [1, 7, 8]), (5, [2, 6, 9]), (6, [3, 5, 10]),
                   (7, [4, 11])]

    def bifpn_cell(self, c, feats, training, st):
        """BiFPN.call / BiFPNNode.call / OpAfterCombine.call (bifpn.py:24-29, 59-67, 89-117)."""
        assert len(feats) == 5, "bifpn.py:105 unpacks exactly P3..P7"
        nodes = list(feats)
        F = self.F
        for j, (lvl, ins) in enumerate(self.BIFPN_NODES):
            pre = f"fpn_cell_{c}/node_{j}"
            size = self.levels_size[lvl]
            w = self.w(f"{pre}/WSM", (len(ins),), ("const", 1.0))
            wsum = w.sum()
            acc = None
            for k, src in enumerate(ins):
                r = self.resample(nodes[src], f"{pre}/resample_{k}", size, training, st) * w[k] / (wsum + 0.0001)
                acc = r if acc is None else acc + r
            op = f"{pre}/op_after_combine"
            y = self.sepconv(self._t(f"{pre}/fuse", swish(self._st(acc))), op, "separable_conv2d/depthwise_kernel",
                             "separable_conv2d/pointwise_kernel", "separable_conv2d/bias", F, ("glorot", 9 * F, 9),
                             ("glorot", F, F), ("const", 0.0))
            y = self._t(f"{pre}/pw", self.bn(y, f"{op}/batch_normalization", training, st))
            nodes.append(y)
        return nodes[-5:]  # (p3_2, p4_2, p5_2, p6_2, p7_2)

    def head(self, net, feats, training, st, masks=None):
        """ClassNet.call / BoxNet.call (class_net.py:79-103, box_net.py:81-102)."""
        tag = "class" if net == "class_net" else "box"
        last = self.NC if net == "class_net" else 4
        nout = self.A * last
        bias0 = -math.log((1 - 0.01) / 0.01) if net == "class_net" else 0.0  # class_net.py:74
        F = self.F
        surv = self.cfg.survival_prob
        vs = lambda fan: ("vs_fan_in", fan)  # noqa: E731
        out = []
        for li, lvl in enumerate(self.levels):
            image = feats[li]
            for i in range(self.cfg.box_class_repeats):
                orig = image
                pre = f"{net}/{tag}-{i}"
                image = self.sepconv(image, pre, "depthwise_kernel", "pointwise_kernel", "bias", F, vs(9 * F), vs(F),
                                     ("const", 0.0))
                image = swish(self.bn(image, f"{net}/{tag}-{i}-bn-{lvl}", training, st))
                if i > 0 and surv:
                    if training:
                        m = masks[net][i - 1][li] if masks is not None else None
                        if m is not None:
                            image = image * torch.as_tensor(m, dtype=self.dtype)[:, None, None, None]
                    image = self._st(image + orig)
            pre = f"{net}/{tag}-predict"
            c = self.sepconv(image, pre, "depthwise_kernel", "pointwise_kernel", "bias", nout, vs(9 * F), vs(F),
                             ("const", bias0))
            B, _, H, W = c.shape
            out.append(c.permute(0, 2, 3, 1).reshape(B, H, W, self.A, last))
        return out

    def _input(self, x_nhwc):
        if isinstance(x_nhwc, torch.Tensor) and x_nhwc.device.type == "meta":
            return x_nhwc.permute(0, 3, 1, 2)
        return torch.as_tensor(np.asarray(x_nhwc), dtype=self.dtype).permute(0, 3, 1, 2)

    def _backbone(self, x, training, st):
        x = self.stem(x, training, st)
        reds = []
        for i in range(len(self.blocks)):
            x = self.mbconv(x, i, training, st)
            if i in self.red_idx:
                reds.append(x)
        return [x] + reds

    def backbone(self, x_nhwc, training, st: Optional[BNState] = None):
        """BackboneModel.call (backbone_model.py:96-148): [features, reduction_1..5], NHWC."""
        return [t.permute(0, 2, 3, 1) for t in self._backbone(self._input(x_nhwc), training, st)]

    def forward(self, x_nhwc, training, masks=None, st: Optional[BNState] = None):
        """EfficientDetNet.call (efficientdet_net.py:76-95): (boxes list, classes list), NHWC
        [B, H, W, A, *]."""
        self._names = {}
        all_feats = self._backbone(self._input(x_nhwc), training, st)
        feats = all_feats[self.cfg.min_level:self.cfg.max_level + 1]
        for level in range(6, self.cfg.max_level + 1):  # efficientdet_net.py:28-35, 84-85
            feats.append(self.resample(feats[-1], f"resample_p{level}", self.levels_size[level], training, st))
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


def param_specs(cfg, blocks_args=None) -> "OrderedDict[str, tuple]":
    """Every variable the reference model creates for ``cfg``, in creation order:
    name -> (shape, initialiser record).  BN moving statistics are listed by ``bn_names``."""
    r = RefEfficientDet(cfg, None, torch.float32, blocks_args)
    r.recording = OrderedDict()
    S = cfg.image_size
    r.forward(torch.zeros((1, S, S, 3), dtype=torch.float32, device="meta"), True)
    rec = r.recording
    bns = rec.pop("__bn__")
    out = OrderedDict((k, v) for k, v in rec.items())
    out.bn_names = list(OrderedDict.fromkeys(bns))  # type: ignore[attr-defined]
    return out


def ref_train_step(ref: RefEfficientDet, x, y_box, y_cls, y_mask, masks=None, lr=0.01, momentum=0.9, clip=10.0,
                   ema_decay=0.9998, mom_state=None, ema_state=None, bn_momentum=0.99):
    """train_step_normal (efficientdet_net_train.py:112-132) + SGD momentum + EMA + BN moving
    update.  Returns (loss, gnorm, new_params dict, grads dict, bnstate, parts)."""
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
    for p in ref.p.values():
        p.requires_grad_(False)
    return loss.detach(), gnorm.detach(), new, {k: g.detach() for k, g in grads.items()}, st, parts
