"""Model hyper-parameters and shape arithmetic.

Restates, without TensorFlow:
  * ``utils/global_params.py:4-141``  the efficientdet-d0 … d7x parameter table,
  * ``utils/global_params.py:144-197`` the detection defaults,
  * ``utils/global_params.py:200-212`` ``get_efficientdet_config`` (incl. the derived
    ``levels_size`` list, ``:206-208``),
  * ``utils/round_filters.py:2-12`` / ``utils/round_repeats.py:3-6`` compound scaling,
  * ``utils/block_args.py:5-12`` the MBConv block-argument record,
  * ``efficientnet/utils/get_feat_sizes.py:4-21`` per-level feature sizes,
  * ``efficientnet/train.py:81-89`` the EfficientNet-B0 base block list.

``Config`` mirrors the reference ``utils/config_class.py:19`` attribute-dict behaviour
(attribute and item access, ``override`` from a dict / ``"a.b=1,c=2"`` string / yaml file)
so host code written against the reference keeps working.
"""
from __future__ import annotations

import ast
import copy
import math
from collections import namedtuple
from typing import Any, Dict, List, Sequence, Tuple

__all__ = [
    "Config", "EfficientDetBlockArgs", "MODEL_PARAMS", "default_detection_configs",
    "get_efficientdet_config", "round_filters", "round_repeats", "get_feat_sizes",
    "efficientnet_b0_blocks", "BlockSpec", "expand_blocks",
]

# ---------------------------------------------------------------------------
# block args (utils/block_args.py:5-12): same field names and all-None defaults
# ---------------------------------------------------------------------------
EfficientDetBlockArgs = namedtuple(
    "EfficientDetBlockArgs",
    ["num_repeat", "kernel_size", "strides", "expand_ratio",
     "input_filters", "output_filters", "se_ratio"],
    defaults=(None,) * 7)


def efficientnet_b0_blocks() -> List[EfficientDetBlockArgs]:
    """The seven B0 stage descriptors used by ``efficientnet/train.py:81-89``."""
    table = [  # repeats, k, stride, expand, in, out, se
        (1, 3, 1, 1, 32, 16), (2, 3, 2, 6, 16, 24), (2, 5, 2, 6, 24, 40),
        (3, 3, 2, 6, 40, 80), (3, 5, 1, 6, 80, 112), (4, 5, 2, 6, 112, 192),
        (1, 3, 1, 6, 192, 320),
    ]
    return [EfficientDetBlockArgs(r, k, (s, s), e, i, o, 0.25) for r, k, s, e, i, o in table]


# ---------------------------------------------------------------------------
# compound scaling helpers
# ---------------------------------------------------------------------------
def round_filters(filters: float, width_coefficient: float, depth_divisor: int) -> int:
    """Channel count after width scaling (``utils/round_filters.py:2-12``).

    Scales by the width multiplier, rounds to the nearest multiple of the divisor (never
    below the divisor) and adds one divisor back if rounding lost more than 10 %.
    """
    scaled = filters * width_coefficient
    out = max(depth_divisor, int(scaled + depth_divisor / 2) // depth_divisor * depth_divisor)
    if out < 0.9 * scaled:
        out += depth_divisor
    return int(out)


def round_repeats(repeats: int, global_params) -> int:
    """Block repeat count after depth scaling (``utils/round_repeats.py:3-6``): ceil(d*r)."""
    return int(math.ceil(global_params.depth_coefficient * repeats))


def get_feat_sizes(image_size: Tuple[int, int], max_level: int) -> List[Tuple[int, int]]:
    """Feature map size per level 0..max_level (``get_feat_sizes.py:4-21``): ceil-halving."""
    h, w = image_size
    sizes = [(h, w)]
    for _ in range(max_level):
        h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        sizes.append((h, w))
    return sizes


# ---------------------------------------------------------------------------
# Config (utils/config_class.py:19-158)
# ---------------------------------------------------------------------------
def _parse_scalar(text: str):
    if text in ("true", "false"):
        return text == "true"
    try:
        return ast.literal_eval(text)
    except (ValueError, SyntaxError):
        return text


class Config:
    """Attribute dictionary with nested-dict promotion and override helpers."""

    def __init__(self, config_dict: Dict[str, Any] | None = None):
        self.update(config_dict)

    def __setattr__(self, k, v):
        self.__dict__[k] = Config(v) if isinstance(v, dict) else copy.deepcopy(v)

    def __getattr__(self, k):
        try:
            return self.__dict__[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __getitem__(self, k):
        return self.__dict__[k]

    def __contains__(self, k):
        return k in self.__dict__

    def __repr__(self):
        return repr(self.as_dict())

    def _merge(self, d: Dict[str, Any], allow_new_keys: bool):
        for k, v in (d or {}).items():
            if k not in self.__dict__:
                if not allow_new_keys:
                    raise KeyError(f"Key `{k}` does not exist for overriding.")
                setattr(self, k, v)
                continue
            cur = self.__dict__[k]
            if isinstance(cur, Config) and isinstance(v, (dict, Config)):
                cur._merge(v.as_dict() if isinstance(v, Config) else v, allow_new_keys)
            else:
                setattr(self, k, v)

    def update(self, config_dict):
        self._merge(config_dict, allow_new_keys=True)

    def override(self, config_dict_or_str, allow_new_keys: bool = False):
        if not config_dict_or_str:
            return
        if isinstance(config_dict_or_str, Config):
            d = config_dict_or_str.as_dict()
        elif isinstance(config_dict_or_str, dict):
            d = config_dict_or_str
        elif isinstance(config_dict_or_str, str):
            if config_dict_or_str.endswith((".yaml", ".yml")):
                import yaml
                with open(config_dict_or_str) as f:
                    d = yaml.load(f, Loader=yaml.SafeLoader)
            else:
                d = self.parse_from_str(config_dict_or_str)
        else:
            raise ValueError(f"Unknown value type: {config_dict_or_str!r}")
        self._merge(d, allow_new_keys)

    @staticmethod
    def parse_from_str(text: str) -> Dict[str, Any]:
        """``"a.b=1,c=[2,3]"`` → nested dict (``config_class.py`` string override form)."""
        out: Dict[str, Any] = {}
        parts: List[str] = []
        depth = 0
        cur = ""
        for ch in text:
            depth += ch in "([{"
            depth -= ch in ")]}"
            if ch == "," and depth == 0:
                parts.append(cur)
                cur = ""
            else:
                cur += ch
        if cur:
            parts.append(cur)
        for kv in parts:
            if not kv.strip():
                continue
            k, v = kv.split("=", 1)
            keys = k.strip().split(".")
            node = out
            for kk in keys[:-1]:
                node = node.setdefault(kk, {})
            node[keys[-1]] = _parse_scalar(v.strip())
        return out

    def as_dict(self) -> Dict[str, Any]:
        return {k: (v.as_dict() if isinstance(v, Config) else copy.deepcopy(v))
                for k, v in self.__dict__.items()}


# ---------------------------------------------------------------------------
# parameter table (utils/global_params.py:4-141)
# ---------------------------------------------------------------------------
def _p(name, backbone, size, fpn, cells, heads, w, d, drop, **extra):
    return dict(name=name, backbone_name=backbone, image_size=size, fpn_num_filters=fpn,
                fpn_cell_repeats=cells, box_class_repeats=heads, width_coefficient=w,
                depth_coefficient=d, dropout_rate=drop, **extra)


MODEL_PARAMS: Dict[str, Dict[str, Any]] = {
    "efficientdet-d0": _p("efficientdet-d0", "efficientnet-b0", 512, 64, 3, 3, 1.0, 1.0, 0.2),
    "efficientdet-d1": _p("efficientdet-d1", "efficientnet-b1", 640, 88, 4, 3, 1.0, 1.1, 0.2),
    "efficientdet-d1-a": _p("efficientdet-d1-a", "efficientnet-b1-a", 640, 88, 4, 3, 0.8, 0.8, 0.2),
    "efficientdet-d2": _p("efficientdet-d2", "efficientnet-b2", 768, 112, 5, 3, 1.1, 1.2, 0.3),
    "efficientdet-d3": _p("efficientdet-d3", "efficientnet-b3", 896, 160, 6, 4, 1.2, 1.4, 0.3),
    "efficientdet-d4": _p("efficientdet-d4", "efficientnet-b4", 1024, 224, 7, 4, 1.4, 1.8, 0.4),
    "efficientdet-d5": _p("efficientdet-d5", "efficientnet-b5", 1280, 288, 7, 4, 1.6, 2.2, 0.4),
    "efficientdet-d6": _p("efficientdet-d6", "efficientnet-b6", 1280, 384, 8, 5, 1.8, 2.6, 0.5,
                          fpn_weight_method="sum"),
    "efficientdet-d7": _p("efficientdet-d7", "efficientnet-b6", 1536, 384, 8, 5, 1.8, 2.6, 0.5,
                          anchor_scale=5.0, fpn_weight_method="sum"),
    "efficientdet-d7x": _p("efficientdet-d7x", "efficientnet-b7", 1536, 384, 8, 5, 2.0, 3.1, 0.5,
                           anchor_scale=4.0, max_level=8, fpn_weight_method="sum"),
}


def default_detection_configs() -> Config:
    """Defaults of ``utils/global_params.py:144-197``."""
    h = Config()
    h.name = ""
    h.backbone_name = ""
    h.batch_norm_momentum = 0.99
    h.batch_norm_epsilon = 1e-3
    h.width_coefficient = 1.0
    h.depth_coefficient = 1.0
    h.dropout_rate = 0.2
    h.depth_divisor = 8
    h.min_level = 3
    h.max_level = 7
    h.image_size = 512
    h.fpn_num_filters = 88
    h.fpn_cell_repeats = 4
    h.fpn_weight_method = "fastattn"   # stored only: the BiFPN path ignores it
    h.box_class_repeats = 3
    h.is_training_bn = True
    h.num_scales = 3
    h.aspect_ratios = [(1.0, 1.0), (1.4, 0.7), (0.7, 1.4)]
    h.anchor_scale = 4.0
    h.num_classes = 81                 # 0 = background
    h.survival_prob = 0.8
    h.alpha = 0.25
    h.gamma = 1.5
    h.nms_configs = {"method": "gaussian", "iou_thresh": None, "score_thresh": None,
                     "sigma": None, "max_nms_inputs": 0, "max_output_size": 1000}
    return h


def get_efficientdet_config(model_name: str = "efficientdet-d4", overrides=None) -> Config:
    """``utils/global_params.py:200-212``; raises ValueError on an unknown name.

    ``overrides`` (dict or "a=1,b=2" string, optional) is applied before ``levels_size`` is
    derived, so e.g. a reduced ``image_size`` for tests yields consistent level sizes."""
    if model_name not in MODEL_PARAMS:
        raise ValueError(f"Unknown model name: {model_name}")
    h = default_detection_configs()
    h.override(MODEL_PARAMS[model_name], allow_new_keys=True)
    if overrides:
        h.override(overrides, allow_new_keys=True)
    sizes = [h.image_size]
    for _ in range(h.max_level):
        sizes.append((sizes[-1] + 1) // 2)
    h.levels_size = sizes
    return h


# ---------------------------------------------------------------------------
# per-block expansion (efficientnet/backbone_model.py:59-93)
# ---------------------------------------------------------------------------
BlockSpec = namedtuple("BlockSpec", ["index", "kernel_size", "stride", "expand_ratio",
                                     "input_filters", "output_filters", "se_filters",
                                     "expanded_filters"])


def expand_blocks(blocks_args: Sequence[EfficientDetBlockArgs], global_params) -> List[BlockSpec]:
    """Unroll stage descriptors into per-block specs exactly as BackboneModel._build does.

    The first block of a stage keeps the stage stride and scaled input width; repeats use
    stride 1 and input = output width.  ``se_filters`` follows ``mb_conv_block.py:98-101``:
    max(1, int(input_filters * se_ratio)) on the *scaled* input width of that block.
    """
    if not isinstance(blocks_args, list):
        raise ValueError("blocks_args should be a list.")
    specs: List[BlockSpec] = []
    for ba in blocks_args:
        assert ba.num_repeat > 0
        cin = round_filters(ba.input_filters, global_params.width_coefficient,
                            global_params.depth_divisor)
        cout = round_filters(ba.output_filters, global_params.width_coefficient,
                             global_params.depth_divisor)
        reps = round_repeats(ba.num_repeat, global_params)
        stride = ba.strides[0] if isinstance(ba.strides, (tuple, list)) else int(ba.strides)
        for r in range(reps):
            i_f = cin if r == 0 else cout
            s = stride if r == 0 else 1
            specs.append(BlockSpec(len(specs), ba.kernel_size, s, ba.expand_ratio, i_f, cout,
                                   max(1, int(i_f * ba.se_ratio)), i_f * ba.expand_ratio))
    return specs
