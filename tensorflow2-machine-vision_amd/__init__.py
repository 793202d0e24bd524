"""MI355X-native EfficientDet hot path (drop-in for tfwcn/tensorflow2-machine-vision's
``ai_api/ai_models/efficientnet`` call()/train_step() surface).

Import as ``import tf2mv_amd`` (repo-root shim; the directory name is not an identifier).
Compute runs in libedet.so (hand-written gfx950 HIP kernels, C-ABI in include/edet.h).
"""
from .config import (Config, EfficientDetBlockArgs, efficientnet_b0_blocks, get_efficientdet_config,
                     get_feat_sizes, round_filters, round_repeats)

__version__ = "0.1.0"


def __getattr__(name):  # lazy: the compute modules need torch + libedet.so
    if name in ("EfficientDetNet", "EfficientDetNetTrain"):
        from . import model
        return getattr(model, name)
    if name in ("Anchors", "Targets"):
        from . import anchors
        return getattr(anchors, name)
    raise AttributeError(name)
