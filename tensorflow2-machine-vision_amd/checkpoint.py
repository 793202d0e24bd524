"""Keras checkpoint naming and layouts <-> the product's parameter table.

The reference saves ``trained_weights_final.h5`` with ``model.save_weights`` /
``model.load_weights`` (efficientnet/train.py:125-153).  Its variable names come from the layer
names the model builds:

  efficientnet-b0/stem/conv2d/kernel               backbone_model.py:51 + stem (Stem)
  efficientnet-b0/blocks_<i>/conv2d[_<j>]/kernel   mb_conv_block.py:45-51 (get_conv_name)
  .../tpu_batch_normalization[_<j>]/{gamma,beta,moving_mean,moving_variance}   (get_bn_name)
  .../depthwise_conv2d/depthwise_kernel, .../se/conv2d[_1]/{kernel,bias}
  resample_p<l>/{conv2d,bn}/..., fpn_cell_<c>/node_<n>/{WSM, resample_<k>/..., op_after_combine/...}
  class_net/class-<i>/{depthwise_kernel,pointwise_kernel,bias}, class_net/class-<i>-bn-<l>/...
  class_net/class-predict/..., box_net/box-<i>/..., box_net/box-predict/...  (class_net.py:63,68)

The product keeps exactly these names (``EfficientDetNetTrain.state_dict()`` keys; the
oracle derives the same table independently, tests/test_oracle_structure.py), so the map is
the identity on names apart from Keras' ``:0`` suffix.  Layouts differ where the product
stores a kernel in its GEMM / stencil form:

  Keras 1x1 Conv2D kernel           [1, 1, Cin, Cout]  <->  product [Cout, Cin]
  Keras SeparableConv2D pointwise   [1, 1, Cin, Cout]  <->  product [Cout, Cin]
  Keras DepthwiseConv2D / separable depthwise [k, k, C, 1]  <->  product [k*k, C]
  stem kernel [3, 3, 3, 32], biases, BN vectors and the BiFPN fusion weights are unchanged.

Reading the .h5 container itself needs h5py, which is not importable in this image;
``read_h5_weights`` imports it lazily and raises otherwise.  Everything else here works on
plain {name: ndarray} dicts.
"""
from __future__ import annotations

from typing import Dict, Mapping

import numpy as np

__all__ = ["keras_name", "product_name", "to_keras", "from_keras", "keras_state_dict", "load_keras_state_dict",
           "read_h5_weights"]


def product_name(keras_var: str) -> str:
    """'efficientnet-b0/blocks_0/conv2d/kernel:0' -> 'efficientnet-b0/blocks_0/conv2d/kernel'."""
    return keras_var[:-2] if keras_var.endswith(":0") else keras_var


def keras_name(name: str) -> str:
    return name + ":0"


def _kind(name: str, ndim_product: int) -> str:
    leaf = name.rsplit("/", 1)[-1]
    if leaf == "depthwise_kernel":
        return "depthwise"
    if leaf == "pointwise_kernel":
        return "pointwise"
    if leaf == "kernel" and ndim_product == 2:
        return "conv1x1"
    return "same"


def to_keras(name: str, a: np.ndarray) -> np.ndarray:
    """Product layout -> Keras layout for one variable."""
    a = np.asarray(a)
    k = _kind(name, a.ndim)
    if k == "depthwise":
        kk, C = a.shape
        ks = int(round(kk ** 0.5))
        assert ks * ks == kk, (name, a.shape)
        return np.ascontiguousarray(a.reshape(ks, ks, C, 1))
    if k in ("pointwise", "conv1x1"):
        return np.ascontiguousarray(a.T.reshape(1, 1, a.shape[1], a.shape[0]))
    return a.copy()


def from_keras(name: str, a: np.ndarray, product_shape=None) -> np.ndarray:
    """Keras layout -> product layout for one variable (``product_shape`` optional check)."""
    a = np.asarray(a)
    leaf = name.rsplit("/", 1)[-1]
    if leaf == "depthwise_kernel":
        assert a.ndim == 4 and a.shape[3] == 1, (name, a.shape)
        out = a.reshape(a.shape[0] * a.shape[1], a.shape[2])
    elif leaf in ("pointwise_kernel", "kernel") and a.ndim == 4 and a.shape[0] == 1 and a.shape[1] == 1 \
            and not name.endswith("stem/conv2d/kernel"):
        out = a.reshape(a.shape[2], a.shape[3]).T
    else:
        out = a
    out = np.ascontiguousarray(out, dtype=np.float32)
    if product_shape is not None:
        assert tuple(out.shape) == tuple(product_shape), (name, out.shape, product_shape)
    return out


def keras_state_dict(state: Mapping[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Product ``state_dict()`` -> {keras variable name ':0': Keras-layout array}."""
    return {keras_name(n): to_keras(n, v) for n, v in state.items()}


def load_keras_state_dict(model, weights: Mapping[str, np.ndarray], strict: bool = True):
    """Load {keras variable name: Keras-layout array} (``:0`` optional) into ``model``
    (anything with ``state_dict()`` / ``load_state_dict()``, e.g. EfficientDetNetTrain).
    strict: every product variable must be present and no unknown name may appear."""
    cur = model.state_dict()
    sd = {}
    unknown = []
    for kn, v in weights.items():
        n = product_name(kn)
        if n not in cur:
            unknown.append(kn)
            continue
        sd[n] = from_keras(n, v, cur[n].shape)
    missing = [n for n in cur if n not in sd]
    if strict and (unknown or missing):
        raise KeyError(f"checkpoint mismatch: {len(missing)} missing (e.g. {missing[:3]}), "
                       f"{len(unknown)} unknown (e.g. {unknown[:3]})")
    for n in missing:
        sd[n] = cur[n]
    model.load_state_dict(sd)
    return missing, unknown


def read_h5_weights(path: str) -> Dict[str, np.ndarray]:
    """Every dataset of a Keras ``save_weights`` .h5 file keyed by its variable name (needs
    h5py; not importable in this image, so this raises ImportError here)."""
    import h5py  # noqa: F401  (optional dependency)
    out: Dict[str, np.ndarray] = {}
    with h5py.File(path, "r") as f:
        def visit(name, obj):
            if isinstance(obj, h5py.Dataset):
                key = name.split("/", 1)[1] if "/" in name else name  # drop the top-level layer group
                out[key] = np.asarray(obj)
        f.visititems(visit)
    return out
