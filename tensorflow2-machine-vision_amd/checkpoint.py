"""Keras checkpoint naming and layouts <-> the product's parameter table.

The reference saves ``trained_weights_final.h5`` with ``model.save_weights`` /
``model.load_weights`` (efficientnet/train.py:125-153), after building the model eagerly with
``model(tf.ones(...))`` (train.py:126).  A variable's name is the chain of the layer names it
was created under, plus ``:0``.  Explicitly named layers keep their names:

  efficientnet-b0/stem/conv2d/kernel               backbone_model.py:51 + stem (Stem)
  efficientnet-b0/blocks_<i>/conv2d[_<j>]/kernel   mb_conv_block.py:45-51 (get_conv_name)
  .../tpu_batch_normalization[_<j>]/{gamma,beta,moving_mean,moving_variance}   (get_bn_name)
  .../depthwise_conv2d/depthwise_kernel, .../se/conv2d[_1]/{kernel,bias}
  resample_p<l>/{conv2d,bn}/...                    efficientdet_net.py:27-33
  class_net/class-<i>/{depthwise_kernel,pointwise_kernel,bias}, class_net/class-<i>-bn-<l>/...
  class_net/class-predict/..., box_net/box-<i>/..., box_net/box-predict/...  (class_net.py:63,68)

The BiFPN is different.  ``BiFPN`` (efficientdet_net.py:37-41), ``BiFPNNode`` (bifpn.py:78-87),
the node's ``ResampleFeatureMap`` layers and ``OpAfterCombine`` (bifpn.py:56) and the latter's
``SeparableConv2D`` / ``BatchNormalization`` (bifpn.py:16-22) get no name, so Keras names them
from the class name in snake case, made unique by a per-process counter in construction order
(first ``bi_fpn``, then ``bi_fpn_1``, ...).  Each edge weight is its own scalar ``WSM_<k>``
(bifpn.py:45-54).  For cell c, node j of a BiFPN with J nodes per cell, g = c*J + j:

  bi_fpn[_c]/bi_fpn_node[_g]/WSM_<k>                                      (scalar, k < n_in)
  bi_fpn[_c]/bi_fpn_node[_g]/resample_feature_map[_r]/{conv2d,bn}/...     r = inputs of earlier nodes + k
  bi_fpn[_c]/bi_fpn_node[_g]/op_after_combine[_g]/separable_conv2d[_g]/{depthwise_kernel,pointwise_kernel,bias}
  bi_fpn[_c]/bi_fpn_node[_g]/op_after_combine[_g]/batch_normalization[_g]/{gamma,beta,moving_mean,moving_variance}

(every other layer of the model that could share these counters is explicitly named, so the
counters start at zero in a fresh process, as in train.py).  The product stores these under
``fpn_cell_<c>/node_<j>/...`` with the node's weights as one ``WSM`` vector of shape (n_in,);
``keras_name_map`` translates.  These BiFPN names follow Keras' naming rule and the
reference's construction order; no reference-written .h5 is available here (TensorFlow and
h5py are absent), so they are **parity-unpinned** (tests/test_checkpoint_names.py derives them
independently from the reference's construction order).

Layouts differ where the product stores a kernel in its GEMM / stencil form:

  Keras 1x1 Conv2D kernel           [1, 1, Cin, Cout]  <->  product [Cout, Cin]
  Keras SeparableConv2D pointwise   [1, 1, Cin, Cout]  <->  product [Cout, Cin]
  Keras DepthwiseConv2D / separable depthwise [k, k, C, 1]  <->  product [k*k, C]
  stem kernel [3, 3, 3, 32], biases and BN vectors are unchanged; a node's WSM vector is
  split into / assembled from its scalars.

Reading the .h5 container itself needs h5py, which is not importable in this image;
``read_h5_weights`` imports it lazily and raises otherwise.  Everything else here works on
plain {name: ndarray} dicts.
"""
from __future__ import annotations

import re
from typing import Dict, Iterable, Mapping, Optional, Tuple

import numpy as np

__all__ = ["keras_name", "product_name", "keras_name_map", "to_keras", "from_keras", "keras_state_dict",
           "load_keras_state_dict", "read_h5_weights"]

_FPN = re.compile(r"^fpn_cell_(\d+)/node_(\d+)/(.*)$")


def _uniq(base: str, i: int) -> str:
    """Keras' zero-based unique layer name: base, base_1, base_2, ..."""
    return base if i == 0 else f"{base}_{i}"


def keras_name_map(names: Iterable[str], wsm_sizes: Optional[Mapping[str, int]] = None) -> Dict[str, object]:
    """product name -> Keras variable name (without ``:0``) for every name in ``names``.
    A node's ``WSM`` vector maps to the list of its scalars' names.  ``wsm_sizes`` gives
    n_in per ``.../WSM`` name (from the state dict's shapes); every node needs it."""
    names = list(names)
    nodes = {}  # (cell, node) -> n_in
    for n in names:
        m = _FPN.match(n)
        if m:
            key = (int(m.group(1)), int(m.group(2)))
            nodes.setdefault(key, None)
            if m.group(3) == "WSM":
                if wsm_sizes is None or n not in wsm_sizes:
                    raise ValueError(f"keras_name_map: the size of {n} is needed")
                nodes[key] = int(wsm_sizes[n])
    if any(v is None for v in nodes.values()):
        raise ValueError("keras_name_map: a BiFPN node without WSM weights")
    per_cell = 1 + max((j for _, j in nodes), default=-1)
    # construction order (bifpn.py:78-87, 95-116): cell by cell, node by node; the resample
    # layers of a node are numbered after those of every earlier node
    first_rfm, r = {}, 0
    for key in sorted(nodes):
        first_rfm[key] = r
        r += nodes[key]
    out: Dict[str, object] = {}
    for n in names:
        m = _FPN.match(n)
        if not m:
            out[n] = n
            continue
        c, j, rest = int(m.group(1)), int(m.group(2)), m.group(3)
        g = c * per_cell + j
        pre = f"{_uniq('bi_fpn', c)}/{_uniq('bi_fpn_node', g)}"
        if rest == "WSM":
            out[n] = [f"{pre}/WSM_{k}" for k in range(nodes[(c, j)])]
            continue
        mr = re.match(r"^resample_(\d+)/(.*)$", rest)
        if mr:
            k = int(mr.group(1))
            out[n] = f"{pre}/{_uniq('resample_feature_map', first_rfm[(c, j)] + k)}/{mr.group(2)}"
            continue
        mo = re.match(r"^op_after_combine/(separable_conv2d|batch_normalization)/(.*)$", rest)
        if not mo:
            raise ValueError(f"keras_name_map: unexpected BiFPN variable {n}")
        out[n] = f"{pre}/{_uniq('op_after_combine', g)}/{_uniq(mo.group(1), g)}/{mo.group(2)}"
    return out


def product_name(keras_var: str) -> str:
    """Strip Keras' ``:0`` suffix (names outside the BiFPN are the product's own)."""
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
    """Product layout -> Keras layout for one variable (a WSM vector stays a vector here;
    ``keras_state_dict`` splits it into scalars)."""
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


def _wsm_sizes(state: Mapping[str, np.ndarray]) -> Dict[str, int]:
    return {n: int(np.asarray(v).size) for n, v in state.items() if n.endswith("/WSM")}


def keras_state_dict(state: Mapping[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Product ``state_dict()`` -> {Keras variable name ':0': Keras-layout array}; a BiFPN
    node's WSM vector becomes its scalars WSM_0..WSM_{n-1} (shape ())."""
    nm = keras_name_map(state.keys(), _wsm_sizes(state))
    out: Dict[str, np.ndarray] = {}
    for n, v in state.items():
        k = nm[n]
        if isinstance(k, list):
            v = np.asarray(v, dtype=np.float32).reshape(-1)
            for i, kk in enumerate(k):
                out[keras_name(kk)] = np.array(v[i], dtype=np.float32)
        else:
            out[keras_name(k)] = to_keras(n, v)
    return out


def load_keras_state_dict(model, weights: Mapping[str, np.ndarray], strict: bool = True):
    """Load {Keras variable name: Keras-layout array} (``:0`` optional) into ``model``
    (anything with ``state_dict()`` / ``load_state_dict()``, e.g. EfficientDetNetTrain).
    BiFPN variables are matched under the reference's Keras names (``keras_name_map``).
    strict: every product variable must be present and no unknown name may appear.
    Returns (missing product names, unknown Keras names)."""
    cur = model.state_dict()
    nm = keras_name_map(cur.keys(), _wsm_sizes(cur))
    inv: Dict[str, Tuple[str, int]] = {}  # keras name -> (product name, WSM index or -1)
    for n, k in nm.items():
        if isinstance(k, list):
            for i, kk in enumerate(k):
                inv[kk] = (n, i)
        else:
            inv[k] = (n, -1)
    sd: Dict[str, np.ndarray] = {}
    wsm: Dict[str, Dict[int, float]] = {}
    unknown = []
    for kn, v in weights.items():
        hit = inv.get(product_name(kn))
        if hit is None:
            unknown.append(kn)
            continue
        n, i = hit
        if i >= 0:
            a = np.asarray(v, dtype=np.float32)
            assert a.size == 1, (kn, a.shape)
            wsm.setdefault(n, {})[i] = float(a.reshape(()))
        else:
            sd[n] = from_keras(n, v, cur[n].shape)
    for n, parts in wsm.items():
        if len(parts) == len(nm[n]):
            sd[n] = np.array([parts[i] for i in range(len(parts))], dtype=np.float32)
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
