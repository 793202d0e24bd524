"""The oracle's model structure is derived from the config and the reference's construction
rules (oracle/ref_model.py header), independently of the product's model object.  These CPU
tests pin the product's parameter table -- every variable's name, shape and initialiser, and
every BatchNorm -- to that derivation, and check the sampled
initial values against the Keras initialiser moments (utils/conv_kernel_initializer.py:4-25,
keras glorot_uniform, tf.initializers.VarianceScaling)."""
import math

import numpy as np
import pytest

from oracle.ref_model import B0_BLOCKS, block_list, param_specs
from tf2mv_amd.config import efficientnet_b0_blocks, expand_blocks, get_efficientdet_config
from tf2mv_amd.model import EfficientDetNet

CASES = [("efficientdet-d0", {}), ("efficientdet-d0", {"image_size": 128, "num_classes": 5}),
         ("efficientdet-d0", {"image_size": 224}), ("efficientdet-d4", {}), ("efficientdet-d4", {"image_size": 256}),
         ("efficientdet-d2", {}), ("efficientdet-d7", {"image_size": 256})]


def _host_model(name, ov, seed=0):
    return EfficientDetNet(efficientnet_b0_blocks(), get_efficientdet_config(name, ov), dtype="f32", device="cpu",
                           seed=seed)


@pytest.mark.parametrize("name,ov", CASES)
def test_parameter_table_matches_reference_rules(name, ov):
    cfg = get_efficientdet_config(name, ov)
    ref = param_specs(cfg)
    m = _host_model(name, ov)
    prod = {n: (tuple(sp.shape), sp.init) for n, sp in m.P.specs.items()}
    assert set(prod) == set(ref), sorted(set(prod) ^ set(ref))[:10]
    bad = [(n, prod[n], ref[n]) for n in ref if prod[n][0] != tuple(ref[n][0]) or prod[n][1] != ref[n][1]]
    assert not bad, bad[:5]
    assert sorted(ref.bn_names) == sorted(b.name for b in m.P.bns)
    # BN channel counts follow the gamma shapes the oracle derived
    assert all(b.C == ref[b.name + "/gamma"][0][0] for b in m.P.bns)


def test_block_list_matches_product_specs():
    for name in ("efficientdet-d0", "efficientdet-d4", "efficientdet-d7"):
        cfg = get_efficientdet_config(name)
        ob = block_list(cfg, B0_BLOCKS)
        pb = expand_blocks(efficientnet_b0_blocks(), cfg)
        assert [(b["k"], b["s"], b["cin"], b["cout"], b["cin"] * b["e"]) for b in ob] == \
               [(p.kernel_size, p.stride, p.input_filters, p.output_filters, p.expanded_filters) for p in pb]
    assert len(block_list(get_efficientdet_config("efficientdet-d0"))) == 16
    assert len(block_list(get_efficientdet_config("efficientdet-d4"))) == 32


def test_d0_trainable_count():
    ref = param_specs(get_efficientdet_config("efficientdet-d0"))
    assert sum(int(np.prod(s)) for s, _ in ref.values()) == 3874802


def _expected_moments(init):
    kind = init[0]
    if kind == "normal":
        return 0.0, init[1], None
    if kind == "glorot":
        lim = math.sqrt(6.0 / (init[1] + init[2]))
        return 0.0, lim / math.sqrt(3.0), lim
    if kind == "vs_fan_in":  # truncated at 2 sigma_t, sigma_t = sqrt(1/fan)/0.8796: variance 1/fan
        return 0.0, math.sqrt(1.0 / init[1]), 2.0 * math.sqrt(1.0 / init[1]) / 0.87962566103423978
    raise ValueError(init)


def test_initialiser_moments():
    """Sampled initial values: mean, standard deviation and support per Keras initialiser
    (a21).  Checked on every tensor with at least 4096 values; bounds are 6 sigma of the
    sampling error of the mean and a 5 % band on the standard deviation."""
    m = _host_model("efficientdet-d0", {}, seed=3)
    sd = m.state_dict()
    checked = 0
    for n, sp in m.P.specs.items():
        v = sd[n].astype(np.float64).ravel()
        if sp.init[0] == "const":
            assert np.all(v == np.float64(np.float32(sp.init[1]))), n
            continue
        if v.size < 4096:
            continue
        mu, sigma, bound = _expected_moments(sp.init)
        assert abs(v.mean() - mu) < 6 * sigma / math.sqrt(v.size), (n, v.mean(), sigma)
        assert abs(v.std() / sigma - 1) < 0.05, (n, v.std(), sigma)
        if bound is not None:
            assert np.abs(v).max() <= bound * (1 + 1e-6), (n, np.abs(v).max(), bound)
        checked += 1
    assert checked > 50
    # the fans the reference rules give for a few named variables
    s = m.P.specs
    assert s["efficientnet-b0/blocks_1/depthwise_conv2d/depthwise_kernel"].init == ("normal", math.sqrt(2.0 / 9))
    assert s["efficientnet-b0/stem/conv2d/kernel"].init == ("normal", math.sqrt(2.0 / (9 * 32)))
    assert s["class_net/class-predict/depthwise_kernel"].init == ("vs_fan_in", 9 * 64)
    assert s["fpn_cell_0/node_0/op_after_combine/separable_conv2d/depthwise_kernel"].init == ("glorot", 9 * 64, 9)
    assert s["class_net/class-predict/bias"].init == ("const", -math.log(99.0))
