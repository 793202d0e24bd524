"""Model-level parity: the full EfficientDet-D0 topology through
libedet vs the fp64 CPU oracle (oracle/ref_model.py) on identical parameters and inputs.

Reduced size for oracle speed: D0 topology at 128x128, batch 2, 5 classes; drop-connect
masks injected (the reference draws them randomly).  fp32 storage: outputs within 1e-3
relative (north_star tolerance).  The bf16 train step is pinned at the headline geometry
(512^2, NC=81) against the oracle with bf16 storage emulated forward and backward
(test_headline_gpu.py::test_d0_512_nc81_train_step_bf16_emulated, which replaced round 5's
cosine-against-a-noise-floor bar here); the bf16 forward likewise in test_headline_gpu.py.
"""
import numpy as np
import pytest
import torch

from oracle.ref_model import RefEfficientDet, ref_train_step
from tf2mv_amd.anchors import Anchors
from tf2mv_amd.config import efficientnet_b0_blocks, get_efficientdet_config
from tf2mv_amd.model import EfficientDetNet, EfficientDetNetTrain

pytestmark = pytest.mark.gpu
SIZE, B, NC = 128, 2, 5


def cfg(survival=0.8):
    return get_efficientdet_config("efficientdet-d0", {"image_size": SIZE, "num_classes": NC, "survival_prob": survival})


def synth(seed=0):
    rng = np.random.default_rng(seed)
    x = rng.random((B, SIZE, SIZE, 3), dtype=np.float32)
    G = 6
    boxes = np.zeros((B, G, 4), np.float32)
    cls = np.zeros((B, G), np.int32)
    n = np.full(B, G, np.int32)
    for b in range(B):
        for k in range(G):
            s = np.exp(rng.uniform(np.log(12), np.log(90)))
            ar = rng.uniform(0.5, 2)
            h, w = s * np.sqrt(ar), s / np.sqrt(ar)
            cy, cx = rng.uniform(0, SIZE, 2)
            boxes[b, k] = [cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2]
            cls[b, k] = rng.integers(1, NC)
    return x, boxes, cls, n


def make_targets(model, anchors, boxes, cls, n):
    t = anchors.generate_targets_batched(torch.tensor(boxes), torch.tensor(cls), torch.tensor(n))
    pyr = t.pyr
    yb, yc, ym = [], [], []
    tb, tc, tm = t.box.cpu().numpy(), t.cls.cpu().numpy(), t.mask.cpu().numpy()
    for s, l in enumerate(model.levels):
        H, W = model.level_hw[l]
        sl = pyr.seg_slice(s)
        yb.append(tb[sl].reshape(B, H, W, 9, 4))
        yc.append(np.eye(NC, dtype=np.float32)[tc[sl]].reshape(B, H, W, 9, NC))
        ym.append(tm[sl].reshape(B, H, W, 9, 1).astype(bool))
    return t, yb, yc, ym


def fixed_masks(model, seed=3):
    rng = np.random.default_rng(seed)
    reps = model.cfg.box_class_repeats - 1
    m = rng.choice([0.0, 1.25], size=(2, reps, len(model.levels), B), p=[0.3, 0.7]).astype(np.float32)
    return m


def rel_err(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def test_bifpn_topology_matches_reference():
    """bifpn.py:108-117: P6'=(P6,P7) P5'=(P5,P6') P4'=(P4,P5') P3''=(P3,P4') P4''=(P4,P4',P3'')
    P5''=(P5,P5',P4'') P6''=(P6,P6',P5'') P7''=(P7,P6'') with ids 0..4 inputs, 5.. nodes."""
    m = EfficientDetNet(efficientnet_b0_blocks(), cfg(), dtype="f32")
    assert [n["inputs"] for n in m.cells[0]] == [[3, 4], [2, 5], [1, 6], [0, 7], [1, 7, 8], [2, 6, 9], [3, 5, 10], [4, 11]]
    assert [n["level"] for n in m.cells[0]] == [6, 5, 4, 3, 4, 5, 6, 7]
    # trainable parameter count of full D0 (3,874,802)
    d0 = EfficientDetNet(efficientnet_b0_blocks(), get_efficientdet_config("efficientdet-d0"), dtype="f32")
    assert d0.P.n_trainable == 3874802


@pytest.mark.parametrize("training", [True, False])
def test_forward_parity_fp32(training):
    m = EfficientDetNet(efficientnet_b0_blocks(), cfg(), dtype="f32", seed=1)
    x, *_ = synth(1)
    if not training:  # non-trivial moving statistics
        sd = m.state_dict()
        rng = np.random.default_rng(7)
        for k in sd:
            if k.endswith("moving_mean"):
                sd[k] = rng.normal(0, 0.3, sd[k].shape).astype(np.float32)
            elif k.endswith("moving_variance"):
                sd[k] = rng.uniform(0.5, 2.0, sd[k].shape).astype(np.float32)
        m.load_state_dict(sd)
    fm = fixed_masks(m)
    masks = {"class_net": torch.tensor(fm[0]).cuda(), "box_net": torch.tensor(fm[1]).cuda()}
    boxes, classes = m.call(torch.tensor(x).cuda(), training=training, masks=masks if training else None)
    ref = RefEfficientDet(m.cfg, m.state_dict())
    rmasks = {"class_net": fm[0], "box_net": fm[1]}
    rb, rc = ref.forward(x, training, rmasks if training else None)
    for l in range(5):
        assert boxes[l].shape == tuple(rb[l].shape) and classes[l].shape == tuple(rc[l].shape)
        assert rel_err(boxes[l].cpu(), rb[l].detach()) < 1e-3, l
        assert rel_err(classes[l].cpu(), rc[l].detach()) < 1e-3, l


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_inference_fused_squeeze_equals_separate_pass(dtype):
    """call(training=False) takes the SE squeeze from the depthwise epilogue
    (edet_dwconv_fwd_squeeze); the same model with the separate edet_se_squeeze pass gives the
    same outputs (the two differ only in the fp32 partial-sum order of the squeeze, and in the
    depthwise form of a few layers: within fp32 rounding, a few bf16 ulp)."""
    m = EfficientDetNet(efficientnet_b0_blocks(), cfg(), dtype=dtype, seed=3)
    sd = m.state_dict()
    rng = np.random.default_rng(8)
    for k in sd:
        if k.endswith("moving_mean"):
            sd[k] = rng.normal(0, 0.3, sd[k].shape).astype(np.float32)
        elif k.endswith("moving_variance"):
            sd[k] = rng.uniform(0.5, 2.0, sd[k].shape).astype(np.float32)
    m.load_state_dict(sd)
    x = torch.tensor(synth(2)[0]).cuda()
    outs = []
    for fused in (True, False):
        m.fused_squeeze = fused
        b, c = m.call(x, training=False)
        outs.append([t.float().cpu().clone() for t in list(b) + list(c)])
    tol = 1e-4 if dtype == "f32" else 3e-2
    for a, r in zip(*outs):
        assert rel_err(a, r) < tol


def _train_model(dtype, seed=1):
    c = cfg()
    anchors = Anchors(c.min_level, c.max_level, (SIZE, SIZE), c.num_scales, c.aspect_ratios, c.anchor_scale)
    m = EfficientDetNetTrain(efficientnet_b0_blocks(), c, anchors, dtype=dtype, seed=seed,
                             lr_schedule={"fixed_lr": 0.01})
    return m, anchors


def test_train_step_parity_fp32():
    m, anchors = _train_model("f32")
    x, boxes, cls, n = synth(2)
    t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
    fm = fixed_masks(m)
    m.fixed_masks = {"class_net": torch.tensor(fm[0]).cuda(), "box_net": torch.tensor(fm[1]).cuda()}
    sd0 = m.state_dict()
    ref = RefEfficientDet(m.cfg, sd0)
    loss_r, gn_r, new_r, grads_r, st, parts = ref_train_step(ref, x, yb, yc, ym, {"class_net": fm[0], "box_net": fm[1]},
                                                             lr=0.01)
    out = m.train_step((torch.tensor(x).cuda(), t))
    loss, gn = float(out["loss"]), float(out["gnorm"])
    assert abs(loss - float(loss_r)) / float(loss_r) < 1e-4, (loss, float(loss_r))
    assert abs(gn - float(gn_r)) / float(gn_r) < 1e-3, (gn, float(gn_r))
    g = m.P.grads_dict()
    gnorm_r = float(gn_r)
    bad = []
    for k, gr in grads_r.items():
        gg = torch.tensor(g[k], dtype=torch.float64)
        if m.P.specs[k].l2:
            gg = gg + 4e-5 * torch.tensor(sd0[k], dtype=torch.float64)
        err = float((gg - gr).norm())
        if err > 1e-3 * float(gr.norm()) + 1e-6 * gnorm_r:
            bad.append((k, err, float(gr.norm())))
    assert not bad, bad[:10]
    sd1 = m.state_dict()
    for k, v in new_r.items():
        np.testing.assert_allclose(sd1[k], v.numpy(), rtol=1e-3, atol=1e-5, err_msg=k)


def test_bn_backward_folds_equal_unfused_path():
    """the BN-backward folds (the input BatchNorm's sums taken inside the kernel that
    produces its gradient) must give the gradients of the unfused path (reduce + apply passes)
    on the whole model.  Same weights, inputs, masks and batch statistics; per-tensor gradients
    within fp32 summation-order noise."""
    from tf2mv_amd import ops
    m, anchors = _train_model("f32")
    x, boxes, cls, n = synth(5)
    t, *_ = make_targets(m, anchors, boxes, cls, n)
    m.fixed_masks = {"class_net": torch.tensor(fixed_masks(m)[0]).cuda(), "box_net": torch.tensor(fixed_masks(m)[1]).cuda()}
    xd = torch.tensor(x).cuda()
    saved = {k: getattr(ops, k) for k in ops.FOLD_SWITCHES}
    grads = []
    try:
        for on in (True, False):
            for k in ops.FOLD_SWITCHES:
                setattr(ops, k, on)
            m.forward_backward((xd, t))
            torch.cuda.synchronize()
            grads.append(m.P.g.clone())
    finally:
        for k, v in saved.items():
            setattr(ops, k, v)
    a, b = grads
    gn = float(b.norm())
    bad = []
    for k, sp in m.P.specs.items():
        ga, gb = a[sp.offset: sp.offset + sp.size].double(), b[sp.offset: sp.offset + sp.size].double()
        err = float((ga - gb).norm())
        if err > 1e-3 * float(gb.norm()) + 1e-6 * gn:
            bad.append((k, err, float(gb.norm())))
    assert not bad, bad[:10]


def test_train_step_reference_format_equals_compact():
    m, anchors = _train_model("f32")
    x, boxes, cls, n = synth(4)
    t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
    m.fixed_masks = {k: torch.ones(2, 5, B).cuda() for k in ("class_net", "box_net")}
    sd0 = m.state_dict()
    l1 = float(m.train_step((torch.tensor(x).cuda(), t))["loss"])
    g1 = m.P.g.clone()
    m.load_state_dict(sd0)
    data = (torch.tensor(x).cuda(), tuple(torch.tensor(a).cuda() for a in yb), tuple(torch.tensor(a).cuda() for a in yc),
            tuple(torch.tensor(a).cuda() for a in ym))
    l2 = float(m.train_step(data)["loss"])
    # identical inputs; fp32 atomics (BN statistics, weight gradients) are order-dependent
    assert abs(l1 - l2) <= 1e-5 * abs(l1)
    for k, sp in m.P.specs.items():
        a, b = g1[sp.offset: sp.offset + sp.size], m.P.g[sp.offset: sp.offset + sp.size]
        assert float((a - b).norm()) <= 1e-3 * float(a.norm()) + 1e-6 * float(g1.norm()), k


def test_training_reduces_loss_bf16():
    m, anchors = _train_model("bf16", seed=3)
    x, boxes, cls, n = synth(6)
    t, *_ = make_targets(m, anchors, boxes, cls, n)
    xs = torch.tensor(x).cuda()
    losses = [float(m.train_step((xs, t))["loss"]) for _ in range(8)]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses


def test_skip_nonfinite_step_leaves_weights_and_moving_stats():
    """SURVEY §5 failure detection at model level: with skip_nonfinite a step on a
    NaN input is reported as skipped and leaves the weights, optimizer slots, step counter AND
    the BN moving statistics unchanged (the batch statistics of that step are NaN); the next
    finite step applies normally."""
    c = cfg()
    anchors = Anchors(c.min_level, c.max_level, (SIZE, SIZE), c.num_scales, c.aspect_ratios, c.anchor_scale)
    m = EfficientDetNetTrain(efficientnet_b0_blocks(), c, anchors, dtype="bf16", seed=2,
                             lr_schedule={"fixed_lr": 0.01}, skip_nonfinite=True)
    x, boxes, cls, n = synth(4)
    t, *_ = make_targets(m, anchors, boxes, cls, n)
    xs = torch.tensor(x).cuda()
    m.train_step((xs, t))  # one finite step: non-trivial moving statistics and momentum
    torch.cuda.synchronize()
    P = m.P
    before = [a.clone() for a in (P.w, P.v, P.ema, P.bn_mm, P.bn_mv, m.step_counter)]
    bad = xs.clone()
    bad[0, 5, 7, 1] = float("nan")
    out = m.train_step((bad, t))
    torch.cuda.synchronize()
    assert float(out["skipped"]) == 1.0 and not np.isfinite(float(out["gnorm"]))
    for a, b in zip((P.w, P.v, P.ema, P.bn_mm, P.bn_mv, m.step_counter), before):
        assert torch.equal(a, b)
    out = m.train_step((xs, t))
    torch.cuda.synchronize()
    assert float(out["skipped"]) == 0.0 and np.isfinite(float(out["loss"]))
    assert not torch.equal(P.bn_mm, before[3]) and bool(torch.isfinite(P.bn_mm).all())


def test_dp_two_identical_replicas_equal_double_batch():
    """Data-parallel math on the HIP path: a world-size-2 replica whose N+ and
    gradient all-reduces see two identical replicas (x2) must equal the single-GPU step on the
    doubled batch [x, x] (identical shards -> per-replica BN == full-batch BN).  The real
    two-process collective plumbing is covered over gloo in tests/test_dp_gloo.py."""
    c = cfg()
    anchors = Anchors(c.min_level, c.max_level, (SIZE, SIZE), c.num_scales, c.aspect_ratios, c.anchor_scale)
    x, boxes, cls, n = synth(6)
    fm = torch.tensor(np.ones((2, c.box_class_repeats - 1, 5, B), np.float32))
    dbl = lambda t: t.mul_(2.0)  # noqa: E731  (SUM over two identical replicas)
    rep = EfficientDetNetTrain(efficientnet_b0_blocks(), c, anchors, dtype="f32", seed=1, world_size=2,
                               grad_allreduce=dbl, npos_allreduce=dbl, lr_schedule={"fixed_lr": 0.01})
    full = EfficientDetNetTrain(efficientnet_b0_blocks(), c, anchors, dtype="f32", seed=1,
                                lr_schedule={"fixed_lr": 0.01})
    rep.fixed_masks = {"class_net": fm[0].cuda(), "box_net": fm[1].cuda()}
    full.fixed_masks = {"class_net": torch.cat([fm[0], fm[0]], -1).cuda(), "box_net": torch.cat([fm[1], fm[1]], -1).cuda()}
    t1 = anchors.generate_targets_batched(torch.tensor(boxes), torch.tensor(cls), torch.tensor(n))
    t2 = anchors.generate_targets_batched(torch.tensor(np.concatenate([boxes, boxes])),
                                          torch.tensor(np.concatenate([cls, cls])), torch.tensor(np.concatenate([n, n])))
    rep.forward_backward((torch.tensor(x).cuda(), t1))
    rep.grad_allreduce(rep.P.g)
    full.forward_backward((torch.tensor(np.concatenate([x, x])).cuda(), t2))
    torch.cuda.synchronize()
    l_rep, l_full = 2 * float(rep.scalars[0]), float(full.scalars[0])
    assert abs(l_rep - l_full) <= 1e-5 * abs(l_full), (l_rep, l_full)
    assert float(rep.scalars[5]) == float(full.scalars[5])  # global N+
    ga, gb = rep.P.grads_dict(), full.P.grads_dict()
    gmax = max(np.linalg.norm(v) for v in gb.values())
    bad = [k for k in gb if np.linalg.norm(ga[k] - gb[k]) > 1e-3 * np.linalg.norm(gb[k]) + 1e-6 * gmax]
    assert not bad, bad[:8]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_forward_is_reproducible(dtype):
    """Every forward reduction that feeds later layers (BN statistics, SE squeeze) sums across
    blocks in fp64, so two identical steps produce bit-identical forward values (loss,
    statistics); before, 1-ulp atomics-order noise flipped max-pool near-ties between runs and
    moved the gradient by percents.  Weight gradients still use fp32 atomics: close, not equal."""
    m, anchors = _train_model(dtype)
    x, boxes, cls, n = synth(4)
    t, *_ = make_targets(m, anchors, boxes, cls, n)
    m.fixed_masks = {k: torch.ones(2, 5, B).cuda() for k in ("class_net", "box_net")}
    sd0 = m.state_dict()
    xs = torch.tensor(x).cuda()
    outs = []
    for _ in range(3):
        m.load_state_dict(sd0)
        m.train_step((xs, t))
        torch.cuda.synchronize()
        outs.append((m.P.bn_tstats.clone(), m.level_parts.clone(), m.P.g.clone()))
    for st, parts, g in outs[1:]:
        # fp64 cross-block order noise (~1e-16) is all that may differ in the statistics
        assert float(((st - outs[0][0]).abs() / (outs[0][0].abs() + 1e-30)).max()) < 1e-12
        assert torch.allclose(parts[:5], outs[0][1][:5], rtol=1e-6, atol=0)
        assert float((g - outs[0][2]).norm()) <= 1e-4 * float(outs[0][2].norm())


def test_test_step_loss_and_map():
    """test_step (efficientdet_net_train.py:135-169): inference-mode loss (with the L2 term)
    within 1e-4 of the oracle; the per-image mAP is the reference's metric on the GPU
    detections, recomputed here from the oracle NMS over the GPU's own outputs."""
    from oracle import ref_anchors as RA
    from tf2mv_amd import metrics
    m, anchors = _train_model("f32")
    x, boxes, cls, n = synth(4)
    t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
    data = (torch.tensor(x).cuda(), torch.tensor(boxes), torch.tensor(cls),
            [torch.tensor(v) for v in yb], [torch.tensor(v) for v in yc], [torch.tensor(v) for v in ym])
    out = m.test_step(data)
    ref = RefEfficientDet(m.cfg, m.state_dict())
    with torch.no_grad():
        rb, rc = ref.forward(x, False)
        rloss, _ = ref.detection_loss(rb, rc, yb, yc, ym)
    assert abs(out["loss"] - float(rloss)) / float(rloss) < 1e-4, (out["loss"], float(rloss))
    # the detections behind the mAP: oracle NMS on the GPU's decoded boxes and logits
    bo, co = m.call(torch.tensor(x).cuda(), training=False)
    dec = anchors.convert_outputs_boxes(bo)
    want = 0.0
    for b in range(B):
        pb, pc, ps = RA.convert_outputs_one([d[b].cpu().numpy() for d in dec], [c[b].float().cpu().numpy() for c in co])
        pred = np.concatenate([pb, pc[:, None], ps[:, None]], -1)
        gt = np.concatenate([boxes[b], cls[b][:, None]], -1)
        want += metrics.get_map_one(gt, pred, NC, 0.5)
    assert 0.0 <= out["mAP"] <= 1.0
    assert out["mAP"] == pytest.approx(want / B, abs=1e-12)


@pytest.mark.parametrize("training", [False, True])
def test_backbone_b0_224_parity_fp32(training):
    """BASELINE config 2's path (EfficientNet-B0 backbone at 224x224): BackboneModel.call's
    [features, reduction_1..5] within 1e-3 relative of the oracle."""
    c = get_efficientdet_config("efficientdet-d0", {"image_size": 224, "num_classes": NC})
    m = EfficientDetNet(efficientnet_b0_blocks(), c, dtype="f32", seed=5)
    x = np.random.default_rng(5).random((2, 224, 224, 3), dtype=np.float32)
    outs = m.backbone(torch.tensor(x).cuda(), training=training)
    ref = RefEfficientDet(m.cfg, m.state_dict()).backbone(x, training)
    assert [tuple(o.shape) for o in outs] == [(2, 7, 7, 320), (2, 112, 112, 16), (2, 56, 56, 24), (2, 28, 28, 40),
                                               (2, 14, 14, 112), (2, 7, 7, 320)]
    for o, r in zip(outs, ref):
        assert rel_err(o.cpu(), r) < 1e-3


def test_d4_topology_forward_parity_fp32():
    """BASELINE config 5's model (EfficientDet-D4: width 1.4, depth 1.8, 224-channel BiFPN x 7
    cells, 4 head repeats) at a reduced 256x256 input, inference mode, vs the oracle."""
    c = get_efficientdet_config("efficientdet-d4", {"image_size": 256, "num_classes": NC, "survival_prob": None})
    m = EfficientDetNet(efficientnet_b0_blocks(), c, dtype="f32", seed=6)
    assert len(m.specs) == 32 and m.F == 224 and len(m.cells) == 7
    x = np.random.default_rng(6).random((1, 256, 256, 3), dtype=np.float32)
    boxes, classes = m.call(torch.tensor(x).cuda(), training=False)
    rb, rc = RefEfficientDet(m.cfg, m.state_dict()).forward(x, False)
    for l in range(5):
        assert rel_err(boxes[l].cpu(), rb[l].detach()) < 1e-3, l
        assert rel_err(classes[l].cpu(), rc[l].detach()) < 1e-3, l


def test_keras_checkpoint_roundtrip_on_product():
    """§8(f) row 4: the product's parameter table written in Keras names/layouts and loaded
    back (checkpoint.py) reproduces every variable, BN moving statistics included, and the
    forward output bit for bit."""
    from tf2mv_amd import checkpoint as CK
    m, _ = _train_model("f32", seed=3)
    sd = m.state_dict()
    kr = CK.keras_state_dict(sd)
    assert kr["efficientnet-b0/blocks_1/conv2d/kernel:0"].shape[:2] == (1, 1)
    x = torch.randn(1, SIZE, SIZE, 3).cuda()
    b0, c0 = m.call(x, training=False)
    b0 = [t.clone() for t in b0]
    m2, _ = _train_model("f32", seed=4)
    missing, unknown = CK.load_keras_state_dict(m2, kr)
    assert not missing and not unknown
    sd2 = m2.state_dict()
    for k in sd:
        np.testing.assert_array_equal(sd2[k], sd[k], err_msg=k)
    b1, _ = m2.call(x, training=False)
    for u, v in zip(b0, b1):
        assert torch.equal(u, v)
