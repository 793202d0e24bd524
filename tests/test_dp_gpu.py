"""Data parallelism on the product path: two ranks, one process each, gloo
collectives, both on cuda:0 of the one-GPU box.  Each rank runs EfficientDetNetTrain through
``dist.graphed_train_step`` -- the same three captured graphs with the N+ and gradient
all-reduces between them that ``bench.py`` replays at N > 1 -- on its own DISTINCT shard of a
global batch.  Checked against the oracle with per-shard ("ghost batch") BatchNorm, which is
what a MirroredStrategy replica computes (facenet/facenet_model.py:297 is the repo's pattern):

* the all-reduced gradient equals the sum over shards of the oracle gradient of the shard loss
  normalised by the global N+ and the global element count (per tensor within 1e-3);
* the replicas' losses sum to the global-batch loss (+ one L2 term) within 1e-4;
* with the clip active (clip_norm below the gradient norm), the two replicas' parameters
  after the optimizer are bit-identical (deterministic gnorm);
* the replicas drew different drop-connect masks (rank folded into the seed).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
SIZE, NC, BL, WORLD = 128, 5, 2, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _global_batch():
    from tests.test_headline_gpu import synth
    return synth(BL * WORLD, SIZE, NC, seed=21, G=5)


def _cfg():
    from tf2mv_amd.config import get_efficientdet_config
    return get_efficientdet_config("efficientdet-d0", {"image_size": SIZE, "num_classes": NC})


def _masks(seed=4):
    rng = np.random.default_rng(seed)
    return rng.choice([0.0, 1.25], size=(2, 2, 5, BL * WORLD), p=[0.3, 0.7]).astype(np.float32)


def _worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    from tests.test_headline_gpu import ActCapture, perturb
    from tf2mv_amd import dist as dp
    from tf2mv_amd.anchors import Anchors
    from tf2mv_amd.config import efficientnet_b0_blocks
    from tf2mv_amd.model import EfficientDetNetTrain
    ctx = dp.init_from_env("gloo")
    ar = dp.make_allreduce(ctx)
    cfg = _cfg()
    anchors = Anchors(cfg.min_level, cfg.max_level, (SIZE, SIZE), cfg.num_scales, cfg.aspect_ratios, cfg.anchor_scale)
    m = EfficientDetNetTrain(efficientnet_b0_blocks(), cfg, anchors, dtype="f32", seed=1, world_size=WORLD,
                             grad_allreduce=ar, npos_allreduce=ar, rank=rank,
                             lr_schedule={"fixed_lr": 0.01, "clip_norm": 0.05})
    m.load_state_dict(perturb(m.state_dict(), 31))
    sd0 = m.state_dict()
    x, boxes, cls, n = _global_batch()
    sl = dp.shard_slice(BL * WORLD, rank, WORLD)
    t = anchors.generate_targets_batched(torch.tensor(boxes[sl]), torch.tensor(cls[sl]), torch.tensor(n[sl]))
    xs = torch.tensor(x[sl]).cuda()
    # the replicas' own drop-connect draws differ (rank-folded seed)
    m._make_masks(BL)
    own = m.drop_masks.clone().cpu()
    fm = _masks()
    m.fixed_masks = {"class_net": torch.tensor(fm[0][..., sl]).cuda(), "box_net": torch.tensor(fm[1][..., sl]).cuda()}
    data = (xs, t)
    with ActCapture() as cap:  # this replica's max-pool decisions (oracle routing, see test_headline_gpu)
        m.call(xs, training=True, masks=m.fixed_masks)
    routes = cap.pool_routes(m)
    del cap
    m.train_step(data)  # eager warm-up: allocates the persistent buffers before capture
    torch.cuda.synchronize()
    m.load_state_dict(sd0)  # back to the initial weights, fresh momentum / step counter
    step = dp.graphed_train_step(m, data, ar)
    step()
    torch.cuda.synchronize()
    out = {"g": m.P.g.cpu(), "w": m.P.w.cpu(), "scal": m.scalars.cpu(), "own_masks": own, "routes": routes}
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    if rank == 0:
        torch.save({k: torch.tensor(v) for k, v in sd0.items()}, os.path.join(outdir, "sd0.pt"))
        torch.save({k: (sp.offset, sp.size, sp.shape, sp.l2) for k, sp in m.P.specs.items()}, os.path.join(outdir, "specs.pt"))
    dp.shutdown(ctx)


@pytest.mark.timeout(600)
def test_dp_two_ranks_distinct_shards_graphed_step():
    from oracle.ref_model import RefEfficientDet
    from tests.test_headline_gpu import ref_targets
    from tf2mv_amd.anchors import Anchors
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(_free_port(), d), nprocs=WORLD, join=True)
        r = [torch.load(os.path.join(d, f"r{k}.pt"), weights_only=True) for k in range(WORLD)]
        sd0 = {k: v.numpy() for k, v in torch.load(os.path.join(d, "sd0.pt"), weights_only=True).items()}
        specs = torch.load(os.path.join(d, "specs.pt"), weights_only=False)
    # replicas: identical all-reduced gradient and bit-identical parameters after a clipped step
    assert torch.equal(r[0]["g"], r[1]["g"])
    assert float(r[0]["scal"][3]) > 0.05  # the clip was active
    assert torch.equal(r[0]["w"], r[1]["w"]), float((r[0]["w"] - r[1]["w"]).abs().max())
    assert not torch.equal(r[0]["own_masks"], r[1]["own_masks"])
    # oracle: per-shard BN, global N+ and element count
    cfg = _cfg()
    anchors = Anchors(cfg.min_level, cfg.max_level, (SIZE, SIZE), cfg.num_scales, cfg.aspect_ratios, cfg.anchor_scale)
    x, boxes, cls, n = _global_batch()
    fm = _masks()
    ref = RefEfficientDet(cfg, sd0)
    keys = [k for k in ref.p if not k.endswith(("/moving_mean", "/moving_variance"))]
    for k in keys:
        ref.p[k].requires_grad_(True)
    tg = anchors.generate_targets_batched(torch.tensor(boxes), torch.tensor(cls), torch.tensor(n))

    class _M:
        levels = list(range(3, 8))
        level_hw = {l: ((SIZE + 2 ** l - 1) // 2 ** l,) * 2 for l in levels}
    _, _, ymg = ref_targets(_M, tg, BL * WORLD, NC)
    npos = float(sum(a.sum() for a in ymg))
    total = None
    for k in range(WORLD):
        sl = slice(k * BL, (k + 1) * BL)
        t = anchors.generate_targets_batched(torch.tensor(boxes[sl]), torch.tensor(cls[sl]), torch.tensor(n[sl]))
        yb, yc, ym = ref_targets(_M, t, BL, NC)
        ref.routes = r[k]["routes"]
        rb, rc = ref.forward(x[sl], True, {"class_net": fm[0][..., sl], "box_net": fm[1][..., sl]})
        lk, _ = ref.detection_loss(rb, rc, yb, yc, ym, with_l2=False, npos_sum=npos, count_scale=WORLD)
        total = lk if total is None else total + lk
    gr = torch.autograd.grad(total, [ref.p[k] for k in keys], allow_unused=True)
    gnorm = float(torch.sqrt(sum((v ** 2).sum() for v in gr if v is not None)))
    l2 = float(ref.l2_loss())
    loss_sum = float(r[0]["scal"][0] + r[1]["scal"][0]) - (WORLD - 1) * l2
    assert abs(loss_sum - (float(total) + l2)) / (float(total) + l2) < 1e-4, (loss_sum, float(total) + l2)
    g = r[0]["g"].double()
    bad = []
    for k, v in zip(keys, gr):
        off, size, shape, _ = specs[k]
        gg = g[off:off + size].view(shape)
        v = torch.zeros(shape, dtype=torch.float64) if v is None else v.detach()
        err = float((gg - v).norm())
        if err > 1e-3 * float(v.norm()) + 1e-6 * gnorm:
            bad.append((k, err, float(v.norm())))
    assert not bad, bad[:8]
