"""Data-parallel path at world size 2 over gloo on the CPU.

* plumbing: ``tf2mv_amd.dist`` rendezvous on 127.0.0.1, equal disjoint shards, the flat SUM
  all-reduce the model's ``grad_allreduce`` / ``npos_allreduce`` hooks use, max-over-ranks
  timing;
* normalisation: two replicas holding identical shards, each computing the oracle loss with the
  global N+ and ``count_scale = world`` and all-reducing its gradient through the same hook,
  must reproduce the single-process gradient of the doubled batch exactly (identical shards
  make per-replica BatchNorm equal full-batch BatchNorm, so the equality is exact, fp64).

The GPU twin, ``tests/test_model_gpu.py::test_dp_two_identical_replicas_equal_double_batch``,
checks the same identity on the HIP path itself.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

SIZE, NC = 128, 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _plumbing(ctx):
    from tf2mv_amd import dist as dp
    sl = dp.shard_slice(8, ctx.rank, ctx.world)
    ar = dp.make_allreduce(ctx)
    flat = torch.arange(1000, dtype=torch.float32) * (ctx.rank + 1)
    ar(flat)
    npos = torch.tensor([5.0 + ctx.rank])
    ar(npos)
    mx = dp.max_over_ranks(ctx, 1.5 * ctx.rank)
    el = dp.timed(ctx, lambda: None, 3, lambda: None)
    return {"shard": torch.tensor([sl.start, sl.stop]), "flat": flat, "npos": npos, "max": torch.tensor(mx),
            "el": torch.tensor(el)}


def _model_and_data():
    from oracle import ref_anchors as RA
    from tf2mv_amd.config import efficientnet_b0_blocks, get_efficientdet_config
    from tf2mv_amd.model import EfficientDetNet

    cfg = get_efficientdet_config("efficientdet-d0", {"image_size": SIZE, "num_classes": NC})
    m = EfficientDetNet(efficientnet_b0_blocks(), cfg, dtype="f32", device="cpu", seed=7)
    rng = np.random.default_rng(11)
    x = rng.random((1, SIZE, SIZE, 3), dtype=np.float32)
    boxes = np.array([[10, 12, 60, 70], [40, 30, 100, 90], [5, 80, 40, 120]], np.float32)
    classes = np.array([1, 3, 2])
    lv = RA.generate_boxes(cfg.min_level, cfg.max_level, (SIZE, SIZE), cfg.num_scales, cfg.aspect_ratios,
                           cfg.anchor_scale)
    ob, oc, om, _ = RA.generate_targets(lv, boxes, classes, NC)
    yb = [b[None] for b in ob]
    yc = [c[None] for c in oc]
    ym = [mm[None] for mm in om]
    return m, x, yb, yc, ym


def _flat_grads(ref, loss):
    keys = [k for k in sorted(ref.p) if not (k.endswith("/moving_mean") or k.endswith("/moving_variance"))]
    gs = torch.autograd.grad(loss, [ref.p[k] for k in keys], allow_unused=True)
    return torch.cat([(g if g is not None else torch.zeros_like(ref.p[k])).reshape(-1) for k, g in zip(keys, gs)])


def _ref(m):
    from oracle.ref_model import RefEfficientDet
    ref = RefEfficientDet(m.cfg, m.state_dict())
    for k, v in ref.p.items():
        v.requires_grad_(not (k.endswith("/moving_mean") or k.endswith("/moving_variance")))
    return ref


def _oracle_dp(ctx):
    from oracle.ref_model import BNState
    from tf2mv_amd import dist as dp
    torch.set_num_threads(2)
    m, x, yb, yc, ym = _model_and_data()  # identical shard on every rank
    ref = _ref(m)
    ar = dp.make_allreduce(ctx)
    npos = torch.tensor([float(sum(np.asarray(a).sum() for a in ym))], dtype=torch.float64)
    ar(npos)  # global N+ (the loss adds the +1)
    box, cls = ref.forward(x, True, None, BNState())
    loss, _ = ref.detection_loss(box, cls, yb, yc, ym, with_l2=False, npos_sum=npos[0], count_scale=ctx.world)
    g = _flat_grads(ref, loss).detach().clone()
    ar(g)
    lt = loss.detach().reshape(1).clone()
    ar(lt)
    return {"grad": g, "loss": lt}


FNS = {"plumbing": _plumbing, "oracle_dp": _oracle_dp}


def _worker(rank, world, port, fn, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from tf2mv_amd import dist as dp
    ctx = dp.init_from_env("gloo")
    assert ctx.world == world and ctx.rank == rank and ctx.distributed
    out = FNS[fn](ctx)
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    dp.shutdown(ctx)


def _run(fn, world=2):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), fn, d), nprocs=world, join=True)
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]


def test_dist_plumbing_gloo():
    outs = _run("plumbing")
    assert [o["shard"].tolist() for o in outs] == [[0, 4], [4, 8]]
    for o in outs:
        torch.testing.assert_close(o["flat"], torch.arange(1000, dtype=torch.float32) * 3)
        assert float(o["npos"]) == 11.0
        assert float(o["max"]) == 1.5
        assert float(o["el"]) >= 0.0


def test_shard_slice_rejects_ragged_batch():
    from tf2mv_amd import dist as dp
    with pytest.raises(ValueError):
        dp.shard_slice(7, 0, 2)
    assert dp.shard_slice(7, 0, 1) == slice(0, 7)


def test_single_process_context_is_noop():
    from tf2mv_amd import dist as dp
    ctx = dp.init_from_env()
    assert not ctx.distributed and dp.make_allreduce(ctx) is None
    assert dp.max_over_ranks(ctx, 2.5) == 2.5


def test_dp_normalisation_oracle_gloo():
    from oracle.ref_model import BNState
    outs = _run("oracle_dp")
    torch.set_num_threads(4)
    m, x, yb, yc, ym = _model_and_data()
    ref = _ref(m)
    x2 = np.concatenate([x, x])
    box, cls = ref.forward(x2, True, None, BNState())
    loss, _ = ref.detection_loss(box, cls, [np.concatenate([a, a]) for a in yb], [np.concatenate([a, a]) for a in yc],
                                 [np.concatenate([a, a]) for a in ym], with_l2=False)
    g = _flat_grads(ref, loss)
    for o in outs:
        torch.testing.assert_close(o["loss"][0], loss.detach(), rtol=1e-10, atol=0)
        err = float((o["grad"] - g).norm() / g.norm())
        assert err < 1e-9, err
