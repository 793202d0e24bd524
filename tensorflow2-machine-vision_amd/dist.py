"""Data-parallel plumbing for the EfficientDet train step.

One process per GPU (torchrun / torch.distributed.run sets RANK, WORLD_SIZE, LOCAL_RANK,
MASTER_ADDR/PORT); backend "nccl" is RCCL on ROCm and runs over the xGMI mesh, "gloo" is the
CPU backend the multi-process tests use.  The reference's EfficientDet trains on one device
(`efficientnet/train.py:145`, `model.fit`); the repo's only data-parallel precedent is
FaceNet's MirroredStrategy (`facenet/train.py:71`, gradient all-reduce at
`facenet/facenet_model.py:297`).  The step here follows that pattern with the global-batch
loss normalisation:

  1. every replica counts its positive anchors; one 1-float all-reduce (SUM) makes N+ global
     (the loss adds the +1 of `efficientdet_net_train.py:46` to the global sum);
  2. the focal mean over a replica's elements is scaled by ``world`` (``focal_count_scale``), so
     the replicas' losses sum to the global-batch loss and their gradients sum to its gradient
     (BatchNorm statistics stay per replica, as under MirroredStrategy);
  3. one flat all-reduce (SUM) of the fp32 gradient buffer (15.5 MB for D0);
  4. L2, global-norm clip, SGD momentum and EMA run redundantly on every replica, so the
     parameters stay bit-identical without a broadcast.

Nothing here touches the data path: the shards are independent images, the only exchange is
the two all-reduces above.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as tdist


@dataclass
class DPContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def distributed(self) -> bool:
        return self.world > 1


def init_from_env(backend: Optional[str] = None, device: Optional[torch.device] = None) -> DPContext:
    """Join the process group named by the torchrun environment (no-op for one process).

    ``backend`` defaults to "nccl" (RCCL) when ``device`` is a GPU, else "gloo"."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world <= 1:
        return DPContext(rank=0, world=1, local_rank=local, backend="none")
    if backend is None:
        backend = "nccl" if (device is not None and device.type == "cuda") else "gloo"
    if not tdist.is_initialized():
        kw = {}
        if backend == "nccl" and device is not None:
            kw["device_id"] = device
        tdist.init_process_group(backend, **kw)
    return DPContext(rank=rank, world=world, local_rank=local, backend=backend)


def shard_slice(global_batch: int, rank: int, world: int) -> slice:
    """Contiguous, equal, disjoint shard of the global batch for ``rank``."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} is not divisible by world size {world}")
    per = global_batch // world
    return slice(rank * per, (rank + 1) * per)


def make_allreduce(ctx: DPContext) -> Optional[Callable[[torch.Tensor], None]]:
    """In-place SUM all-reduce callback for the model's ``grad_allreduce`` /
    ``npos_allreduce`` hooks (None for a single replica)."""
    if not ctx.distributed:
        return None

    def _ar(t: torch.Tensor) -> None:
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM)

    return _ar


def barrier(ctx: DPContext) -> None:
    if ctx.distributed:
        tdist.barrier()


def max_over_ranks(ctx: DPContext, value: float, device: Optional[torch.device] = None) -> float:
    """The slowest replica's value (the bench's timed region is max over ranks)."""
    if not ctx.distributed:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device if ctx.backend == "nccl" else "cpu")
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def timed(ctx: DPContext, fn: Callable[[], None], steps: int, sync: Callable[[], None]) -> float:
    """Run ``fn`` ``steps`` times between barrier+sync brackets; return the max-over-ranks
    wall time in seconds."""
    sync()
    barrier(ctx)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    barrier(ctx)
    sync()
    return time.perf_counter() - t0


def graphed_train_step(model, data, allreduce: Optional[Callable[[torch.Tensor], None]] = None) -> Callable[[], None]:
    """Capture ``model.train_step(data)`` in HIP graphs and return the replay callable.

    One replica: the whole step is one graph.  Data parallel: three graphs -- prepare
    (targets, this replica's N+) | compute (forward, fused loss, backward) | optimizer -- with
    the N+ all-reduce and the flat gradient all-reduce issued between them on the same
    stream, so the collectives stay outside the captured work (RCCL/gloo calls are not
    captured).  ``data``'s tensors must stay alive and in place while the graphs are used.

    The model must have run one eager step on ``data``'s shapes first: persistent buffers
    (drop-connect masks, split-reduction workspaces, the engine's activation arena) are
    allocated on first use, and an allocation inside capture would be baked into the graph
    from the capture pool.  Capture runs on torch.cuda.graph's own side stream."""
    if getattr(model, "steps_run", 0) < 1:
        raise RuntimeError("graphed_train_step: run one eager model.train_step(data) first (warm-up)")
    # the warm-up must have run on these shapes: an eager step at another batch or image size
    # would leave the persistent buffers sized for it and capture would allocate the rest
    sig = model.shape_signature(data)
    if getattr(model, "last_step_signature", None) != sig:
        raise RuntimeError(f"graphed_train_step: the last eager step ran on {model.last_step_signature}, "
                           f"not on this data's {sig}; run one eager model.train_step(data) first")
    if allreduce is None:
        # the single graph captures model.train_step, which would call the hooks inside capture
        if model.grad_allreduce is not None or model.npos_allreduce is not None:
            raise ValueError("graphed_train_step: the model has all-reduce hooks but allreduce is None")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            model.train_step(data)
        return g.replay
    g0, g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g0):
        t_pyr = model.prepare_step(data)
    with torch.cuda.graph(g1):
        model.compute_step(data, *t_pyr)
    with torch.cuda.graph(g2):
        model.apply_gradients()

    def step():
        g0.replay()
        allreduce(model.scalars[5:6])
        g1.replay()
        allreduce(model.P.g)
        g2.replay()

    step.graphs = (g0, g1, g2)  # keep the graphs alive with the callable
    return step


def shutdown(ctx: DPContext) -> None:
    if ctx.distributed and tdist.is_initialized():
        tdist.barrier()
        tdist.destroy_process_group()
