"""bench.py's N > 1 branch on the one-GPU box.

The driver's 8-GPU scaling run (BASELINE config 4) launches

    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K --warmup W

and that branch -- the three captured graphs with the N+ and gradient all-reduces between them
(`dist.graphed_train_step`), rank 0's instrumented steps with the state snapshot and restore,
the global-loss reduction and `max_over_ranks` -- is run here exactly so, with torchrun as the
launcher, two ranks sharing cuda:0 over gloo (`EDET_DP_BACKEND=gloo`; RCCL needs one GPU per
rank).  Checked:

* one JSON line on stdout with n_gpus 2, the global batch and a positive finite rate;
* the reported loss is the replicas' data terms summed plus ONE L2 term
  (`efficientdet_net_train.py:41-52` at the global batch);
* after the run the replicas' weights, momentum, EMA and step counters are bit-identical:
  rank 0 ran its extra instrumented (non-all-reduced) steps and restored its state, and the
  optimizer is deterministic over the all-reduced gradient.
Reference pattern: facenet/facenet_model.py:297 (MirroredStrategy gradient all-reduce).
"""
import json
import math
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(900)
def test_bench_two_ranks_torchrun_gloo(tmp_path):
    env = dict(os.environ, EDET_DP_BACKEND="gloo", EDET_BENCH_DUMP=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1"]
    # rank 0's progress goes to a file as it runs (a report directory when one is given)
    logdir = os.environ.get("EDET_REPORT_DIR") or str(tmp_path)
    os.makedirs(logdir, exist_ok=True)
    log = os.path.join(logdir, "bench_dp2.log")
    with open(log, "w") as ferr:
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=ferr, text=True, timeout=840)
    with open(log) as f:
        err = f.read()
    assert r.returncode == 0, (r.stdout[-2000:], err[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 2 * 32
    assert out["value"] > 0 and math.isfinite(out["value"]) and out["steps"] == 3
    assert out["roofline"] is not None and out["roofline"]["frac"] > 0
    ranks = [torch.load(tmp_path / f"rank{k}.pt", weights_only=True) for k in range(2)]
    # global loss = sum of the replicas' data terms + one L2 term (each replica's scalars[0]
    # holds its data term plus the identical L2 term)
    l2 = ranks[0]["l2_term"]
    assert l2 == ranks[1]["l2_term"] and l2 > 0
    want = float(ranks[0]["scalars"][0]) + float(ranks[1]["scalars"][0]) - l2
    assert math.isfinite(out["loss"]) and abs(out["loss"] - want) <= 1e-4 * abs(want), (out["loss"], want)
    assert float(ranks[0]["scalars"][0]) != float(ranks[1]["scalars"][0])  # distinct shards
    # replicas bit-identical after rank 0's instrumented steps and state restore
    for k in ("w", "v", "ema", "step"):
        assert torch.equal(ranks[0][k], ranks[1][k]), (k, float((ranks[0][k].double() - ranks[1][k].double()).abs().max()))
    assert int(ranks[0]["step"][0]) == 2 + 1 + 3  # eager warm-ups + graph warm-up + timed steps
