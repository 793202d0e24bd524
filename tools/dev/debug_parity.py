"""Layer-by-layer product vs oracle comparison (forward values or backward d(value)).

    python tools/dev/debug_parity.py MODEL SIZE BATCH NC DTYPE MODE [TRAINING]
      MODE fwd : every single-segment activation's value after call(training)
      MODE grad: every activation's d(value) from the tape trace of one forward_backward
Prints, in execution order, name / relative error (norm of difference over norm of the oracle)
/ max abs error over the oracle's RMS.  Same perturbed parameters and data as
tests/test_headline_gpu.py."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.ref_model import RefEfficientDet  # noqa: E402
from tests.test_headline_gpu import drop_masks, perturb, ref_targets, synth  # noqa: E402
from tf2mv_amd import ops, runtime  # noqa: E402
from tf2mv_amd.anchors import Anchors  # noqa: E402
from tf2mv_amd.config import efficientnet_b0_blocks, get_efficientdet_config  # noqa: E402
from tf2mv_amd.model import EfficientDetNetTrain  # noqa: E402

name, S, B, NC, dtype, mode = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], sys.argv[6]
training = (sys.argv[7] != "0") if len(sys.argv) > 7 else True
seed = int(os.environ.get("SEED", "11"))
torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
cfg = get_efficientdet_config(name, {"image_size": S, "num_classes": NC})
anchors = Anchors(cfg.min_level, cfg.max_level, (S, S), cfg.num_scales, cfg.aspect_ratios, cfg.anchor_scale)
m = EfficientDetNetTrain(efficientnet_b0_blocks(), cfg, anchors, dtype=dtype, seed=seed, lr_schedule={"fixed_lr": 0.01})
sd = perturb(m.state_dict(), seed + 100)
if dtype == "bf16":
    sd = {k: (v if k.endswith(("moving_mean", "moving_variance")) else
              torch.tensor(v).to(torch.bfloat16).float().numpy()) for k, v in sd.items()}
m.load_state_dict(sd)
x, boxes, cls, n = synth(B, S, NC, seed)
if dtype == "bf16":
    x = torch.tensor(x).to(torch.bfloat16).float().numpy()
t = anchors.generate_targets_batched(torch.tensor(boxes), torch.tensor(cls), torch.tensor(n))
fm = drop_masks(m, B, seed)
masks = {"class_net": torch.tensor(fm[0]).cuda(), "box_net": torch.tensor(fm[1]).cuda()}
xs = torch.tensor(x).cuda()

ref = RefEfficientDet(cfg, m.state_dict())
ref.trace = {}
rows = []


def nhwc(v):
    return v.detach().permute(0, 2, 3, 1).reshape(-1, v.shape[1]).double()


def report(nm, a, r):
    a = a.double()
    d = a - r
    rel = float(d.norm() / r.norm().clamp_min(1e-300))
    rms = float(r.pow(2).mean().sqrt())
    rows.append((nm, rel, float(d.abs().max()) / max(rms, 1e-300), rms))


if mode == "fwd":
    acts = []
    orig_init = runtime.Act.__init__

    def logging_init(self, *a, **k):
        orig_init(self, *a, **k)
        acts.append(self)
    runtime.Act.__init__ = logging_init
    m.call(xs, training=training, masks=masks if training else None)
    runtime.Act.__init__ = orig_init
    seen = {}
    vals = []
    for a in acts:
        if a.pyr.nseg != 1 or not a.name:
            continue
        nm = a.name
        if nm.startswith("resample_p") and a.bns is None:
            nm = nm + "/pool"
        v = ops.materialize(m.eng, a).raw[: a.pyr.rows, : a.C].float().cpu()
        vals.append((nm, v))
    with torch.no_grad():
        ref.forward(x, training, {"class_net": fm[0], "box_net": fm[1]} if training else None)
    for nm, v in vals:
        if nm in ref.trace:
            report(nm, v, nhwc(ref.trace[nm]))
else:
    yb, yc, ym = ref_targets(m, t, B, NC)
    m.fixed_masks = masks
    m.grad_trace = []
    m.forward_backward((xs, t))
    torch.cuda.synchronize()
    keys = [k for k in ref.p if not k.endswith(("/moving_mean", "/moving_variance"))]
    for k in keys:
        ref.p[k].requires_grad_(True)
    rb, rc = ref.forward(x, True, {"class_net": fm[0], "box_net": fm[1]})
    loss, _ = ref.detection_loss(rb, rc, yb, yc, ym)
    loss.backward()
    seen = {}
    for nm, d, scale in m.grad_trace:
        key = nm
        if key in seen and key.startswith("resample_p"):
            key = nm  # second take of a resample name is the conv (backward order: pool first)
        elif key.startswith("resample_p"):
            key = nm + "/pool"
        seen[nm] = 1
        if key in ref.trace and ref.trace[key].grad is not None:
            report(key, d.cpu(), nhwc(ref.trace[key].grad))
for nm, rel, mx, rms in rows:
    flag = " <<<" if rel > 1e-3 else ""
    print(f"{nm:70s} rel {rel:.2e}  maxabs/rms {mx:.2e}  rms {rms:.2e}{flag}")
