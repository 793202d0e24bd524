"""Debug: compare activation gradients (tape trace) of the fp32 and bf16 GPU models."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np
import torch
from test_model_gpu import _train_model, synth, make_targets, fixed_masks

runs = {}
for dt in ("f32", "bf16"):
    m, anchors = _train_model(dt, seed=1)
    x, boxes, cls, n = synth(5)
    t, *_ = make_targets(m, anchors, boxes, cls, n)
    fm = fixed_masks(m)
    m.fixed_masks = {"class_net": torch.tensor(fm[0]).cuda(), "box_net": torch.tensor(fm[1]).cuda()}
    m.grad_trace = []
    m.forward_backward((torch.tensor(x).cuda(), t))
    torch.cuda.synchronize()
    runs[dt] = (m.grad_trace, m.P.grads_dict(), m)
tr32, g32, m32 = runs["f32"]
tr16, g16, _ = runs["bf16"]
print("trace lengths", len(tr32), len(tr16))
for (n1, a, s1), (n2, b, s2) in zip(tr32, tr16):
    assert n1 == n2
    err = float((a - b).norm() / a.norm().clamp_min(1e-30))
    print(f"{n1:60s} |d|={float(a.norm()):10.3e} rel_err={err:8.4f}")
print("--- param grads")
for k in m32.P.order:
    a, b = g32[k].ravel(), g16[k].ravel()
    na = np.linalg.norm(a)
    print(f"{k:70s} |g|={na:10.3e} rel={np.linalg.norm(a - b) / max(na, 1e-30):8.4f}")
