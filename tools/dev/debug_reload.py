"""Is load_state_dict(state_dict()) an identity for the next step's gradients?  Compare
buffers and gradients of: fresh model, and the same model after one train_step + reload."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from test_model_gpu import _train_model, synth, make_targets

m, anchors = _train_model("f32")
x, boxes, cls, n = synth(4)
t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
m.fixed_masks = {k: torch.ones(2, 5, 2).cuda() for k in ("class_net", "box_net")}
xs = torch.tensor(x).cuda()
P = m.P
names = ["w", "wct", "ema", "bn_mm", "bn_mv", "bn_count", "bn_istats"]
snap = lambda: {k: getattr(P, k).clone() for k in names}  # noqa: E731
s0 = snap()
sd0 = m.state_dict()
m.forward_backward((xs, t))
gA = P.g.clone()
m.apply_gradients()
m.load_state_dict(sd0)
s1 = snap()
for k in names:
    a, b = s0[k], s1[k]
    print(f"{k:10s} equal={torch.equal(a, b)} maxdiff={float((a.double() - b.double()).abs().max()):.3e}")
m.forward_backward((xs, t))
gB = P.g.clone()
print("grad rel fresh vs reloaded:", float((gA - gB).norm() / gA.norm()))
m.load_state_dict(sd0)
m.forward_backward((xs, t))
gC = P.g.clone()
print("grad rel reloaded vs reloaded:", float((gB - gC).norm() / gB.norm()))
