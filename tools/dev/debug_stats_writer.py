"""Find which C-ABI call modifies the BN statistics arena after the forward pass
(snapshot bn_tstats after every call of one fp32 train step)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from tf2mv_amd import _lib as L
from test_model_gpu import _train_model, synth, make_targets

dtype = sys.argv[1] if len(sys.argv) > 1 else "f32"
m, anchors = _train_model(dtype)
x, boxes, cls, n = synth(4)
t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
m.fixed_masks = {k: torch.ones(2, 5, 2).cuda() for k in ("class_net", "box_net")}
xs = torch.tensor(x).cuda()
m.forward_backward((xs, t))  # warm: allocations settle
torch.cuda.synchronize()
orig = L._Lib.call
log = []
state = {"prev": None, "i": 0}


def traced(self, name, *args):
    rc = orig(self, name, *args)
    torch.cuda.synchronize()
    cur = m.P.bn_tstats.clone()
    if state["prev"] is not None and not torch.equal(cur, state["prev"]):
        d = (cur - state["prev"]).abs()
        idx = torch.nonzero(d.max(0).values > 0).flatten()
        log.append((state["i"], name, int(idx.numel()), idx[:8].tolist()))
    state["prev"] = cur
    state["i"] += 1
    return rc


L._Lib.call = traced
m.forward_backward((xs, t))
torch.cuda.synchronize()
L._Lib.call = orig
print("calls:", state["i"])
for e in log:
    print(e)
