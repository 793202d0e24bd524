"""Uninitialised-read detector: every Engine.empty() buffer is NaN-filled; a kernel that reads
memory nobody wrote turns it into NaN.  Reports the first traced gradient / final tensors
that are non-finite."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from tf2mv_amd import runtime
from test_model_gpu import _train_model, synth, make_targets

dtype = sys.argv[1] if len(sys.argv) > 1 else "f32"
_orig_empty = runtime.Engine.empty


def nan_empty(self, rows, C, dtype=None):
    t = _orig_empty(self, rows, C, dtype)
    if t.is_floating_point():
        t.fill_(float("nan"))
    return t


runtime.Engine.empty = nan_empty
m, anchors = _train_model(dtype)
x, boxes, cls, n = synth(4)
t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
m.fixed_masks = {k: torch.ones(2, 5, 2).cuda() for k in ("class_net", "box_net")}
m.grad_trace = []
m.forward_backward((torch.tensor(x).cuda(), t))
torch.cuda.synchronize()
print("loss", float(m.scalars[0]), "npos", float(m.scalars[5]))
print("grad nonfinite:", int((~torch.isfinite(m.P.g)).sum()), "of", m.P.g.numel())
print("stats nonfinite:", int((~torch.isfinite(m.P.bn_tstats)).sum()))
for i, (name, g, sc) in enumerate(m.grad_trace):
    bad = int((~torch.isfinite(g)).sum())
    if bad:
        rows = torch.nonzero(~torch.isfinite(g))[:, 0]
        print(f"first non-finite d(value): [{i}] {name} shape={tuple(g.shape)} count={bad} rows {int(rows.min())}..{int(rows.max())}")
        break
bad_params = [k for k, sp in m.P.specs.items() if not torch.isfinite(m.P.g[sp.offset: sp.offset + sp.size]).all()]
print("params with non-finite grads:", len(bad_params), bad_params[:6])
