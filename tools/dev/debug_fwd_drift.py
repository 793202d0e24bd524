"""Which BN's statistics vary between identical train steps (fp64 order noise ~1e-16; a real
divergence is >1e-10)?  Prints the first drifting BN in forward order for each rerun."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from test_model_gpu import _train_model, synth, make_targets

dtype = sys.argv[1] if len(sys.argv) > 1 else "f32"
use_step = len(sys.argv) > 2 and sys.argv[2] == "step"
m, anchors = _train_model(dtype)
x, boxes, cls, n = synth(4)
t, *_ = make_targets(m, anchors, boxes, cls, n)
m.fixed_masks = {k: torch.ones(2, 5, 2).cuda() for k in ("class_net", "box_net")}
sd0 = m.state_dict()
xs = torch.tensor(x).cuda()
st = []
for r in range(4):
    m.load_state_dict(sd0)
    if use_step:
        m.train_step((xs, t))
    else:
        m.forward_backward((xs, t))
    torch.cuda.synchronize()
    st.append(m.P.bn_tstats.clone())
for r in range(1, 4):
    rel = ((st[r] - st[0]).abs() / (st[0].abs() + 1e-30)).max(0).values
    o = 0
    first = None
    for bn in m.P.bns:
        v = float(rel[o:o + bn.C].max())
        if v > 1e-10 and first is None:
            first = (bn.name, v)
        o += bn.C
    print(f"run {r}: max rel {float(rel.max()):.2e}  first drifting BN: {first}")
