"""Compact targets vs targets converted from the reference format: compare the target
tensors on segment rows, then the loss parts and gradients of the same fp32 step."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from tf2mv_amd.anchors import Targets
from test_model_gpu import _train_model, synth, make_targets

m, anchors = _train_model("f32")
x, boxes, cls, n = synth(4)
t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
pyr = t.pyr
t2 = Targets.from_reference(tuple(torch.tensor(a).cuda() for a in yb), tuple(torch.tensor(a).cuda() for a in yc),
                            tuple(torch.tensor(a).cuda() for a in ym), pyr, m.A, "cuda")
for s in range(pyr.nseg):
    sl = pyr.seg_slice(s)
    print(f"seg {s}: box eq {torch.equal(t.box[sl], t2.box[sl])} cls eq {torch.equal(t.cls[sl], t2.cls[sl])} "
          f"mask eq {torch.equal(t.mask[sl], t2.mask[sl])}  cls uniq {torch.unique(t.cls[sl]).tolist()[:8]} vs {torch.unique(t2.cls[sl]).tolist()[:8]}")
    if not torch.equal(t.cls[sl], t2.cls[sl]):
        d = torch.nonzero(t.cls[sl] != t2.cls[sl])
        print("   first cls diffs", [(int(r), int(a), int(t.cls[sl][r, a]), int(t2.cls[sl][r, a])) for r, a in d[:5].tolist()])
m.fixed_masks = {k: torch.ones(2, 5, 2).cuda() for k in ("class_net", "box_net")}
sd0 = m.state_dict()
xs = torch.tensor(x).cuda()
res = []
for tt in (t, t2):
    m.load_state_dict(sd0)
    m.forward_backward((xs, tt))
    torch.cuda.synchronize()
    res.append((float(m.scalars[0]), float(m.scalars[5]), m.level_parts.clone(), m.P.g.clone()))
print("loss", res[0][0], res[1][0], "npos", res[0][1], res[1][1])
print("level parts", res[0][2].tolist(), res[1][2].tolist())
print("grad rel", float((res[0][3] - res[1][3]).norm() / res[0][3].norm()))
