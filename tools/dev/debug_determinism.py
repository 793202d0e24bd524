"""Run the same fp32 train step (same weights, same data) several times and report how far
the BN statistics and per-tensor gradients move between runs (atomics-order noise vs races)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch
from test_model_gpu import _train_model, synth, make_targets

dtype = sys.argv[1] if len(sys.argv) > 1 else "f32"
m, anchors = _train_model(dtype)
x, boxes, cls, n = synth(4)
t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
m.fixed_masks = {k: torch.ones(2, 5, 2).cuda() for k in ("class_net", "box_net")}
sd0 = m.state_dict()
xs = torch.tensor(x).cuda()
runs = []
for r in range(4):
    m.load_state_dict(sd0)
    m.forward_backward((xs, t))
    torch.cuda.synchronize()
    runs.append((m.P.g.clone(), m.P.bn_tstats.clone(), float(m.scalars[0])))
g0, s0, l0 = runs[0]
for r in range(1, 4):
    g, s, l = runs[r]
    print(f"run {r}: loss {l0:.8f} vs {l:.8f}  stats maxrel {float(((s - s0).abs() / (s0.abs() + 1e-6)).max()):.3e}")
    worst = []
    for k, sp in m.P.specs.items():
        a, b = g0[sp.offset: sp.offset + sp.size], g[sp.offset: sp.offset + sp.size]
        rel = float((a - b).norm()) / (float(a.norm()) + 1e-12)
        worst.append((rel, k))
    worst.sort(reverse=True)
    gmax = max(float(g0[sp.offset: sp.offset + sp.size].norm()) for sp in m.P.specs.values())
    sig = []
    for k, sp in m.P.specs.items():
        a, b = g0[sp.offset: sp.offset + sp.size], g[sp.offset: sp.offset + sp.size]
        if float(a.norm()) >= 1e-2 * gmax and not k.endswith("bias"):
            sig.append((float((a - b).norm()) / float(a.norm()), k))
    sig.sort(reverse=True)
    print("   global rel", float((g - g0).norm()) / float(g0.norm()))
    print("   worst significant:", [(f"{a:.2e}", k) for a, k in sig[:5]])
    st = m.P.specs["efficientnet-b0/stem/conv2d/kernel"]
    print("   stem rel", float((g[st.offset:st.offset + st.size] - g0[st.offset:st.offset + st.size]).norm()) / float(g0[st.offset:st.offset + st.size].norm()))
# stats arena breakdown: which BN drifts first (forward order)
s1 = runs[1][1]
rel = ((s1 - s0).abs() / (s0.abs() + 1e-3)).cpu().numpy()
idx = np.nonzero(rel.max(0) > 1e-4)[0]
print("stats entries with rel>1e-4:", idx.size, "first at", idx[:10])
o = 0
shown = 0
for bn in m.P.bns:
    r = rel[:, o:o + bn.C].max() if rel.ndim == 2 else rel[o:o + bn.C].max()
    if r > 1e-5 and shown < 12:
        print(f"   drift {r:.2e} at BN {bn.name}")
        shown += 1
    o += bn.C
