"""Run the same fp32 step 4 times with the tape's gradient trace on and print, in backward
order, the first activations whose d(value) differs between runs by more than 1e-3."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from test_model_gpu import _train_model, synth, make_targets

dtype = sys.argv[1] if len(sys.argv) > 1 else "f32"
m, anchors = _train_model(dtype)
x, boxes, cls, n = synth(4)
t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
m.fixed_masks = {k: torch.ones(2, 5, 2).cuda() for k in ("class_net", "box_net")}
sd0 = m.state_dict()
xs = torch.tensor(x).cuda()
traces = []
for r in range(4):
    m.load_state_dict(sd0)
    m.grad_trace = []
    m.forward_backward((xs, t))
    torch.cuda.synchronize()
    traces.append(m.grad_trace)
for r in range(1, 4):
    print(f"--- run {r} vs run 0 ({len(traces[r])} entries)")
    shown = 0
    for i, ((na, a, _), (nb, b, _)) in enumerate(zip(traces[0], traces[r])):
        assert na == nb
        rel = float((a - b).norm()) / (float(a.norm()) + 1e-30)
        nonfinite = int((~torch.isfinite(b)).sum())
        if rel > 1e-3 or nonfinite:
            print(f"  [{i}] {na} shape={tuple(a.shape)} rel={rel:.3e} nonfinite={nonfinite} |a|={float(a.norm()):.3e}")
            shown += 1
            if shown >= 8:
                break
# where does the first divergence sit: a few elements (argmax flip) or everywhere (race)?
for r in range(1, 4):
    for i, ((na, a, _), (nb, b, _)) in enumerate(zip(traces[0], traces[r])):
        d = (a - b).abs()
        if float(d.norm()) > 1e-3 * float(a.norm()):
            flat = d.flatten()
            top = torch.topk(flat, 6)
            share = float((top.values ** 2).sum() / (flat ** 2).sum())
            C = a.shape[1]
            pos = [(int(k) // C, int(k) % C) for k in top.indices]
            print(f"run {r}: first divergent [{i}] {na}: elements > 1e-7: {int((flat > 1e-7).sum())} of {flat.numel()},"
                  f" top-6 carry {share:.3f} of diff^2, at (row, ch) {pos}")
            break
