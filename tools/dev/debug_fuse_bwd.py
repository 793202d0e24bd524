"""Snapshot every bifpn_fuse_bwd launch (dF in, each input's dx out, weight grads) over 4
identical fp32 steps and report the first launch whose outputs differ between runs."""
import sys, os, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from tf2mv_amd import _lib as L
from tf2mv_amd.runtime import stream
from test_model_gpu import _train_model, synth, make_targets

m, anchors = _train_model("f32")
x, boxes, cls, n = synth(4)
t, yb, yc, ym = make_targets(m, anchors, boxes, cls, n)
m.fixed_masks = {k: torch.ones(2, 5, 2).cuda() for k in ("class_net", "box_net")}
sd0 = m.state_dict()
xs = torch.tensor(x).cuda()
orig = L._Lib.call
cur = []


def grab(ptr, numel):
    out = torch.empty(numel, dtype=torch.float32, device="cuda")
    orig(L.lib(), "edet_memcpy_async", ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ptr), numel * 4, stream())
    return out


def traced(self, name, *args):
    if name == "edet_bifpn_fuse_bwd":
        dt, nin, fb, wv, B, H, W, C, y, dF, dw, s = args
        torch.cuda.synchronize()
        snap_in = {"dF": grab(dF.value, B * H * W * C)}
        pre = [grab(fb[i].dx, B * fb[i].H * fb[i].W * C) if fb[i].accumulate else None for i in range(nin)]
        rc = orig(self, name, *args)
        torch.cuda.synchronize()
        outs = [grab(fb[i].dx, B * fb[i].H * fb[i].W * C) for i in range(nin)]
        cur.append((snap_in, pre, outs, [(fb[i].mode, fb[i].accumulate, fb[i].H) for i in range(nin)]))
        return rc
    return orig(self, name, *args)


L._Lib.call = traced
runs = []
for r in range(4):
    m.load_state_dict(sd0)
    cur = []
    m.forward_backward((xs, t))
    torch.cuda.synchronize()
    runs.append(cur)
L._Lib.call = orig
rel = lambda a, b: float((a - b).norm()) / (float(a.norm()) + 1e-30)  # noqa: E731
for r in range(1, 4):
    print(f"--- run {r}")
    for k, (a, b) in enumerate(zip(runs[0], runs[r])):
        ed = rel(a[0]["dF"], b[0]["dF"])
        for i in range(len(a[2])):
            pr = rel(a[1][i], b[1][i]) if a[1][i] is not None else 0.0
            o = rel(a[2][i], b[2][i])
            if o > 1e-3 or ed > 1e-3 or pr > 1e-3:
                print(f"  call {k} input {i} (mode,acc,H)={a[3][i]}  dF rel {ed:.2e}  dx-before rel {pr:.2e}  dx-after rel {o:.2e}")
