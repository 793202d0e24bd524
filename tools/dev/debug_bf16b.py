"""Debug 2: gradient sensitivity. (i) fp32 vs fp32 with a 2^-9 relative input perturbation and
bf16-rounded weights; (ii) bf16 vs fp32 at a realistic size (B=8, 512x512)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np
import torch
from tf2mv_amd.anchors import Anchors
from tf2mv_amd.config import efficientnet_b0_blocks, get_efficientdet_config
from tf2mv_amd.model import EfficientDetNetTrain


def run(dtype, size, B, x, boxes, cls, sd=None, round_w=False):
    c = get_efficientdet_config("efficientdet-d0", {"image_size": size})
    a = Anchors(3, 7, (size, size), 3, c.aspect_ratios, 4.0)
    m = EfficientDetNetTrain(efficientnet_b0_blocks(), c, a, dtype=dtype, seed=1, lr_schedule={"fixed_lr": 0.01})
    if sd is not None:
        m.load_state_dict(sd)
    if round_w:
        sd2 = {k: torch.tensor(v).bfloat16().float().numpy() for k, v in m.state_dict().items()}
        m.load_state_dict(sd2)
    m.fixed_masks = {k: torch.ones(2, 5, B).cuda() for k in ("class_net", "box_net")}
    t = a.generate_targets_batched(torch.tensor(boxes), torch.tensor(cls), torch.full((B,), boxes.shape[1], dtype=torch.int32))
    m.forward_backward((torch.tensor(x).cuda(), t))
    torch.cuda.synchronize()
    return m.P.grads_dict(), m.state_dict(), float(m.scalars[0])


def cmp(tag, g1, g2):
    keys = list(g1)
    a = np.concatenate([g1[k].ravel() for k in keys]); b = np.concatenate([g2[k].ravel() for k in keys])
    cos = a @ b / (np.linalg.norm(a) * np.linalg.norm(b))
    rel = sorted(((np.linalg.norm(g1[k] - g2[k]) / max(np.linalg.norm(g1[k]), 1e-30), k) for k in keys), reverse=True)
    med = np.median([r for r, _ in rel])
    print(f"{tag}: cosine={cos:.5f} median per-tensor rel err={med:.4f} worst={rel[:4]}", flush=True)


def data(size, B, seed):
    rng = np.random.default_rng(seed)
    x = rng.random((B, size, size, 3), dtype=np.float32)
    G = 7
    boxes = np.zeros((B, G, 4), np.float32)
    cls = rng.integers(1, 81, (B, G)).astype(np.int32)
    for b in range(B):
        for k in range(G):
            s = np.exp(rng.uniform(np.log(16), np.log(size * 0.8)))
            ar = rng.uniform(0.5, 2)
            h, w = s * np.sqrt(ar), s / np.sqrt(ar)
            cy, cx = rng.uniform(0, size, 2)
            boxes[b, k] = [cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2]
    return x, boxes, cls


for size, B in ((128, 2), (512, 8)):
    x, boxes, cls = data(size, B, 0)
    g32, sd, l32 = run("f32", size, B, x, boxes, cls)
    xp = (x * (1 + 2.0 ** -9 * np.random.default_rng(1).standard_normal(x.shape))).astype(np.float32)
    gp, _, lp = run("f32", size, B, xp, boxes, cls, sd)
    cmp(f"size={size} B={B} fp32 vs fp32(input*(1+2^-9 noise))", g32, gp)
    gw, _, lw = run("f32", size, B, x, boxes, cls, sd, round_w=True)
    cmp(f"size={size} B={B} fp32 vs fp32(bf16-rounded weights)", g32, gw)
    g16, _, l16 = run("bf16", size, B, x, boxes, cls, sd)
    cmp(f"size={size} B={B} fp32 vs bf16", g32, g16)
    print("losses", l32, lp, lw, l16, flush=True)
