"""Per-call kernel micro-benchmark at the model's real shapes.

Runs one eager D0 train step; every libedet launch is executed once normally and then
replayed R times back-to-back between two HIP events on the launch stream, so each call's
steady-state duration is measured without the eager launch gaps of a single-event timing.
Replays re-run accumulating kernels (values drift; irrelevant for timing).

  python scripts/kbench.py [--reps 10] [--filter conv1x1] [--top 80] [--batch 32]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--filter", default="")
    ap.add_argument("--top", type=int, default=80)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--model", default="efficientdet-d0")
    ap.add_argument("--out", default="")
    ap.add_argument("--dev", default="", help="edet_dev_set slots for the timed replays, e.g. 7=1")
    ap.add_argument("--seq", default="", help="also write every call's us in launch order")
    ap.add_argument("--abi-any", action="store_true",
                    help="A/B against an older build (EDET_LIB): accept its ABI version, drop entry points it lacks")
    args = ap.parse_args()
    if args.abi_any:
        import ctypes
        from tf2mv_amd import _lib as L0
        d = ctypes.CDLL(L0.LIB_PATH)
        for name in [n for n in L0.SIGNATURES if not hasattr(d, n)]:
            del L0.SIGNATURES[name]
        L0.ABI_VERSION = d.edet_abi_version()

    from tf2mv_amd import _lib as L
    from tf2mv_amd.anchors import Anchors
    from tf2mv_amd.config import efficientnet_b0_blocks, get_efficientdet_config
    from tf2mv_amd.model import EfficientDetNetTrain

    dev = torch.device("cuda", 0)
    cfg = get_efficientdet_config(args.model)
    S, B = cfg.image_size, args.batch
    anchors = Anchors(cfg.min_level, cfg.max_level, (S, S), cfg.num_scales, cfg.aspect_ratios, cfg.anchor_scale, device=dev)
    model = EfficientDetNetTrain(efficientnet_b0_blocks(), cfg, anchors, dtype="bf16", device=dev, seed=0,
                                 lr_schedule={"warmup_steps": 100, "total_steps": 10000})
    model.eng.overlap = False  # isolated replays
    # every weight-gradient call replayed with its own split sum: a deferral window
    # (edet_partials_defer) would record one sum per replay and flush them all at the end
    from tf2mv_amd import runtime as R
    R.DEFER_PARTIALS = False
    x, t = bench.synthetic_batch(anchors, B, S, 1000, dev, model.eng.tdtype)
    model.train_step((x, t))
    torch.cuda.synchronize()

    orig = L.call
    rec = []
    skip = {"edet_memset_async", "edet_memcpy_async", "edet_set_workspace"}

    def timed(name, *a):
        r = orig(name, *a)
        if name in skip or (args.filter and not any(f in name for f in args.filter.split(","))):
            return r
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        orig(name, *a)  # warm
        s.record()
        for _ in range(args.reps):
            orig(name, *a)
        e.record()
        rec.append((name, s, e, bench.algorithmic_bytes(name, a, 2), bench.shape_tag(name, a)))
        return r

    for kv in filter(None, args.dev.split(",")):
        k, v = kv.split("=")
        if L.lib().fns["edet_dev_set"](int(k), int(v)) < 0:
            raise SystemExit("--dev needs the EDET_DEV build: make -C tensorflow2-machine-vision_amd dev; "
                             "EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so")
    L.call = timed  # every package module calls through this one _lib module object
    model.train_step((x, t))
    torch.cuda.synchronize()
    L.call = orig
    if args.dev:
        for i in range(64):
            L.lib().fns["edet_dev_set"](i, 0)

    rows, agg = [], {}
    for name, s, e, b, tag in rec:
        us = s.elapsed_time(e) * 1e3 / args.reps
        rows.append((us, name, tag, b))
        a = agg.setdefault(name, [0, 0.0, 0])
        a[0] += 1
        a[1] += us
        a[2] += b or 0
    rows.sort(reverse=True)
    lines = []
    tot = sum(r[0] for r in rows)
    lines.append(f"total {tot:.1f} us over {len(rows)} calls (replay average, reps={args.reps})")
    for name, (n, us, b) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        gb = f"{b / (us * 1e3):8.1f} GB/s" if b else ""
        lines.append(f"  {name:26s} calls={n:4d} {us:9.1f} us {gb}")
    for us, name, tag, b in rows[: args.top]:
        gb = f"{b / (us * 1e3):8.1f} GB/s" if b else ""
        lines.append(f"{us:9.1f} us  {name:24s} {tag:40s} {gb}")
    txt = "\n".join(lines)
    print(txt)
    if args.seq:
        with open(args.seq, "w") as f:
            for name, s, e, b, tag in rec:
                f.write(f"{s.elapsed_time(e) * 1e3 / args.reps:.2f} {name} {tag}\n")
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
