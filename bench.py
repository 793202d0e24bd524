"""EfficientDet-D0 bf16 train-step throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 32] [--dtype bf16]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one full EfficientDet-D0 train step (forward, fused focal+Huber loss, backward,
gradient all-reduce when N>1, L2 + clip + SGD-momentum + EMA, BN moving statistics) over one
synthetic 512x512 batch of 32 images per GPU (weak scaling).  Inputs and targets are resident
in HBM before the timed region.  The step is captured once in a HIP graph and replayed.

Prints ONE JSON line on rank 0 with value = images/s over all ranks, plus
  roofline       : the device kernel with the most time in the step (by base name; the
                   library reports which kernel each call launched): its algorithmic bytes per
                   launch / its average launch duration, timed by wall-clock probes around its
                   launches inside the captured step graph (less the interval of an empty probe
                   pair in the same graph), vs 8 TB/s HBM; `traffic` = PMC
                   HBM bytes per launch from profiles/pmc_traffic.json
  roofline_table : every kernel above 2 % of the step's kernel time (instrumented eager step,
                   HIP events per call): calls, ms, avg us, bytes/launch, GB/s, fraction, PMC ratio
  roofline_step  : all launches' algorithmic bytes / the timed step time
  cpu_baseline   : BASELINE config 1 (D0 forward, one 512x512 image) through the oracle (fp32
                   torch-CPU restatement of the reference semantics, not TF) on the host cores,
                   median of 10 after 2 warm-ups, plus the oracle train step; rank 0 at N=1 only
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def synthetic_batch(anchors, B, size, seed, device, dtype):
    """x ~ U[0,1); 7 GT boxes/image, size log-uniform 16..400 px, aspect U[0.5,2], class U{1..80}."""
    rng = np.random.default_rng(seed)
    x = torch.tensor(rng.random((B, size, size, 3), dtype=np.float32), device=device).to(dtype)
    G = 7
    boxes = np.zeros((B, G, 4), np.float32)
    cls = rng.integers(1, 81, (B, G)).astype(np.int32)
    for b in range(B):
        for k in range(G):
            s = np.exp(rng.uniform(np.log(16), np.log(400)))
            ar = rng.uniform(0.5, 2.0)
            h, w = s * np.sqrt(ar), s / np.sqrt(ar)
            cy, cx = rng.uniform(0, size, 2)
            boxes[b, k] = [cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2]
    t = anchors.generate_targets_batched(torch.tensor(boxes), torch.tensor(cls), torch.full((B,), G, dtype=torch.int32))
    return x, t


# ---------------------------------------------------------------- per-kernel instrumentation
def algorithmic_bytes(name, args, es):
    """Minimum HBM bytes of one launch: every operand read once, every output written once
    (activations in the storage dtype, fp32 statistics / parameters / gradients at 4 B)."""
    from tf2mv_amd import _lib as L

    def rows(p):
        p = getattr(p, "_obj", p)
        return sum(p.batch * p.H[i] * p.W[i] for i in range(p.nseg))

    def obj(x):
        return getattr(x, "_obj", x)

    if name == "edet_conv1x1_fwd":
        p, K, N = args[2], args[3], args[5]
        return rows(p) * (K + N) * es + K * N * es
    if name == "edet_conv1x1_dgrad":
        p, N, K, acc = args[3], args[4], args[6], args[9]
        return rows(p) * (N + K * (1 + acc)) * es + K * N * es
    if name == "edet_conv1x1_dgrad_fold":  # dy, x of the folded value, dx
        p, N, K = args[3], args[4], args[6]
        return rows(p) * (N + 2 * K) * es + K * N * es
    if name == "edet_dwconv_dgrad_fold":  # dy, x, dx (the caller takes this entry only where it
        pout, C, pin = args[2], args[3], args[8]  # launches the folded kernel: ops._dgrad_fold_kernel_route)
        return (rows(pout) + 2 * rows(pin)) * C * es
    if name == "edet_conv1x1_dgrad_sesum":  # dy, W, the gated value's raw y, dx
        p, N, K = args[3], args[4], args[6]
        return rows(p) * (N + 2 * K) * es + K * N * es
    if name == "edet_dwconv_bwd_lazy":  # (dtype, lz, pin, C, k, dyl, pout, w, dx, acc, dw, fold, s): dv, y, x, dx
        pin, C, acc = args[2], args[3], args[9]
        return rows(pin) * (4 + acc) * C * es
    if name == "edet_conv1x1_wgrad":
        p, K, N = args[2], args[3], args[6]
        return rows(p) * (K + N) * es
    if name in ("edet_dwconv_fwd", "edet_dwconv_fwd_squeeze"):
        pin, C, pout = args[2], args[3], args[8]
        return (rows(pin) + rows(pout)) * C * es
    if name == "edet_dwconv_wgrad":
        pin, C, pout = args[2], args[3], args[7]
        return (rows(pin) + rows(pout)) * C * es
    if name == "edet_dwconv_dgrad":
        pout, C, pin, acc = args[2], args[3], args[8], args[9]
        return (rows(pout) + rows(pin) * (1 + acc)) * C * es
    if name == "edet_dwconv_bwd":  # (dtype, lz, pin, C, k, s, dy, pout, w, dx, acc, dw, fold, stream)
        pin, C, pout, acc = args[2], args[3], args[7], args[10]
        return (rows(pout) + rows(pin) * (2 + acc)) * C * es  # dy, x, dx (+ dx read)
    if name == "edet_lazy_materialize":
        return 2 * rows(args[2]) * args[3] * es
    if name == "edet_lazy_bwd_reduce":
        return 2 * rows(args[2]) * args[3] * es
    if name == "edet_lazy_bwd_apply":
        return (3 + args[10]) * rows(args[2]) * args[3] * es
    if name == "edet_detection_loss":
        p, A, NC = args[5], args[6], args[7]
        return rows(p) * A * (2 * NC * es + 2 * 4 * es + 4 + 16)
    if name in ("edet_stem_fwd", "edet_stem_wgrad"):
        B, H, W, Co = args[2], args[3], args[4], args[6]
        return B * H * W * 3 * es + B * ((H + 1) // 2) * ((W + 1) // 2) * Co * es
    if name == "edet_se_squeeze":  # (dtype, lz, B, HW, C, svec, s)
        return args[2] * args[3] * args[4] * es
    if name in ("edet_gate_bn_reduce", "edet_gate_grad"):  # x and dv
        return 2 * args[2] * args[3] * args[4] * es
    if name == "edet_residual_fwd":  # (dtype, lzx, lzres, pyr, C, scale, y, s)
        return 3 * rows(args[3]) * args[4] * es
    if name == "edet_maxpool_fwd":  # (dtype, lz, B, H, W, C, y, s)
        B, H, W, C = args[2], args[3], args[4], args[5]
        return B * (H * W + ((H + 1) // 2) * ((W + 1) // 2)) * C * es
    if name == "edet_maxpool_bwd":  # (dtype, lz, B, H, W, C, dy, dx, acc, s)
        B, H, W, C, acc = args[2], args[3], args[4], args[5], args[8]
        return B * (H * W * (2 + acc) + ((H + 1) // 2) * ((W + 1) // 2)) * C * es
    if name == "edet_maxpool_fwd_taps":  # (dtype, lz, B, H, W, C, y, taps, s): + one tap byte per output
        B, H, W, C = args[2], args[3], args[4], args[5]
        return B * (H * W * es + ((H + 1) // 2) * ((W + 1) // 2) * (es + 1)) * C
    if name == "edet_maxpool_bwd_taps":  # (dtype, B, H, W, C, taps, dy, dx, acc, s): taps + dy, dx
        B, H, W, C, acc = args[1], args[2], args[3], args[4], args[8]
        return B * (H * W * (1 + acc) * es + ((H + 1) // 2) * ((W + 1) // 2) * (es + 1)) * C
    # (dtype, n, fi, w, B, H, W, C, ...); the one-pass backward (_dv, ABI 10) reads the raw F and
    # the value gradient where the two-pass form read y and dF: the same bytes
    if name in ("edet_bifpn_fuse_fwd", "edet_bifpn_fuse_bwd", "edet_bifpn_fuse_bwd_dv"):
        n, fi, B, H, W, C = args[1], obj(args[2]), args[4], args[5], args[6], args[7]
        ins = sum(B * fi[i].H * fi[i].W for i in range(n)) * C * es
        out = B * H * W * C * es
        if name == "edet_bifpn_fuse_fwd":
            return ins + out
        dx = sum(B * fi[i].H * fi[i].W * (1 + fi[i].accumulate) for i in range(n)) * C * es
        return ins + 2 * out + dx  # inputs (weight gradient), y and dF, dx
    if name == "edet_opt_norm":
        return 8 * args[2]
    if name == "edet_opt_apply":  # w, v, ema read+write, g read, compute copy write
        return 7 * 4 * args[4] + es * args[4]
    if name == "edet_count_positives":
        return args[1]
    return None


def shape_tag(name, args):
    """Short description of a launch's problem size (per-call detail table)."""
    def rows(p):
        p = getattr(p, "_obj", p)
        return sum(p.batch * p.H[i] * p.W[i] for i in range(p.nseg))

    def lazy(lz):
        lz = getattr(lz, "_obj", lz)
        return ("bn" if lz.bn.enabled else "") + ("+sw" if lz.act else "") + ("+g" if lz.gate else "")

    try:
        if name == "edet_conv1x1_fwd":
            return f"M={rows(args[2])} K={args[3]} N={args[5]} {lazy(args[1])}"
        if name == "edet_conv1x1_dgrad":
            return f"M={rows(args[3])} N={args[4]} K={args[6]} acc={args[9]}"
        if name == "edet_conv1x1_wgrad":
            return f"M={rows(args[2])} K={args[3]} N={args[6]} {lazy(args[1])}"
        if name in ("edet_dwconv_fwd", "edet_dwconv_wgrad", "edet_dwconv_fwd_squeeze"):
            return f"in={rows(args[2])} C={args[3]} k={args[4]} s={args[5]}"
        if name == "edet_dwconv_bwd":
            return f"in={rows(args[2])} C={args[3]} k={args[4]} s={args[5]}" + (" fold" if args[12] else "")
        if name == "edet_dwconv_dgrad":
            return f"out={rows(args[2])} C={args[3]} k={args[4]} s={args[5]}"
        if name == "edet_conv1x1_dgrad_fold":
            return f"M={rows(args[3])} N={args[4]} K={args[6]} fold"
        if name == "edet_dwconv_dgrad_fold":
            return f"out={rows(args[2])} C={args[3]} k={args[4]} s={args[5]} fold"
        if name == "edet_conv1x1_dgrad_sesum":
            return f"M={rows(args[3])} N={args[4]} K={args[6]} sesum"
        if name == "edet_dwconv_bwd_lazy":
            return f"in={rows(args[2])} C={args[3]} k={args[4]} lazy-dy" + (" fold" if args[11] else "")
        if name in ("edet_lazy_bwd_reduce", "edet_lazy_bwd_apply", "edet_lazy_materialize"):
            return f"M={rows(args[2])} C={args[3]} {lazy(args[1])}"
    except Exception:  # noqa: BLE001
        pass
    return ""


class KernelTimer:
    """Wraps _lib.call: HIP events on the launch stream around every libedet kernel call."""

    def __init__(self, es):
        from tf2mv_amd import _lib as L
        self.L, self.es = L, es
        self.rec = []
        self.orig = L.call

    def __enter__(self):
        L = self.L

        def timed(name, *args):
            if name in ("edet_memset_async", "edet_memcpy_async"):
                return self.orig(name, *args)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            L.launched_kernels()
            s.record()
            r = self.orig(name, *args)
            e.record()
            ks = L.launched_kernels()
            self.rec.append((name, s, e, algorithmic_bytes(name, args, self.es), shape_tag(name, args),
                             ks[0] if ks else name))
            return r

        L.call = timed
        import tf2mv_amd.ops, tf2mv_amd.model, tf2mv_amd.runtime, tf2mv_amd.anchors  # noqa
        for mod in (tf2mv_amd.ops, tf2mv_amd.model, tf2mv_amd.runtime, tf2mv_amd.anchors):
            mod.L.call = timed  # modules hold the _lib module object; patching it once suffices
        return self

    def __exit__(self, *exc):
        self.L.call = self.orig

    def empty_pairs(self):
        """N_EMPTY begin/end pairs with nothing between them, on the current stream (captured with
        the step): their average interval is the dependent-launch boundary the end probe adds to
        every timed launch (the begin probe runs before the kernel's own boundary)."""
        import ctypes
        from tf2mv_amd.runtime import stream
        st = stream()
        for k in range(self.N_EMPTY):
            slot = ctypes.c_void_p(self.slots.data_ptr() + 24 * (self.max_calls + k))
            self.orig("edet_probe", slot, 0, st)
            self.orig("edet_probe", slot, 1, st)

    def detail(self, path, top=2000):
        """Per-call table (slowest first): name, shape, us, achieved GB/s."""
        torch.cuda.synchronize()
        rows = []
        for name, s, e, b, tag, kern in self.rec:
            ms = s.elapsed_time(e)
            rows.append((ms, name, tag, (b / (ms * 1e6)) if (b and ms > 0) else None, b or 0, kern))
        rows.sort(reverse=True)
        with open(path, "w") as f:
            for ms, name, tag, gbs, b, kern in rows[:top]:
                g = "" if gbs is None else f"{gbs:8.1f} GB/s"
                f.write(f"{ms * 1e3:9.1f} us  {name:24s} {tag:40s} {g:14s} {b:12d} B  {kern}\n")

    def summary(self, by="entry"):
        """Per entry point (by="entry") or per device kernel (by="kernel", the first kernel a
        call launched): [calls, ms, algorithmic bytes, all bytes known, entry points]."""
        torch.cuda.synchronize()
        agg = {}
        for name, s, e, b, _, kern in self.rec:
            ms = s.elapsed_time(e)
            a = agg.setdefault(name if by == "entry" else kern, [0, 0.0, 0.0, True, set()])
            a[0] += 1
            a[1] += ms
            a[4].add(name)
            if b is None:
                a[3] = False
            else:
                a[2] += b
        return agg


class ProbeTimer:
    """Wraps every launch of the C-ABI functions ``funcs`` with edet_probe begin/end on its
    stream.  The probes are ordinary kernels, so they can be captured into the step's HIP graph
    (timing events cannot): replaying K captured steps accumulates each launch's duration on the
    GPU's constant-rate wall clock.  Only calls that launched exactly the device kernel
    ``kernel`` count in the result (an entry point may pick different kernels per shape)."""

    N_EMPTY = 64  # back-to-back begin/end probe pairs: the probes' own boundary, subtracted

    def __init__(self, funcs, kernel, es, max_calls=1024):
        from tf2mv_amd import _lib as L
        self.L, self.funcs, self.kernel, self.es = L, set(funcs), kernel, es
        self.slots = torch.zeros((max_calls + self.N_EMPTY) * 3, dtype=torch.int64, device="cuda")
        self.max_calls = max_calls
        self.bytes, self.match = [], []
        self.orig = L.call

    def __enter__(self):
        import ctypes
        L = self.L

        def probed(name, *args):
            if name not in self.funcs:
                return self.orig(name, *args)
            i = len(self.bytes)
            assert i < self.max_calls
            slot = ctypes.c_void_p(self.slots.data_ptr() + 24 * i)
            st = args[-1]  # every entry point takes its stream last
            self.orig("edet_probe", slot, 0, st)
            L.launched_kernels()
            r = self.orig(name, *args)
            ks = L.launched_kernels()
            self.orig("edet_probe", slot, 1, st)
            self.bytes.append(algorithmic_bytes(name, args, self.es))
            self.match.append(ks == [self.kernel])
            return r

        L.call = probed
        import tf2mv_amd.ops, tf2mv_amd.model, tf2mv_amd.runtime, tf2mv_amd.anchors  # noqa
        for mod in (tf2mv_amd.ops, tf2mv_amd.model, tf2mv_amd.runtime, tf2mv_amd.anchors):
            mod.L.call = probed
        return self

    def __exit__(self, *exc):
        self.L.call = self.orig

    def empty_pairs(self):
        """N_EMPTY begin/end pairs with nothing between them, on the current stream (captured with
        the step): their average interval is the dependent-launch boundary the end probe adds to
        every timed launch (the begin probe runs before the kernel's own boundary)."""
        import ctypes
        from tf2mv_amd.runtime import stream
        st = stream()
        for k in range(self.N_EMPTY):
            slot = ctypes.c_void_p(self.slots.data_ptr() + 24 * (self.max_calls + k))
            self.orig("edet_probe", slot, 0, st)
            self.orig("edet_probe", slot, 1, st)

    def result(self):
        import ctypes
        torch.cuda.synchronize()
        khz = ctypes.c_int(0)
        self.orig("edet_wall_clock_khz", ctypes.byref(khz))
        n = len(self.bytes)
        sl = self.slots.view(-1, 3)[:n].cpu()
        sel = [i for i in range(n) if self.match[i] and self.bytes[i] is not None]
        launches = int(sum(int(sl[i, 2]) for i in sel))
        ticks = int(sum(int(sl[i, 1]) for i in sel))
        raw_us = ticks / max(launches, 1) / (khz.value / 1000.0)
        em = self.slots.view(-1, 3)[self.max_calls:self.max_calls + self.N_EMPTY].cpu()
        e_n = int(em[:, 2].sum())
        overhead_us = (int(em[:, 1].sum()) / e_n / (khz.value / 1000.0)) if e_n else 0.0
        # the headline is the raw probe interval (subtracting the empty pair's whole
        # interval took the average below rocprof's kernel duration); the corrected figure is
        # reported beside it, never used for `achieved`
        avg_us = raw_us
        corr_us = raw_us - overhead_us if raw_us > overhead_us else raw_us
        bpl = sum(self.bytes[i] for i in sel) / max(len(sel), 1)
        return {"launches": launches, "calls_per_step": len(sel), "avg_launch_us": avg_us,
                "avg_launch_us_raw": raw_us, "avg_launch_us_less_probe_pair": corr_us,
                "probe_overhead_us": overhead_us, "bytes_per_launch": bpl,
                "achieved_GBps": bpl / avg_us * 1e-3 if avg_us > 0 else None, "clock_khz": khz.value}


def probe_roofline(step_fn, funcs, kernel, steps, es):
    """Average launch duration of ``kernel`` (launched from the entry points ``funcs``) over
    ``steps`` replays of a captured graph of ``step_fn`` (one eager step) that carries the
    probes, and its algorithmic bytes per launch."""
    pt = ProbeTimer(funcs, kernel, es)
    with pt:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step_fn()
            pt.empty_pairs()
    g.replay()  # warm
    torch.cuda.synchronize()
    pt.slots.zero_()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    r = pt.result()
    r["ms_per_step"] = (time.perf_counter() - t0) / steps * 1e3
    del g
    return r


# workload key of this run ("efficientdet-d0 train B=32 S=512 bf16"); a PMC summary made from
# another workload (scripts/pmc_*.py --workload) is not evidence about this one
WORKLOAD_KEY = None


def workload_key(model, kind, B, S, dtype):
    return f"{model} {kind} B={B} S={S} {dtype}"


def _pmc_entry(fname, kernel, calls_per_step):
    """``kernel``'s entry of a committed rocprofv3 PMC summary under profiles/, or None when
    absent or stale: the summary's workload key must be this run's, and the profiled run's
    dispatches per step must equal the launches this step makes (a summary from an older tree
    counts other launches)."""
    path = os.path.join(ROOT, "profiles", fname)
    try:
        with open(path) as f:
            d = json.load(f)
        if WORKLOAD_KEY is None or d.get("workload") != WORKLOAD_KEY:
            return None
        k = d.get("kernels", {}).get(kernel)
        if k is None:
            return None
        per = k.get("dispatches_per_step")
        if per is None or calls_per_step is None or abs(per - calls_per_step) > 0.5:
            return None
        return k
    except (OSError, ValueError, KeyError):
        return None


def pmc_traffic(kernel, calls_per_step=None):
    """HBM bytes per launch of ``kernel`` from profiles/pmc_traffic.json (two PMC passes,
    FETCH_SIZE x2 + WRITE_SIZE per the gfx950 correction; scripts/pmc_traffic.py), or None."""
    k = _pmc_entry("pmc_traffic.json", kernel, calls_per_step)
    return None if k is None else float(k["traffic_bytes_per_launch"])


def pmc_mfma(kernel, calls_per_step=None):
    """Fraction of the chip's MFMA issue cycles ``kernel`` used (SQ_VALU_MFMA_BUSY_CYCLES over
    1024 SIMDs x the kernel's cycles, profiles/pmc_mfma.json from scripts/pmc_mfma.py), or None."""
    k = _pmc_entry("pmc_mfma.json", kernel, calls_per_step)
    return None if k is None else float(k["mfma_busy_frac"])


def pmc_limiter(kernel, calls_per_step=None, hbm_frac=None):
    """What bounds ``kernel`` (profiles/pmc_limiter.json, two PMC passes of wave-time breakdown,
    instruction mix, LDS conflicts and L2 hits; scripts/pmc_limiter.py): (limiter line, the
    counter-derived fractions behind it), or (None, None)."""
    k = _pmc_entry("pmc_limiter.json", kernel, calls_per_step)
    if k is None:
        return None, None
    from scripts.pmc_limiter import limiter_from
    keep = ("waves_per_simd", "wait_frac", "issue_stall_frac", "active_valu_frac", "active_lds_frac",
            "active_vmem_frac", "lds_conflict_rate", "l2_hit")
    return limiter_from(k, hbm_frac), {n: round(float(k[n]), 3) for n in keep if n in k}


def _cpu_share():
    """Host cores this process may use: the affinity set, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(model, anchors, fwd_runs=10, train_runs=3):
    """BASELINE config 1 on the host: the EfficientDet-D0 forward on one 512x512 image
    (inference-mode BN, moving statistics (0, 1) as initialised) through the oracle -- the
    fp32 torch-CPU restatement of the reference's TF2 semantics, not TF itself, which is not
    installable here -- on every core this process may use; median of ``fwd_runs`` after two
    warm-ups.  Second field: the oracle's fp32 train step (forward + loss + backward) on one
    image with bench-like targets (7 GT boxes), median of ``train_runs`` after one warm-up."""
    from oracle import ref_anchors as RA
    from oracle.ref_model import RefEfficientDet
    cores = _cpu_share()
    torch.set_num_threads(cores)
    ref = RefEfficientDet(model.cfg, model.state_dict(), dtype=torch.float32)
    cfg = model.cfg
    S = cfg.image_size
    rng = np.random.default_rng(0)
    x = rng.random((1, S, S, 3), dtype=np.float32)

    def med(fn, warm, runs):
        for _ in range(warm):
            fn()
        ts = []
        for _ in range(runs):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), ts

    with torch.no_grad():
        fwd_s, fwd_ts = med(lambda: ref.forward(x, False), 2, fwd_runs)
    # train-step field: realistic targets (bench.py's synthetic GT, oracle target encoding)
    G = 7
    boxes = np.zeros((G, 4), np.float32)
    for k in range(G):
        sz = np.exp(rng.uniform(np.log(16), np.log(400)))
        ar = rng.uniform(0.5, 2.0)
        h, w = sz * np.sqrt(ar), sz / np.sqrt(ar)
        cy, cx = rng.uniform(0, S, 2)
        boxes[k] = [cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2]
    cls = rng.integers(1, cfg.num_classes, G)
    lv = RA.generate_boxes(cfg.min_level, cfg.max_level, (S, S), cfg.num_scales, cfg.aspect_ratios, cfg.anchor_scale)
    ob, oc, om, _ = RA.generate_targets(lv, boxes, cls, cfg.num_classes)
    yb, yc, ym = [b[None] for b in ob], [c[None] for c in oc], [mm[None] for mm in om]
    keys = [k for k in ref.p if not k.endswith(("moving_mean", "moving_variance"))]

    def train_once():
        for k in keys:
            ref.p[k].requires_grad_(True)
        box, cl = ref.forward(x, True)
        loss, _ = ref.detection_loss(box, cl, yb, yc, ym)
        torch.autograd.grad(loss, [ref.p[k] for k in keys], allow_unused=True)

    tr_s, tr_ts = med(train_once, 1, train_runs)
    npos = int(sum(np.asarray(m).sum() for m in ym))
    return {"value": round(1.0 / fwd_s, 4), "unit": "images/s", "cores": cores, "kind": "port",
            "config": "BASELINE config 1: EfficientDet-D0 forward, one 512x512 image, CPU",
            "sample": f"median of {fwd_runs} single-image D0 forwards (inference BN) after 2 warm-ups, oracle fp32 "
                      f"torch-CPU restatement of the reference TF2 semantics (not TF); runs "
                      + ", ".join(f"{t:.3f}" for t in fwd_ts) + " s",
            "cpu_model": _cpu_model(),
            "train_step": {"value": round(1.0 / tr_s, 4), "unit": "images/s",
                           "sample": f"median of {train_runs} one-image fp32 train steps (forward + focal/Huber "
                                     f"loss + backward), 7 GT boxes -> {npos} positive anchors, after 1 warm-up"}}


def kernel_tables(step_fn, args, el):
    """One eager ``step_fn`` under HIP events per library call -> (roofline of the kernel with
    the most step time, timed by probes in a captured graph of the step; roofline_table of every
    kernel above 2 % of the kernel time; roofline_step; per-entry-point summary)."""
    es = 2 if args.dtype == "bf16" else 4
    roofline = None
    with KernelTimer(es) as kt:
        step_fn()
    agg = kt.summary()
    kag = kt.summary("kernel")
    if os.environ.get("EDET_KERNEL_DETAIL"):
        kt.detail(os.environ["EDET_KERNEL_DETAIL"])
    total_ms = sum(a[1] for a in agg.values())
    top = sorted(agg.items(), key=lambda kv: -kv[1][1])
    kernels = {k: {"calls": a[0], "ms": round(a[1], 4), "GBps": (round(a[2] / (a[1] * 1e6), 1) if a[3] and a[1] > 0 else None)}
               for k, a in top[:12]}
    log(f"[bench] instrumented eager step: {total_ms:.2f} ms of kernel time")
    for k, a in top[:12]:
        log(f"   {k:28s} calls={a[0]:4d} ms={a[1]:8.3f} share={a[1] / total_ms * 100:5.1f}%"
            + (f" {a[2] / (a[1] * 1e6):8.1f} GB/s" if a[3] else ""))
    # per device kernel (base name: a kernel's compile-time cases are one kernel, as rocprof
    # rows are summed in profiles/): every kernel above 2 % of the step's kernel time
    ktop = sorted(kag.items(), key=lambda kv: -kv[1][1])
    table = []
    for k, a in ktop:
        if a[1] < 0.02 * total_ms:
            continue
        gbs = a[2] / (a[1] * 1e6) if a[3] and a[1] > 0 else None
        tr = pmc_traffic(k, a[0])
        mf = pmc_mfma(k, a[0])
        lim, lim_pmc = pmc_limiter(k, a[0], None if gbs is None else gbs / HBM_PEAK_GBS)
        table.append({"kernel": k, "calls": a[0], "ms": round(a[1], 4), "share": round(a[1] / total_ms, 4),
                      "avg_us": round(a[1] * 1e3 / a[0], 2),
                      "bytes_per_launch": round(a[2] / a[0]) if a[3] else None,
                      "achieved_GBps": None if gbs is None else round(gbs, 1),
                      "frac": None if gbs is None else round(gbs / HBM_PEAK_GBS, 4),
                      "pmc_traffic_ratio": (round(tr / (a[2] / a[0]), 3) if (tr and a[3] and a[2]) else None),
                      "mfma_frac": None if mf is None else round(mf, 4),
                      "limiter": lim, "limiter_pmc": lim_pmc,
                      "entry_points": sorted(a[4])})
    known = sum(a[2] for a in kag.values() if a[3])
    step_level = {"algorithmic_bytes": round(known), "ms_per_step": round(el / args.steps * 1e3, 3),
                  "achieved_GBps": round(known / (el / args.steps) * 1e-9, 1),
                  "frac": round(known / (el / args.steps) * 1e-9 / HBM_PEAK_GBS, 4),
                  "note": "sum of every launch's algorithmic bytes (launches with a formula: "
                          f"{sum(a[0] for a in kag.values() if a[3])} of {sum(a[0] for a in kag.values())}) "
                          "over the timed step"}
    # headline roofline: the kernel with the most time in the step, its launches timed by
    # wall-clock probes inside the captured step graph
    dom = next(((k, a) for k, a in ktop if a[3]), None)
    if dom is not None and args.graph:
        kname, a = dom
        pr = probe_roofline(step_fn, a[4], kname, args.steps, es)
        ach = pr["achieved_GBps"]
        traffic = pmc_traffic(kname, a[0])
        roofline = {"bound": "hbm", "kernel": kname, "entry_points": sorted(a[4]), "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": None if traffic is None else round(traffic),
                    "bytes_per_launch": round(pr["bytes_per_launch"]), "avg_launch_us": round(pr["avg_launch_us"], 2),
                    "avg_launch_us_less_probe_pair": round(pr["avg_launch_us_less_probe_pair"], 2),
                    "probe_overhead_us": round(pr["probe_overhead_us"], 2),
                    "launches": pr["launches"], "share_of_kernel_time": round(a[1] / total_ms, 4),
                    "timing": "wall-clock probes in the captured step graph, "
                    f"{args.steps} replays ({pr['ms_per_step']:.2f} ms/step with probes); avg_launch_us is "
                    "the raw begin-to-end probe interval (it includes the probes' own launch boundary, so "
                    "it is an upper bound on the kernel's duration); avg_launch_us_less_probe_pair "
                    f"subtracts the interval of {ProbeTimer.N_EMPTY} empty begin/end pairs in the same graph"}
        log(f"[bench] roofline {kname}: {pr['launches']} launches, avg {pr['avg_launch_us']:.2f} us raw "
            f"({pr['avg_launch_us_less_probe_pair']:.2f} less {pr['probe_overhead_us']:.2f} probe pair), "
            f"{pr['bytes_per_launch'] / 1e6:.2f} MB/launch -> {ach:.1f} GB/s")
    return roofline, table, step_level, kernels


def bench_backbone(args):
    """BASELINE config 2: EfficientNet-B0 backbone forward (inference BN), 224x224, one GPU,
    B = --batch (64 for the config).  Same timing contract as the train step."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from tf2mv_amd import dist as dp
    from tf2mv_amd.config import efficientnet_b0_blocks, get_efficientdet_config
    from tf2mv_amd.model import EfficientDetNet

    ctx = dp.init_from_env("nccl", dev)
    world, rank = ctx.world, ctx.rank
    cfg = get_efficientdet_config("efficientdet-d0", {"image_size": 224})
    B = args.batch
    global WORKLOAD_KEY
    WORKLOAD_KEY = workload_key("efficientnet-b0", "backbone", B, 224, args.dtype)
    model = EfficientDetNet(efficientnet_b0_blocks(), cfg, dtype=args.dtype, device=dev, seed=0)
    rng = np.random.default_rng(1000 + rank)
    x = torch.tensor(rng.random((B, 224, 224, 3), dtype=np.float32), device=dev).to(model.eng.tdtype)
    for _ in range(2):
        model.backbone(x, training=False)
    torch.cuda.synchronize()
    step = lambda: model.backbone(x, training=False)  # noqa: E731
    if args.graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            model.backbone(x, training=False)
        step = g.replay
    for _ in range(args.warmup):
        step()
    el = dp.timed(ctx, step, args.steps, torch.cuda.synchronize)
    el = dp.max_over_ranks(ctx, el, dev)
    value = world * B * args.steps / el
    log(f"[bench] backbone B0@224 B={B}/gpu: {args.steps} steps in {el:.3f}s -> {value:.1f} img/s")
    roofline = table = step_level = kernels = None
    if args.kernel_timing and rank == 0:
        roofline, table, step_level, kernels = kernel_tables(lambda: model.backbone(x, training=False), args, el)
    if rank == 0:
        print(json.dumps({
            "metric": "EfficientNet-B0 backbone forward images/sec", "value": round(value, 2), "unit": "images/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic",
            "config": {"workload": f"efficientnet-b0 backbone forward 224x224, B={B}/GPU, inference BN",
                       "model": "efficientnet-b0", "global_batch": B * world, "image_size": 224,
                       "parallelism": f"dp{world}", "graph": bool(args.graph)},
            "roofline": roofline, "roofline_table": table, "roofline_step": step_level, "kernels": kernels}),
            flush=True)
    dp.shutdown(ctx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--model", default="efficientdet-d0")
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--kernel-timing", type=int, default=1)
    ap.add_argument("--overlap", type=int, default=0, help="weight gradients on a side stream")
    ap.add_argument("--workload", default="train", choices=["train", "backbone"],
                    help="train: the headline D0 train step; backbone: BASELINE config 2 (B0 @224 forward)")
    args = ap.parse_args()
    if args.workload == "backbone":
        return bench_backbone(args)

    # EDET_DP_BACKEND=gloo with more ranks than GPUs rehearses the N > 1 path on one GPU
    # (ranks share devices round-robin); the default is one rank per GPU over RCCL
    backend = os.environ.get("EDET_DP_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from tf2mv_amd import dist as dp

    ctx = dp.init_from_env(backend, dev)  # RCCL over xGMI for N > 1
    world, rank = ctx.world, ctx.rank

    from tf2mv_amd.anchors import Anchors
    from tf2mv_amd.config import efficientnet_b0_blocks, get_efficientdet_config
    from tf2mv_amd.model import EfficientDetNetTrain

    cfg = get_efficientdet_config(args.model)
    S, B = cfg.image_size, args.batch
    global WORKLOAD_KEY
    WORKLOAD_KEY = workload_key(args.model, "train", B, S, args.dtype)
    anchors = Anchors(cfg.min_level, cfg.max_level, (S, S), cfg.num_scales, cfg.aspect_ratios, cfg.anchor_scale, device=dev)
    ar = dp.make_allreduce(ctx)
    model = EfficientDetNetTrain(efficientnet_b0_blocks(), cfg, anchors, dtype=args.dtype, device=dev, seed=0,
                                 world_size=world, grad_allreduce=ar, npos_allreduce=ar, rank=rank,
                                 lr_schedule={"warmup_steps": 100, "total_steps": 10000,
                                              "adjusted_lr": 0.08 * B * world / 64})
    model.eng.overlap = bool(args.overlap)
    x, t = synthetic_batch(anchors, B, S, 1000 + rank, dev, model.eng.tdtype)
    data = (x, t)
    log(f"[bench] {args.model} B={B}/gpu world={world} dtype={args.dtype} params={model.P.n_trainable}")

    # eager warm-up (allocates persistent buffers), then capture
    for _ in range(2):
        model.train_step(data)
    torch.cuda.synchronize()
    log(f"[bench] eager warm-up ok, loss={float(model.scalars[0]):.4f} gnorm={float(model.scalars[3]):.4f}")

    step = lambda: model.train_step(data)  # noqa: E731
    if args.graph:
        # one graph at N = 1; at N > 1 prepare | N+ all-reduce | compute | gradient
        # all-reduce | optimizer, the collectives between the captured graphs
        step = dp.graphed_train_step(model, data, ar)
        torch.cuda.synchronize()
        log("[bench] graph captured")

    for i in range(args.warmup):
        step()
    el = dp.timed(ctx, step, args.steps, torch.cuda.synchronize)
    el = dp.max_over_ranks(ctx, el, dev)
    value = world * B * args.steps / el
    # global-batch loss: the replicas' data terms sum to it (Multi-GPU); each
    # replica's scalars[0] also holds the (identical) L2 term once
    scal_timed = model.scalars.cpu()  # the last timed step's scalars (rank 0's instrumentation reruns them)
    lt = model.scalars[0:1].clone()
    if ar is not None:
        ar(lt)
    l2 = float(model.sched.l2_weight) * 0.5 * float(model.scalars[2])
    loss = float(lt) - (world - 1) * l2
    gnorm = float(model.scalars[3])
    log(f"[bench] {args.steps} steps in {el:.3f}s -> {value:.1f} img/s  loss={loss:.4f} gnorm={gnorm:.4f}")

    roofline = kernels = table = step_level = None
    if args.kernel_timing and rank == 0:
        # the instrumented steps below run on rank 0 alone: snapshot the optimizer-visible
        # state and restore it afterwards so rank 0 leaves in step with the other replicas
        P = model.P
        saved = [(t, t.clone()) for t in (P.w, P.v, P.ema, P.bn_mm, P.bn_mv, model.step_counter)]
        if ctx.distributed:
            model.grad_allreduce = None
            model.npos_allreduce = None
        model.eng.overlap = False  # per-kernel attribution: one stream, no concurrency
        roofline, table, step_level, kernels = kernel_tables(lambda: model.train_step(data), args, el)
        model.eng.overlap = bool(args.overlap)
        for t, c in saved:
            t.copy_(c)
        P.refresh_compute_copy()
        model.grad_allreduce, model.npos_allreduce = ar, ar

    cpu = None
    if args.cpu_baseline and rank == 0 and world == 1:
        log("[bench] cpu baseline (oracle, fp32) ...")
        cpu = cpu_baseline(model, anchors)
        log(f"[bench] cpu baseline {cpu['value']:.3f} img/s on {cpu['cores']} threads")

    if rank == 0:
        out = {
            "metric": f"EfficientDet-{args.model.split('-')[-1].upper()} bf16 train-step images/sec",
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic",
            "config": {"workload": f"{args.model} full train step {S}x{S}, B={B}/GPU, focal+Huber loss, SGD+EMA",
                       "model": args.model, "global_batch": B * world, "image_size": S,
                       "parallelism": f"dp{world}", "graph": bool(args.graph)},
            "loss": round(loss, 5),  # global-batch loss of the last timed step
            "gnorm": round(gnorm, 5),
            "roofline": roofline,
            "roofline_table": table,
            "roofline_step": step_level,
            "cpu_baseline": cpu,
            "kernels": kernels,
        }
        print(json.dumps(out), flush=True)
    dump = os.environ.get("EDET_BENCH_DUMP")
    if dump:
        # test hook (tests/test_bench_dp_gpu.py): every rank's optimizer-visible state after the
        # run, so replicas can be compared bit for bit (rank 0 after its instrumentation restore)
        P = model.P
        torch.save({"w": P.w.cpu(), "v": P.v.cpu(), "ema": P.ema.cpu(), "step": model.step_counter.cpu(),
                    "scalars": scal_timed, "l2_term": l2, "loss": loss, "value": value, "world": world},
                   os.path.join(dump, f"rank{rank}.pt"))
    dp.shutdown(ctx)


if __name__ == "__main__":
    main()
