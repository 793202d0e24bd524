"""Per-launch table of a kbench plan sweep (tools/gpu_run.sh kbench writes DIR/kb_<variant>_<rep>.txt):
python tools/sweep_table.py DIR BASELINE_VARIANT [--min-gain 0.05]"""
import collections
import glob
import os
import re
import sys


def load(f):
    d = collections.defaultdict(list)
    for line in open(f):
        m = re.match(r'\s+([\d.]+) us\s+(edet_\w+)\s+(.*?)\s{2,}', line)
        if m:
            d[(m.group(2), m.group(3).strip())].append(float(m.group(1)))
    return d


def main():
    path, base = sys.argv[1], sys.argv[2]
    gain = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
    runs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "kb_*_*.txt")):
        v = os.path.basename(f)[3:-4].rsplit("_", 1)[0]
        runs[v].append(load(f))
    R = {}
    for v, tabs in runs.items():
        agg = collections.defaultdict(float)
        for t in tabs:
            for k, xs in t.items():
                agg[k] += sum(xs) / len(tabs)
        R[v] = agg
    vs = [base] + sorted(v for v in R if v != base)
    best_total = 0.0
    for k in sorted(R[base], key=lambda k: -R[base][k]):
        vals = {v: R[v].get(k, 1e9) for v in vs}
        b = min(vals, key=vals.get)
        best_total += vals[b]
        if vals[b] < (1 - gain) * vals[base]:
            print(f"{k[0][5:]:18s} {k[1]:30s} base {vals[base]:7.1f}  best {b:>8s} {vals[b]:7.1f}  " +
                  " ".join(f"{v}:{vals[v]:.1f}" for v in vs[1:]))
    print("totals " + " ".join(f"{v}:{sum(R[v].values()):.1f}" for v in vs) + f" per-launch-best:{best_total:.1f}")


main()
