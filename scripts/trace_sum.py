"""Per-kernel time of one graph-replayed step from a rocprofv3 --kernel-trace CSV directory.

    python scripts/trace_sum.py DIR [top] [match]
The step is the span between the last two launches of k_dropmask (the step's first kernel)."""
import collections
import csv
import glob
import re
import sys


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    match = sys.argv[3] if len(sys.argv) > 3 else ""
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "k_dropmask" in r["Kernel_Name"]]
    seg = rows[idx[-2]:idx[-1]]
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        k = re.sub(r"\(.*", "", re.sub(r"<.*", "", r["Kernel_Name"]).replace("void ", "").replace("edet::", ""))
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"kernels {len(seg)}  span {span:.1f} us  kernel sum {tot:.1f} us")
    # idle time between consecutive kernels of the step (graph node boundaries)
    gaps = []
    for a, b in zip(seg, seg[1:]):
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        gaps.append((g, re.sub(r"<.*|\(.*", "", a["Kernel_Name"].replace("void ", "").replace("edet::", "")),
                     re.sub(r"<.*|\(.*", "", b["Kernel_Name"].replace("void ", "").replace("edet::", ""))))
    gs = sorted(g for g, _, _ in gaps)
    if gs:
        print(f"gaps: sum {sum(gs):.1f} us over {len(gs)}, median {gs[len(gs) // 2]:.2f}, "
              f"p90 {gs[int(len(gs) * 0.9)]:.2f}, max {gs[-1]:.2f}, negative (overlap) {sum(1 for g in gs if g < 0)}")
        for g, a, b in sorted(gaps, reverse=True)[:8]:
            print(f"   gap {g:7.2f} us  {a} -> {b}")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        if match in k:
            print(f"{k:28s} {n:4d} {t:9.1f} us {100 * t / tot:5.1f}%  avg {t / n:7.2f}")


if __name__ == "__main__":
    main()
