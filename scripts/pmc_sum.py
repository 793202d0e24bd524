"""Per-kernel averages of rocprofv3 --pmc CSV output directories (one line per kernel name).

    python scripts/pmc_sum.py DIR [DIR ...] [--match SUBSTR]
Counter values are summed over dispatches and divided by the dispatch count of that kernel;
the kernel trace gives the average duration."""
import collections
import csv
import glob
import os
import sys


def summarize(d, match):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in cc:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if match and match not in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    dur = collections.defaultdict(list)
    for f in kt:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if match and match not in k:
                continue
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in agg.items():
        n = max(1, len(disp[k]))
        us = sum(dur[k]) / len(dur[k]) if dur[k] else float("nan")
        vals = " ".join(f"{c}={x / n:.4g}" for c, x in sorted(v.items()))
        print(f"{os.path.basename(d)} | {k[:70]} | n={n} {us:.1f}us | {vals}")


def main():
    args = sys.argv[1:]
    match = ""
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        del args[i:i + 2]
    for d in args:
        summarize(d, match)


if __name__ == "__main__":
    main()
