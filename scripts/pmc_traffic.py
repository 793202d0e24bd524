"""HBM traffic per launch from two rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d <fetch_dir> -o run --output-format csv -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d <write_dir> -o run --output-format csv -- python bench.py ...
    python scripts/pmc_traffic.py --fetch <fetch_dir> --write <write_dir> --out profiles/pmc_traffic.json

FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950 (TCC slots).  Both are derived
counters in KiB.  On gfx950 FETCH_SIZE reports half of the bytes of wide coalesced streaming
reads (128-B requests tallied at 64 B), so reads are doubled; WRITE_SIZE is exact for 16-B
streaming stores.  Output: per kernel (short name), mean bytes per dispatch.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name):
    m = re.search(r"edet::(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:60]


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = collections.defaultdict(lambda: [0.0, set()])
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            k = short(row["Kernel_Name"])
            acc[k][0] += float(row["Counter_Value"])
            acc[k][1].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    return {k: (v[0], len(v[1])) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=6,
                    help="train steps the profiled command ran (bench.py --steps 3 --warmup 1 --graph 0: 2 eager "
                         "warm-ups + 1 + 3); bench.py uses dispatches / steps to reject a stale entry")
    ap.add_argument("--tag", default="")
    ap.add_argument("--workload", default="efficientdet-d0 train B=32 S=512 bf16",
                    help="workload key of the profiled command (bench.py workload_key()); bench.py ignores a "
                         "summary whose key differs from the run it reports")
    a = ap.parse_args()
    fe = per_kernel(a.fetch, "FETCH_SIZE")
    wr = per_kernel(a.write, "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), KiB per dispatch; "
                     "read bytes = 2 x FETCH_SIZE (gfx950 correction), write bytes = WRITE_SIZE",
           "tag": a.tag, "workload": a.workload, "steps": a.steps, "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        f_kib, nf = fe.get(k, (0.0, 0))
        w_kib, nw = wr.get(k, (0.0, 0))
        if not nf or not nw:
            continue
        rd = 2.0 * f_kib * 1024.0 / nf
        wb = w_kib * 1024.0 / nw
        out["kernels"][k] = {"dispatches": nf, "dispatches_per_step": nf / a.steps, "read_bytes_per_launch": rd,
                             "write_bytes_per_launch": wb, "traffic_bytes_per_launch": rd + wb}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["traffic_bytes_per_launch"] * kv[1]["dispatches"])[:25]:
        print(f"{k:28s} n={v['dispatches']:5d}  read {v['read_bytes_per_launch'] / 1e6:9.2f} MB  "
              f"write {v['write_bytes_per_launch'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
