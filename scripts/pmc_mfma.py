"""MFMA utilisation per kernel from one rocprofv3 PMC pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d <dir> -o run \\
        --output-format csv -- python bench.py --steps 3 --warmup 1 --graph 0 --cpu-baseline 0 --kernel-timing 0
    python scripts/pmc_mfma.py --dir <dir> --out profiles/pmc_mfma.json

SQ_VALU_MFMA_BUSY_CYCLES counts MFMA busy cycles summed over every SIMD (32 per
v_mfma_f32_32x32x16_bf16, 16 per 16x16x32; MI355X_MICROARCH.md, cycle constants);
GRBM_GUI_ACTIVE is the kernel's GPU-busy cycles summed over the 8 XCDs.  The fraction of the
chip's matrix issue capacity a kernel used is therefore
    mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8).
(ROCm 7.2 ships no gfx950 derived-counter formulas; this is the definition used here.)
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--tag", default="")
    ap.add_argument("--workload", default="efficientdet-d0 train B=32 S=512 bf16",
                    help="workload key of the profiled command (bench.py workload_key()); bench.py ignores a "
                         "summary whose key differs from the run it reports")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {a.dir}")
    acc = collections.defaultdict(lambda: {"mfma": 0.0, "grbm": 0.0, "ids": set()})
    for f in files:
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            did = row.get("Dispatch_Id") or row.get("Correlation_Id")
            if row.get("Counter_Name") == "SQ_VALU_MFMA_BUSY_CYCLES":
                acc[k]["mfma"] += float(row["Counter_Value"])
            elif row.get("Counter_Name") == "GRBM_GUI_ACTIVE":
                acc[k]["grbm"] += float(row["Counter_Value"])
            acc[k]["ids"].add(did)
    out = {"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE; mfma_busy_frac = MFMA busy cycles / "
                     "(1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)", "tag": a.tag, "workload": a.workload, "steps": a.steps, "kernels": {}}
    for k, v in acc.items():
        n = len(v["ids"])
        if not n or v["grbm"] <= 0:
            continue
        out["kernels"][k] = {"dispatches": n, "dispatches_per_step": n / a.steps,
                             "mfma_busy_cycles_per_launch": v["mfma"] / n, "gui_active_per_launch": v["grbm"] / n,
                             "mfma_busy_frac": v["mfma"] / (1024.0 * v["grbm"] / 8.0)}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["mfma_busy_cycles_per_launch"] * kv[1]["dispatches"]):
        if v["mfma_busy_cycles_per_launch"] > 0:
            print(f"{k:28s} n={v['dispatches']:5d}  mfma_busy_frac {v['mfma_busy_frac']:.4f}")


if __name__ == "__main__":
    main()
