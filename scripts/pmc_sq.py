"""Summarise SQ counter passes (rocprofv3 --pmc ... --kernel-trace, csv) per kernel: mean per
dispatch of every counter found under the given directories, plus the usual ratios.
    python scripts/pmc_sq.py DIR [DIR ...]"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                m = re.search(r"edet::(k_\w+)", row["Kernel_Name"])
                k = m.group(1) if m else row["Kernel_Name"][:40]
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in acc.items():
        v = {c: sum(x) / len(x) for c, x in cs.items()}
        print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())})
        wc = v.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in v:
                    print(f"   {c}/WAVE_CYCLES = {v[c] / wc:.3f}")
        if "SQ_INSTS_LDS" in v and "SQ_LDS_BANK_CONFLICT" in v:
            print(f"   bank conflict cycles per LDS inst = {v['SQ_LDS_BANK_CONFLICT'] / max(1, v['SQ_INSTS_LDS']):.3f}")


if __name__ == "__main__":
    main()
