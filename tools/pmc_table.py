"""Per-kernel averages of every counter in rocprofv3 counter_collection.csv files.

    python tools/pmc_table.py <dir> [<dir> ...]     (one line per kernel and counter)
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"edet::(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:50]


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        n = max(len(v) for v in cs.values())
        print(f"{k}  (dispatches {n})")
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()
