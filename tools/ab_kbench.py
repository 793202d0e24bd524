"""Same-box A/B of two kbench tables per entry point and per launch (tools/gpu_run.sh kbench writes
kb_<i>_old.txt / kb_<i>_new.txt): python tools/ab_kbench.py DIR"""
import collections
import glob
import os
import re
import sys


def load(f):
    d, e = collections.defaultdict(list), {}
    for line in open(f):
        m = re.match(r'\s+([\d.]+) us\s+(edet_\w+)\s+(.*?)\s{2,}', line)
        if m:
            d[(m.group(2), m.group(3).strip())].append(float(m.group(1)))
        m = re.match(r'\s+(edet_\w+)\s+calls=\s*(\d+)\s+([\d.]+) us', line)
        if m:
            e[m.group(1)] = float(m.group(3))
    return d, e


def avg(tabs):
    d, e = collections.defaultdict(float), collections.defaultdict(float)
    for dd, ee in tabs:
        for k, v in dd.items():
            d[k] += sum(v) / len(tabs)
        for k, v in ee.items():
            e[k] += v / len(tabs)
    return d, e


def main():
    root = sys.argv[1]
    old = avg([load(f) for f in sorted(glob.glob(os.path.join(root, "kb_*_old.txt")))])
    new = avg([load(f) for f in sorted(glob.glob(os.path.join(root, "kb_*_new.txt")))])
    print(f"total {sum(old[1].values()):.1f} -> {sum(new[1].values()):.1f} us")
    for k in sorted(new[1], key=lambda k: -new[1][k]):
        a, b = old[1].get(k, 0.0), new[1][k]
        print(f"  {k:26s} {a:8.1f} -> {b:8.1f}  {b - a:+7.1f}")
    rows = sorted((new[0].get(k, 0.0) - old[0].get(k, 0.0), k, old[0].get(k, 0.0), new[0].get(k, 0.0))
                  for k in set(old[0]) | set(new[0]))
    print("most improved launches:")
    for r in rows[:15]:
        print(f"  {r[0]:+7.1f} {r[2]:7.1f} {r[3]:7.1f} {r[1]}")
    print("most regressed launches:")
    for r in rows[-15:]:
        print(f"  {r[0]:+7.1f} {r[2]:7.1f} {r[3]:7.1f} {r[1]}")


if __name__ == "__main__":
    main()
