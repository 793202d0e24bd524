"""Where each kernel's time goes, from two rocprofv3 PMC passes (counters that
explain time, not bytes).

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \\
        SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --kernel-trace -d <A> ...
    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT \\
        SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d <B> ...
    python scripts/pmc_limiter.py --a <A> --b <B> --steps 6 --out profiles/pmc_limiter.json

Pass A is the wave-time breakdown: SQ_WAIT_ANY (waves parked on s_waitcnt or a barrier),
SQ_WAIT_INST_ANY (issue stalls) and SQ_ACTIVE_INST_ANY are disjoint parts of SQ_WAVE_CYCLES
(MI355X_MICROARCH.md, rocprofv3 PMC slots); ACTIVE_INST_VALU / LDS / VMEM say which pipe the
issuing cycles went to.  Pass B is the instruction mix, the LDS bank-conflict rate
(SQ_LDS_BANK_CONFLICT over SQ_LDS_IDX_ACTIVE, both LDS-array cycles) and the L2 hit rate.
Resident waves per SIMD = SQ_WAVE_CYCLES (quad-cycles, summed over waves) x 4 over the kernel's
cycles (GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs.  Each pass fits the per-pass slots (8 SQ,
4 TCC, 2 GRBM).  bench.py reads the JSON for the `limiter` field of its roofline_table rows
(`limiter_from`, below, is the rule).
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

PASS_A = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
          "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "GRBM_GUI_ACTIVE"]
PASS_B = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT",
          "SQ_LDS_IDX_ACTIVE", "SQ_BUSY_CYCLES", "TCC_HIT_sum", "TCC_MISS_sum", "GRBM_GUI_ACTIVE"]


def short(name):
    m = re.search(r"edet::(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:60]


def read_pass(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(set)
    for f in files:
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            ids[k].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    return acc, ids


def limiter_from(m, hbm_frac=None):
    """One line naming what bounds the kernel, with the counter value behind it."""
    if hbm_frac is not None and hbm_frac >= 0.6:
        return f"HBM bandwidth ({hbm_frac:.2f} of peak)"
    w, occ = m.get("wait_frac"), m.get("waves_per_simd")
    if w is None:
        return None
    if m.get("lds_conflict_rate", 0) >= 0.3 and m.get("active_lds_frac", 0) >= 0.15:
        return f"LDS bank conflicts ({m['lds_conflict_rate']:.2f} of LDS cycles, LDS issue {m['active_lds_frac']:.2f})"
    if m.get("active_valu_frac", 0) >= 0.45:
        return f"VALU issue (VALU active {m['active_valu_frac']:.2f} of wave time)"
    if m.get("issue_stall_frac", 0) >= 0.3:
        return f"instruction issue stalls ({m['issue_stall_frac']:.2f} of wave time)"
    if w >= 0.5:
        return (f"memory latency: waves parked on waitcnt / barrier {w:.2f} of wave time at "
                f"{occ:.1f} resident waves per SIMD")
    return f"mixed: wait {w:.2f}, VALU {m.get('active_valu_frac', 0):.2f}, LDS {m.get('active_lds_frac', 0):.2f}, {occ:.1f} waves/SIMD"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", required=True)
    ap.add_argument("--b", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--tag", default="")
    ap.add_argument("--workload", default="efficientdet-d0 train B=32 S=512 bf16")
    a = ap.parse_args()
    pa, ia = read_pass(a.a)
    pb, ib = read_pass(a.b)
    out = {"source": "rocprofv3 two PMC passes: " + " ".join(PASS_A) + " | " + " ".join(PASS_B),
           "tag": a.tag, "workload": a.workload, "steps": a.steps, "kernels": {}}
    for k, c in pa.items():
        n = len(ia[k])
        if not n or c["SQ_WAVE_CYCLES"] <= 0 or c["GRBM_GUI_ACTIVE"] <= 0:
            continue
        wc = c["SQ_WAVE_CYCLES"]
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        m = {"dispatches": n, "dispatches_per_step": n / a.steps,
             "waves_per_launch": c["SQ_WAVES"] / n,
             "waves_per_simd": wc * 4.0 / (cyc * 1024.0),
             "wait_frac": c["SQ_WAIT_ANY"] / wc, "issue_stall_frac": c["SQ_WAIT_INST_ANY"] / wc,
             "active_frac": c["SQ_ACTIVE_INST_ANY"] / wc, "active_valu_frac": c["SQ_ACTIVE_INST_VALU"] / wc,
             "active_lds_frac": c["SQ_ACTIVE_INST_LDS"] / wc, "active_vmem_frac": c["SQ_ACTIVE_INST_VMEM"] / wc}
        b = pb.get(k)
        if b is not None and len(ib[k]) == n:
            tot = b["SQ_INSTS_VALU"] + b["SQ_INSTS_LDS"] + b["SQ_INSTS_VMEM"] + b["SQ_INSTS_SALU"]
            m.update({"insts_per_wave": tot / max(m["waves_per_launch"] * n, 1.0),
                      "valu_insts_share": b["SQ_INSTS_VALU"] / max(tot, 1.0),
                      "lds_insts_share": b["SQ_INSTS_LDS"] / max(tot, 1.0),
                      "vmem_insts_share": b["SQ_INSTS_VMEM"] / max(tot, 1.0),
                      "lds_conflict_rate": b["SQ_LDS_BANK_CONFLICT"] / max(b["SQ_LDS_IDX_ACTIVE"], 1.0),
                      "l2_hit": b["TCC_HIT_sum"] / max(b["TCC_HIT_sum"] + b["TCC_MISS_sum"], 1.0)})
        m["limiter"] = limiter_from(m)
        out["kernels"][k] = m
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    rows = sorted(out["kernels"].items(), key=lambda kv: -kv[1]["dispatches"])
    print(f"{'kernel':24s} {'n':>5s} {'w/SIMD':>6s} {'wait':>5s} {'stall':>5s} {'valu':>5s} {'lds':>5s} "
          f"{'vmem':>5s} {'ldsconf':>7s} {'L2hit':>5s}  limiter")
    for k, m in rows:
        print(f"{k:24s} {m['dispatches']:5d} {m['waves_per_simd']:6.2f} {m['wait_frac']:5.2f} "
              f"{m['issue_stall_frac']:5.2f} {m['active_valu_frac']:5.2f} {m['active_lds_frac']:5.2f} "
              f"{m['active_vmem_frac']:5.2f} {m.get('lds_conflict_rate', float('nan')):7.3f} "
              f"{m.get('l2_hit', float('nan')):5.2f}  {m['limiter']}")


if __name__ == "__main__":
    main()
