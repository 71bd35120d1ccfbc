#!/usr/bin/env python3
"""Per-kernel wave-state table of one tools/pmc_wait.sh pass: per-launch means of the counters
(summed over the XCDs of a dispatch), and WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY /
WAIT_INST_LDS as % of SQ_WAVE_CYCLES (parked on a wait or barrier / issue-stalled / issuing /
stalled on LDS).

usage: python tools/pmc_table.py gpurun_out/<tag>/pmc"""
import csv
import os
import sys
from collections import defaultdict


def main():
    path = os.path.join(sys.argv[1], "run_counter_collection.csv")
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for r in csv.DictReader(open(path)):
        per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(float))
    n = defaultdict(int)
    for (k, _), c in per.items():
        n[k] += 1
        for name, v in c.items():
            agg[k][name] += v
    print(f"{'kernel':42s} {'waveCyc':>9s} {'wait%':>6s} {'stall%':>6s} {'issue%':>6s} "
          f"{'ldsSt%':>6s} {'VALU':>9s} {'LDS':>9s} {'MFMA':>9s}")
    for k in sorted(agg, key=lambda k: -agg[k]["SQ_WAVE_CYCLES"] / n[k]):
        c = {name: v / n[k] for name, v in agg[k].items()}
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        pct = lambda name: 100.0 * c.get(name, 0.0) / wc  # noqa: E731
        short = k.replace("void ", "")[:42]
        print(f"{short:42s} {wc:9.3g} {pct('SQ_WAIT_ANY'):6.1f} {pct('SQ_WAIT_INST_ANY'):6.1f} "
              f"{pct('SQ_ACTIVE_INST_ANY'):6.1f} {pct('SQ_WAIT_INST_LDS'):6.1f} "
              f"{c.get('SQ_INSTS_VALU', 0):9.3g} {c.get('SQ_INSTS_LDS', 0):9.3g} "
              f"{c.get('SQ_INSTS_MFMA', 0):9.3g}")


if __name__ == "__main__":
    main()
