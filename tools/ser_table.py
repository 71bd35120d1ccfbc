#!/usr/bin/env python3
"""Per-kernel average duration from tools/serprof.sh output (gpurun_out/ser)."""
import csv, os, sys
sys.path.insert(0, os.path.dirname(__file__))
from summarize_profile import short
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ser"
tot = 0.0
for r in csv.DictReader(open(os.path.join(root, "run_kernel_stats.csv"))):
    us = float(r["AverageNs"]) / 1e3
    if int(r["Calls"]) >= 20:
        tot += us
    print(f"{short(r['Name'])[:24]:24s} {r['Calls']:>5} {us:8.2f}")
print(f"sum of per-step kernels {tot:.1f} us")
