#!/usr/bin/env python3
"""One step's kernel sequence from a rocprofv3 kernel trace: duration and the idle gap before
each launch (usage: step_timeline.py <run_kernel_trace.csv> [first-kernel substring])."""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2] if len(sys.argv) > 2 else "conv12_fwd"
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
prev = None
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{r['Kernel_Name'][:50]:50s} q{r['Queue_Id']} dur {(e - s) / 1e3:7.2f} "
          f"gap {(s - prev) / 1e3 if prev else 0:7.2f}")
    prev = e
print(f"step (start to next start): {(int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3:.1f} us")
