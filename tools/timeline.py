#!/usr/bin/env python3
"""Print one learner step's kernel timeline (start offset, duration, stream) from a rocprofv3
kernel trace: tools/timeline.py gpurun_out/<dir> [step_index_from_end]."""
import csv, os, sys
sys.path.insert(0, os.path.dirname(__file__))
from summarize_profile import short
root = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
f = [x for x in os.listdir(root) if x.endswith("kernel_trace.csv")][0]
rows = sorted(csv.DictReader(open(os.path.join(root, f))), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == "Conv1Fwd"]
i0, i1 = starts[-k - 1], starts[-k]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{short(r['Kernel_Name'])[:22]:22s} q{r['Queue_Id']:>2} {s / 1e3:8.2f} -> {e / 1e3:8.2f}  ({(e - s) / 1e3:6.2f})")
print(f"step period {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.2f} us")
