#!/usr/bin/env python3
"""Host-staged pass (bench.py host_staged) from a rocprofv3 kernel trace: for the last steps,
the h2d_pull_kernel launches (the next batch's PCIe copy) against the learner kernels that ran
beside them -- start / end, how much of each pull overlaps compute, and the step period.
usage: tools/hs_timeline.py <dir with *kernel_trace.csv> [steps]"""
import csv, os, sys

root = sys.argv[1]
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
f = [os.path.join(d, x) for d, _, fs in os.walk(root) for x in fs if x.endswith("kernel_trace.csv")][0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40],
       r.get("Queue_Id", "?")) for r in rows]
pulls = [x for x in iv if "h2d_pull" in x[2]]
comp = [x for x in iv if "h2d_pull" not in x[2]]
if not pulls:
    sys.exit("no h2d_pull_kernel launches in the trace")
steps = [x for x in comp if "conv12_fwd" in x[2] or "Conv12Fwd" in x[2]]
print(f"{len(pulls)} pull launches; {len(steps)} forward launches")
for p in pulls[-nsteps:]:
    s, e = p[0], p[1]
    ov = [(max(s, c[0]), min(e, c[1]), c[2]) for c in comp if c[1] > s and c[0] < e]
    busy = sum(b - a for a, b, _ in ov)
    print(f"pull q{p[3]} {(e - s) / 1e3:8.2f} us, compute beside it {busy / 1e3:8.2f} us: " +
          ", ".join(f"{n}:{(b - a) / 1e3:.1f}" for a, b, n in ov[:12]))
fw = [x[0] for x in steps]
if len(fw) > 2:
    per = [(b - a) / 1e3 for a, b in zip(fw[-nsteps - 1:-1], fw[-nsteps:])]
    print("step periods (us):", " ".join(f"{x:.1f}" for x in per))
