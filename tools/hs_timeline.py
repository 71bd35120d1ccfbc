#!/usr/bin/env python3
"""Host-staged pass (bench.py host_staged) from a rocprofv3 kernel (+ memory-copy) trace: for the
last steps, the next batch's PCIe transfers -- h2d_pull_kernel launches and host-to-device
SDMA copies -- against the learner kernels that ran beside them: start / end, how much of each
transfer overlaps compute, and the step period.
usage: tools/hs_timeline.py <dir with *kernel_trace.csv [*memory_copy_trace.csv]> [steps]"""
import csv, os, sys

root = sys.argv[1]
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
f = [os.path.join(d, x) for d, _, fs in os.walk(root) for x in fs if x.endswith("kernel_trace.csv")][0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40],
       r.get("Queue_Id", "?")) for r in rows]
pulls = [x for x in iv if "h2d_pull" in x[2]]
comp = [x for x in iv if "h2d_pull" not in x[2]]
mc = [os.path.join(d, x) for d, _, fs in os.walk(root) for x in fs if x.endswith("memory_copy_trace.csv")]
if mc:
    for r in csv.DictReader(open(mc[0])):
        d = r.get("Direction", "")
        if "HOST_TO_DEVICE" in d.upper() or d == "":
            pulls.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", r.get("Stream_Id", "?")))
    pulls.sort()
    # one transfer per step: merge copies that overlap or follow within 5 us
    merged = []
    for p in pulls:
        if merged and p[0] <= merged[-1][1] + 5000:
            merged[-1] = (merged[-1][0], max(merged[-1][1], p[1]), merged[-1][2], merged[-1][3])
        else:
            merged.append(p)
    pulls = merged
if not pulls:
    sys.exit("no h2d_pull_kernel launches or host-to-device copies in the trace")
steps = [x for x in comp if "conv12_fwd" in x[2] or "Conv12Fwd" in x[2]]
print(f"{len(pulls)} transfers; {len(steps)} forward launches")
for p in pulls[-nsteps:]:
    s, e = p[0], p[1]
    ov = [(max(s, c[0]), min(e, c[1]), c[2]) for c in comp if c[1] > s and c[0] < e]
    busy = sum(b - a for a, b, _ in ov)
    print(f"xfer {p[2]} {(e - s) / 1e3:8.2f} us, compute beside it {busy / 1e3:8.2f} us: " +
          ", ".join(f"{n}:{(b - a) / 1e3:.1f}" for a, b, n in ov[:12]))
fw = [x[0] for x in steps]
if len(fw) > 2:
    per = [(b - a) / 1e3 for a, b in zip(fw[-nsteps - 1:-1], fw[-nsteps:])]
    print("step periods (us):", " ".join(f"{x:.1f}" for x in per))
