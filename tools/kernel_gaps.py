#!/usr/bin/env python3
"""Per-kernel durations and the idle gap before each launch, from rocprofv3 kernel traces
(tools/r05_graph_trace.sh): the learner step's 8 launches, over the last `n` steps of the run.
The gap of a launch is its start minus the previous launch's end on the same queue.

usage: python tools/kernel_gaps.py gpurun_out/<tag> [n_steps]"""
import csv
import glob
import os
import statistics
import sys

STEP = ["conv12_fwd", "FcFwd", "head_step", "fc_bwd", "lnc3_conv12_bwd", "wgrad23", "reduce_grads",
        "adam_kernel"]


def short(name):
    for s in STEP:
        if s in name:
            return s
    if "gemm_tile" in name and "FcFwd" in name:
        return "FcFwd"
    return None


def analyse(path, n):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # the last n complete steps: walk back from the end to n conv12_fwd launches
    starts = [i for i, r in enumerate(rows) if short(r[2]) == "conv12_fwd"]
    first = starts[-n - 1] if len(starts) > n else starts[0]
    last = starts[-1]
    dur = {s: [] for s in STEP}
    gap = {s: [] for s in STEP}
    steps = []
    for i in range(first, last):
        k = short(rows[i][2])
        if k is None:
            continue
        dur[k].append((rows[i][1] - rows[i][0]) / 1e3)
        if i > 0:
            gap[k].append((rows[i][0] - rows[i - 1][1]) / 1e3)
    for a, b in zip(starts, starts[1:]):
        if a >= first and b <= last:
            steps.append((rows[b][0] - rows[a][0]) / 1e3)
    return dur, gap, steps


def main():
    root = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    for d in sorted(glob.glob(os.path.join(root, "*", "run_kernel_trace.csv"))):
        dur, gap, steps = analyse(d, n)
        tag = os.path.basename(os.path.dirname(d))
        print(f"{tag}: step (launch to launch) median {statistics.median(steps):.2f} us over "
              f"{len(steps)} steps")
        tot_d = tot_g = 0.0
        for k in STEP:
            if not dur[k]:
                continue
            md, mg = statistics.median(dur[k]), statistics.median(gap[k])
            tot_d += md
            tot_g += mg
            print(f"  {k:18s} dur {md:7.2f}  gap before {mg:6.2f}")
        print(f"  {'sum':18s} dur {tot_d:7.2f}  gaps {tot_g:6.2f}")


if __name__ == "__main__":
    main()
