#!/usr/bin/env python3
"""The drop-in learner loop alone (bench.py learner_loop's device_replay record, sync_every 100)
for rocprofv3 kernel traces: what the loop adds to the learner step on the device.

usage: python tools/loop_trace.py [steps] [device|host]   (under rocprofv3 --kernel-trace)
       python tools/loop_trace.py --analyse <rocprofv3 output dir> [last_n_steps]
The host replay's H2D copies are listed too when the run was also traced with
--memory-copy-trace."""
import csv
import glob
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def run(steps, kind="device"):
    import torch
    import bench
    from impala_amd.agent import DistributedAgent
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    from impala_amd.replay import DeviceReplayBuffer, ReplayBuffer
    dev = torch.device("cuda:0")
    B, T, A, cap = 64, 20, 15, 1000
    rb = DeviceReplayBuffer(cap, T, A, device=dev, seed=5) if kind == "device" else \
        ReplayBuffer(cap, seed=5)
    for t in bench.synthetic_trajectories(cap, T, A, 4242):
        rb.append(t)
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
    ln = ImpalaLearner(m, rb, batch_size=B, rollout_length=T, learning_starts=cap)
    ag = DistributedAgent(None, ln, sync_every=100)
    ag.train(steps)
    torch.cuda.synchronize()
    print("loop done", steps, kind)


def analyse(d, last):
    path = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[-1]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "conv12_fwd" in r[2]]
    starts = starts[-(last + 1):]
    per = {}
    order = []
    for a, b in zip(starts, starts[1:]):
        for i in range(a, b):
            name = rows[i][2]
            gap = rows[i][0] - rows[i - 1][1]
            dur = rows[i][1] - rows[i][0]
            if name not in per:
                per[name] = ([], [])
                order.append(name)
            per[name][0].append(dur)
            per[name][1].append(gap)
    step = [rows[b][0] - rows[a][0] for a, b in zip(starts, starts[1:])]
    print(f"{len(step)} steps, median step {statistics.median(step) / 1e3:.1f} us")
    cps = sorted(glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True))
    if cps:
        t_lo, t_hi = rows[starts[0]][0], rows[starts[-1]][0]
        copies = []
        with open(cps[-1]) as f:
            for r in csv.DictReader(f):
                a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                if t_lo <= a <= t_hi:
                    copies.append((a, b, int(r.get("Bytes", 0) or 0)))
        copies.sort()
        big = [c for c in copies if c[2] > 1 << 20]
        if big:
            dur = [(b - a) / 1e3 for a, b, _ in big]
            gbs = [n / (b - a) for a, b, n in big]
            print(f"  {len(big)} H2D copies > 1 MB in the window: median {statistics.median(dur):.1f} us, "
                  f"{statistics.median(gbs):.1f} GB/s each")
            # per step: the forward's start minus the end of the last big copy before it
            waits = []
            for a in starts[1:]:
                t = rows[a][0]
                ends = [c[1] for c in big if c[1] <= t]
                if ends:
                    waits.append((t - max(ends)) / 1e3)
            if waits:
                print(f"  forward start - last copy end: median {statistics.median(waits):.1f} us")
    for n in order:
        d_, g_ = per[n]
        print(f"  {n:60s} n={len(d_):4d} dur {statistics.median(d_) / 1e3:7.2f} us  gap before "
              f"{statistics.median(g_) / 1e3:6.2f} us")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 100)
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 300,
            sys.argv[2] if len(sys.argv) > 2 else "device")
