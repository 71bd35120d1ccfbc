#!/usr/bin/env python3
"""Does a per-step stream marker change the fp32 step's kernel durations?  (r05a trace: with a
timing event recorded before every step, every kernel of the step ran 7-8 % shorter than in
back-to-back steps; profiles/r05a.)  Phases of --steps steps each, in a fixed order, the wall
time per step of each; run under rocprofv3 --kernel-trace for the per-kernel view.

usage: python tools/marker_ab.py [steps] [dtype]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from impala_amd.engine import Engine  # noqa: E402
from impala_amd.model import AtariPPOModel  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
dev = torch.device("cuda:0")
m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype=dtype, seed=0)
e = Engine(m, batch_size=64, rollout_length=20)
m._train_engine = e
batch = bench.synthetic_batch(64, 20, 15, 1234, dev)
ev_t = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
ev_n = [torch.cuda.Event(enable_timing=False) for _ in range(steps + 1)]
dummy = torch.zeros(1, device=dev)


def run(mode):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        if mode == "event_timing":
            ev_t[i].record()
        elif mode == "event_notiming":
            ev_n[i].record()
        elif mode == "event_timing_every4" and i % 4 == 0:
            ev_t[i].record()
        elif mode == "tiny_kernel":
            dummy.add_(1.0)
        elif mode == "host_gap":
            torch.cuda.synchronize()
        e.train_step(*batch)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


for _ in range(10):
    e.train_step(*batch)
modes = ["plain", "event_timing", "plain", "event_notiming", "plain", "event_timing_every4",
         "plain", "tiny_kernel", "plain", "host_gap", "event_timing", "plain"]
for md in modes:
    print(f"{md:22s} {run(md):.4f} ms/step", flush=True)
