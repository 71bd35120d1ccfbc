#!/usr/bin/env python3
"""Short timed regions after bench.py's settle, three kinds in rotation: a timing event per step
(the round-5 StepClock), the device step clock (each step's first kernel stamps the device
clock; bench.py's StepClock now), and unmarked.  Which instrumentation costs step time, and
does the order (time since the settle) decide?  (r05final: the event-marked headline ran
0.2360 ms/step and the unmarked run right after it 0.2536.)  Settle 250 ms, then 9 regions of
`steps` steps, each bracketed by device syncs.

usage: python tools/region_order.py [fp32|bf16] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from impala_amd.engine import Engine  # noqa: E402
from impala_amd.model import AtariPPOModel  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else "fp32"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda:0")
m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype=dtype, seed=0)
e = Engine(m, batch_size=64, rollout_length=20)
m._train_engine = e
batch = bench.synthetic_batch(64, 20, 15, 1234, dev)


def step():
    e.train_step(*batch)


for _ in range(5):
    step()
torch.cuda.synchronize()
n = bench.settle(step, 250.0)
print(f"[{dtype}] settle {n} steps", flush=True)
for r in range(9):
    kind = ("events", "device", "none")[r % 3]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)] if kind == "events" else None
    clock = bench.StepClock(e, steps) if kind == "device" else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        if ev:
            ev[i].record()
        step()
    if ev:
        ev[steps].record()
    if clock:
        clock.close()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    extra = ""
    if ev:
        s = bench.step_time_stats([ev[i].elapsed_time(ev[i + 1]) for i in range(steps)])
        extra = f" median {s['ms_per_step_median']} first {s['step_ms'][0]}"
    elif clock:
        s = clock.summary()
        extra = f" median {s['ms_per_step_median']} first {s['step_ms'][0]} sum {s['steps_sum_ms']}"
    print(f"  region {r} {kind:7s} {ms:.4f} ms/step{extra}", flush=True)
