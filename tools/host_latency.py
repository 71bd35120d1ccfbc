#!/usr/bin/env python3
"""Where the ~60 us between a timed region's wall time and the sum of its step events goes
(profiles/r05final: wall − Σ step events = 57–82 µs per 20-step region): the host's enqueue
time of one train_step call, of one torch event record, and torch.cuda.synchronize()'s own
latency on an idle device.  Medians over 200 samples each.

usage: python tools/host_latency.py [fp32|bf16]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from impala_amd.engine import Engine  # noqa: E402
from impala_amd.model import AtariPPOModel  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else "fp32"
dev = torch.device("cuda:0")
m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype=dtype, seed=0)
e = Engine(m, batch_size=64, rollout_length=20)
m._train_engine = e
batch = bench.synthetic_batch(64, 20, 15, 1234, dev)
for _ in range(20):
    e.train_step(*batch)
torch.cuda.synchronize()


def med_us(xs):
    return round(float(np.median(xs)) * 1e6, 2)


enq, first, sync_idle, rec, region_gap = [], [], [], [], []
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.train_step(*batch)  # host enqueue of one step, device idle at the call
    t1 = time.perf_counter()
    enq.append(t1 - t0)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    first.append(t2 - t0)  # one step, sync to sync
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    sync_idle.append(time.perf_counter() - t3)
    t4 = time.perf_counter()
    ev0.record()
    rec.append(time.perf_counter() - t4)
    # device time of one step between two events, against its sync-to-sync wall time
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    ev0.record()
    e.train_step(*batch)
    ev1.record()
    torch.cuda.synchronize()
    region_gap.append((time.perf_counter() - t5) - ev0.elapsed_time(ev1) * 1e-3)
print(f"[{dtype}] train_step host enqueue (device idle) {med_us(enq)} us; one step sync-to-sync "
      f"{med_us(first)} us; synchronize() on an idle device {med_us(sync_idle)} us; event "
      f"record {med_us(rec)} us; one-step wall minus its events {med_us(region_gap)} us", flush=True)
