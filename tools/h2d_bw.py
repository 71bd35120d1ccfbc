#!/usr/bin/env python3
"""PCIe H2D rate of the staging ring alone (impala_stage of one B=64 T=20 rollout batch from
page-locked host memory into a device slot, repeated) and beside the learner step: prints
GB/s for the copy path selected by IMPALA_H2D_KERNEL (workgroups of h2d_pull_kernel; 0 =
hipMemcpyAsync / SDMA).  usage: IMPALA_H2D_KERNEL=8 python tools/h2d_bw.py [reps]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from impala_amd.engine import Engine
from impala_amd.model import AtariPPOModel
import bench

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
dev = torch.device("cuda:0")
m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=0)
e = Engine(m, batch_size=64, rollout_length=20)
m._train_engine = e
batch = bench.synthetic_batch(64, 20, 15, 1234, dev)
host = [t.cpu().pin_memory() for t in batch]
nbytes = sum(t.numel() * t.element_size() for t in host)
e.stage_init(2)
for _ in range(3):
    e.stage(0, *host)
    e.stage_wait(0)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(reps):
    e.stage(k % 2, *host)
    e.stage_wait(k % 2)
dt = time.perf_counter() - t0
alone = nbytes * reps / dt / 1e9
# beside the step: copies of slot 1 while the step runs on slot 0's batch (device-resident)
for _ in range(3):
    e.train_step(*batch)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(reps):
    e.stage(1, *host)
    e.train_step(*batch)
    e.stage_wait(1)
torch.cuda.synchronize()
dt2 = time.perf_counter() - t0
print(f"H2D path {os.environ.get('IMPALA_H2D_KERNEL', 'default(8)')}: alone {alone:.1f} GB/s "
      f"({nbytes / 1e6:.2f} MB per batch); beside the fp32 step {nbytes * reps / dt2 / 1e9:.1f} GB/s, "
      f"{dt2 * 1e3 / reps:.3f} ms per step+copy")
