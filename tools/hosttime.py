#!/usr/bin/env python3
"""Host-side enqueue cost of one learner step vs its device time (is the step launch-bound?)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import synthetic_batch
from impala_amd.engine import Engine
from impala_amd.model import AtariPPOModel

dev = torch.device("cuda", 0)
B, T, A = 64, 20, 15
model = AtariPPOModel((3, 64, 64), A, device=dev, dtype="bf16", seed=0)
eng = Engine(model, batch_size=B, rollout_length=T)
batch = synthetic_batch(B, T, A, 1234, dev)
for _ in range(20):
    eng.train_step(*batch)
torch.cuda.synchronize()
n = 300
t0 = time.perf_counter()
for _ in range(n):
    eng.train_step(*batch)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue {1e6 * (t1 - t0) / n:.1f} us/step, total {1e6 * (t2 - t0) / n:.1f} us/step")
