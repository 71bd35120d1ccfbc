#!/usr/bin/env python3
"""Step time with and without the live kernel stamps armed (hipExtLaunchKernel start / stop
events), K steps between device syncs, as bench.py's timed region."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import synthetic_batch
from impala_amd.engine import Engine
from impala_amd.model import AtariPPOModel

dev = torch.device("cuda", 0)
B, T, A, K = 64, 20, 15, int(os.environ.get("K", "100"))
model = AtariPPOModel((3, 64, 64), A, device=dev, dtype="bf16", seed=0)
eng = Engine(model, batch_size=B, rollout_length=T)
batch = synthetic_batch(B, T, A, 1234, dev)
for _ in range(20):
    eng.train_step(*batch)
torch.cuda.synchronize()
names = eng.kernel_names()
top2 = ["ln_conv3_conv2_dgrad_conv1_wgrad", "conv1_conv2_conv3_fwd"]


def run(armed):
    for k in armed:
        eng.timer_start(k, K)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        eng.train_step(*batch)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for k in armed:
        eng.timer_read(k)
    return 1e6 * dt / K


for rep in range(3):
    print(f"K={K} none {run([]):.1f} us  top2 {run(top2):.1f} us  all {run(names):.1f} us", flush=True)
