#!/usr/bin/env python3
"""Host-staged loop shapes over the impala_stage ring (2 slots, fp32 C2 step, 200 steps each):
  free     bench.py's loop: stage(k+1) -> step(k) -> release, no host wait
  learner  ImpalaLearner's: stage_wait(slot of k+1) before restaging it (its host buffers are
           refilled), then stage(k+1) -> step(k) -> release
  lock     stage(k+1) -> step(k) -> release -> stage_wait(k+1)
usage: python tools/hs_loop.py [steps]   (copy path from IMPALA_H2D_* as in impala_stage_init)"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from impala_amd.engine import Engine
from impala_amd.model import AtariPPOModel
import bench

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda:0")
m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=0)
e = Engine(m, batch_size=64, rollout_length=20)
m._train_engine = e
batch = bench.synthetic_batch(64, 20, 15, 1234, dev)
hosts = [[t.cpu().pin_memory() for t in batch] for _ in range(2)]
nbytes = sum(t.numel() * t.element_size() for t in hosts[0])
e.stage_init(2)


def run(n, mode):
    e.stage(0, *hosts[0])
    for k in range(n):
        s = k % 2
        if k + 1 < n:
            if mode == "learner":
                e.stage_wait(1 - s)
            e.stage(1 - s, *hosts[1 - s])
        e.train_step(e.slot_batch(s))
        e.slot_release(s)
        if mode == "lock" and k + 1 < n:
            e.stage_wait(1 - s)


env = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("IMPALA_H2D"))
for mode in ("free", "learner", "lock", "free"):
    run(10, mode)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps, mode)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"loop {mode:8s} [{env or 'default'}]: {dt * 1e3:.4f} ms/step, "
          f"{64 * 20 / dt / 1e6:.3f} M frames/s, {nbytes / dt / 1e9:.1f} GB/s", flush=True)
