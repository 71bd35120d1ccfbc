#!/usr/bin/env python3
"""Round 6: the host-list staging of one C2 batch, timed piece by piece on the GPU box.
impala_stage_rows (synchronous: the host collate into the slot's page-locked block, then the
copies enqueued) and then impala_stage_wait (the copies done), per call, 40 calls after 5
warm-up; the replay is bench.py's 1000 synthetic trajectories.
usage: IMPALA_STAGE_THREADS=<n> python tools/collate_probe.py"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from impala_amd.engine import Engine  # noqa: E402
from impala_amd.model import AtariPPOModel  # noqa: E402
from impala_amd.replay import ReplayBuffer  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, T, A = 64, 20, 15
    rb = ReplayBuffer(1000, seed=1)
    for t in bench.synthetic_trajectories(1000, T, A, 4242):
        rb.append(t)
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
    e = Engine(m, batch_size=B, rollout_length=T)
    e.stage_init(3)
    col, cp = [], []
    for i in range(45):
        _, batch, _ = rb.sample(B)
        s = i % 3
        e.stage_wait(s)
        t0 = time.perf_counter()
        e.stage_rows(s, batch.row_ptrs)
        t1 = time.perf_counter()
        e.stage_wait(s)
        t2 = time.perf_counter()
        if i >= 5:
            col.append((t1 - t0) * 1e3)
            cp.append((t2 - t1) * 1e3)
    print(f"threads {os.environ.get('IMPALA_STAGE_THREADS', '8')}: stage_rows (collate + enqueue) "
          f"median {np.median(col):.3f} ms (min {min(col):.3f}); then copies {np.median(cp):.3f} ms "
          f"(min {min(cp):.3f}); 15.8 MB", flush=True)
    # pipelined: the staging thread collates batch k+1 while batch k's copies run (3 slots, a
    # slot restaged once its copies are done), no learner step in between
    batches = [rb.sample(B)[1] for _ in range(60)]
    torch.cuda.synchronize()
    for i, batch in enumerate(batches):
        s = i % 3
        if i == 10:
            t0 = time.perf_counter()
        e.stage_wait(s)
        e.stage_rows(s, batch.row_ptrs, background=True)
    for s in range(3):
        e.stage_wait(s)
    per = (time.perf_counter() - t0) * 1e3 / (len(batches) - 10)
    print(f"threads {os.environ.get('IMPALA_STAGE_THREADS', '8')}: pipelined staging (async, 3 slots) "
          f"{per:.3f} ms per batch", flush=True)


if __name__ == "__main__":
    main()
