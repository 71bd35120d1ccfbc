#!/usr/bin/env python3
"""Round 6: the device-replay drop-in loop with the metrics read every step (sync_every 1, the
reference's float(v) per step): where the host's time goes between a step's metrics read and
the next step's launch, the window in which the device has nothing queued.
usage: python tools/sync1_probe.py [steps]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from impala_amd import _lib, agent as agent_mod  # noqa: E402
from impala_amd.agent import DistributedAgent  # noqa: E402
from impala_amd.learner import ImpalaLearner  # noqa: E402
from impala_amd.model import AtariPPOModel  # noqa: E402
from impala_amd.replay import DeviceReplayBuffer  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda:0")
    B, T, A, cap = 64, 20, 15, 1000
    rb = DeviceReplayBuffer(cap, T, A, device=dev, seed=5)
    for t in bench.synthetic_trajectories(cap, T, A, 4242):
        rb.append(t)
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
    ln = ImpalaLearner(m, rb, batch_size=B, rollout_length=T, learning_starts=cap)
    ag = DistributedAgent(None, ln, sync_every=1)
    ag.train(20)
    torch.cuda.synchronize()
    marks = {"read_end": [], "launch": [], "read_start": []}
    L = _lib.lib()
    f_step, f_rows = L.impala_train_step, L.impala_train_step_rows
    marks["returned"] = []

    def step_wrap(*a):
        marks["launch"].append(time.perf_counter())
        r = f_step(*a)
        marks["returned"].append(time.perf_counter())
        return r

    def rows_wrap(*a):
        marks["launch"].append(time.perf_counter())
        r = f_rows(*a)
        marks["returned"].append(time.perf_counter())
        return r
    L.impala_train_step = step_wrap
    L.impala_train_step_rows = rows_wrap
    rv = agent_mod._read_values

    def read_wrap(p):
        marks["read_start"].append(time.perf_counter())
        r = rv(p)
        marks["read_end"].append(time.perf_counter())
        return r
    agent_mod._read_values = read_wrap
    t0 = time.perf_counter()
    ag.train(steps)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    L.impala_train_step = f_step
    L.impala_train_step_rows = f_rows
    agent_mod._read_values = rv
    ret = np.array(marks["returned"])
    re, la, rs = (np.array(marks[k]) for k in ("read_end", "launch", "read_start"))
    n = min(len(re), len(la)) - 1
    gap = (la[1:n + 1] - re[:n]) * 1e6          # metrics read done -> next step's train call
    enq = (rs[:n] - la[:n]) * 1e6               # train call -> this step's metrics read starts
    wait = (re[:n] - rs[:n]) * 1e6              # the read itself (device wait + D2H)
    call = (ret[:n] - la[:n]) * 1e6             # the library call (the step's launches)
    print(f"sync_every 1, {steps} steps: {wall * 1e3:.4f} ms per step (wall), "
          f"IMPALA_REPLAY_ROWS={os.environ.get('IMPALA_REPLAY_ROWS', '1')}")
    for name, x in (("read -> next train call", gap), ("library call", call),
                    ("train call -> read start", enq),
                    ("read (wait + copy)", wait)):
        print(f"  {name:26s} median {np.median(x):7.1f} us  p90 {np.percentile(x, 90):7.1f}")


if __name__ == "__main__":
    main()
