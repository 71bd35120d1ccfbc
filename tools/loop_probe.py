#!/usr/bin/env python3
"""Round 6: where the host thread's time goes in the drop-in loop over the host replay
(ImpalaLearner.train_step x 300, metrics never read): every Engine / replay call the learner
makes is wrapped with a host timer; medians per call and per step.
usage: python tools/loop_probe.py [host|device] [prefetch]"""
import collections
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from impala_amd.engine import Engine  # noqa: E402
from impala_amd.learner import ImpalaLearner  # noqa: E402
from impala_amd.model import AtariPPOModel  # noqa: E402
from impala_amd.replay import DeviceReplayBuffer, ReplayBuffer  # noqa: E402

T_ = collections.defaultdict(list)


def wrap(obj, name, label=None):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        T_[label or name].append(time.perf_counter() - t0)
        return r
    setattr(obj, name, g)


def bench_loop():
    """bench.py's learner_loop record alone, in a fresh process (no headline regions first)."""
    import argparse
    import json
    args = argparse.Namespace(batch=64, rollout=20, actions=15, loop_capacity=1000, loop_steps=100, loop_warmup=None,
                              warmup=5, dtype="fp32")
    out = bench.run_learner_loop(args, torch.device("cuda:0"), 0.22)
    for r in bench.LOOP_REPLAYS:
        print("bench-loop", r, json.dumps({k: (v["ms_per_step"], v["ms_per_step_median"])
                                           for k, v in out[r].items()}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "bench":
        return bench_loop()
    kind = sys.argv[1] if len(sys.argv) > 1 else "host"
    prefetch = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dev = torch.device("cuda:0")
    B, T, A, cap = 64, 20, 15, 1000
    rb = DeviceReplayBuffer(cap, T, A, device=dev, seed=5) if kind == "device" else ReplayBuffer(cap, seed=5)
    for t in bench.synthetic_trajectories(cap, T, A, 4242):
        rb.append(t)
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32", seed=0)
    ln = ImpalaLearner(m, rb, batch_size=B, rollout_length=T, learning_starts=cap, prefetch=prefetch)
    e = ln.engine
    for n in ("stage_wait", "stage_rows", "slot_batch", "train_step", "slot_release", "bind_metrics"):
        wrap(e, n)
    wrap(rb, "sample")
    wrap(ln, "train_step", "learner.train_step")
    for _ in range(30):
        ln.train_step()
    torch.cuda.synchronize()
    T_.clear()
    t0 = time.perf_counter()
    n = 300
    for _ in range(n):
        ln.train_step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / n
    print(f"{kind} prefetch {prefetch}: {wall:.3f} ms per train_step (wall)")
    for k, v in sorted(T_.items(), key=lambda kv: -sum(kv[1])):
        v = np.array(v) * 1e3
        print(f"  {k:22s} calls {len(v):4d}  median {np.median(v):.3f} ms  p90 {np.percentile(v, 90):.3f}"
              f"  per step {v.sum() / n:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
