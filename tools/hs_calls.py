#!/usr/bin/env python3
"""Where does the host-staged pass's one ~7-8 ms stall sit?  (r05a: exactly one slow step in
the driver's --steps 20 --warmup 5 runs, none in --steps 100 --warmup 10 runs.)  bench.py's
run_host_staged loop in a fresh process, warm-up W then S timed iterations, every library call
of every iteration timed on the host; iterations with a call over 1 ms are printed.

usage: python tools/hs_calls.py [warmup] [steps]   (copy path from IMPALA_H2D_* env)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from impala_amd.engine import Engine  # noqa: E402
from impala_amd.model import AtariPPOModel  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 5
S = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda:0")
m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=0)
e = Engine(m, batch_size=64, rollout_length=20)
m._train_engine = e
batch = bench.synthetic_batch(64, 20, 15, 1234, dev)
for _ in range(30):
    e.train_step(*batch)
torch.cuda.synchronize()
hosts = [[t.cpu().pin_memory() for t in batch] for _ in range(2)]
t_init = time.perf_counter()
e.stage_init(2)
t_init = time.perf_counter() - t_init
env = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("IMPALA_H2D"))
print(f"[{env or 'default'}] stage_init {t_init * 1e3:.2f} ms", flush=True)


def timed(rec, name, fn, *a):
    t = time.perf_counter()
    r = fn(*a)
    rec[name] = rec.get(name, 0.0) + (time.perf_counter() - t) * 1e3
    return r


def run(n, tag):
    recs = []
    t_run = time.perf_counter()
    rec = {}
    timed(rec, "stage0", e.stage, 0, *hosts[0])
    for k in range(n):
        s = k % 2
        if k + 1 < n:
            timed(rec, "stage_wait", e.stage_wait, 1 - s)
            timed(rec, "stage", e.stage, 1 - s, *hosts[1 - s])
        b = timed(rec, "slot_batch", e.slot_batch, s)
        timed(rec, "train_step", e.train_step, b)
        timed(rec, "slot_release", e.slot_release, s)
        recs.append(rec)
        rec = {}
    t = time.perf_counter()
    torch.cuda.synchronize()
    sync = (time.perf_counter() - t) * 1e3
    total = (time.perf_counter() - t_run) * 1e3
    print(f"{tag}: {n} iterations {total:.2f} ms ({total / n:.4f} ms/it), final sync {sync:.2f} ms",
          flush=True)
    for k, r in enumerate(recs):
        if max(r.values()) > 1.0:
            print(f"  it {k}: " + " ".join(f"{a}={b:.2f}" for a, b in r.items()), flush=True)


run(W, "warmup")
run(S, "timed")
run(S, "timed2")
