#!/usr/bin/env python3
"""Bitwise A/B of two library builds: run 4 learner steps (fp32 and bf16, B=64 T=20, one
synthetic batch) with the library IMPALA_HIP_LIB names (default: the product) and save the
parameters, Adam moments and metrics after every step; with two saved files, compare them.
Steps 2..4 run on the kernel-layout weights Adam re-emitted, so equal results also mean equal
re-emitted weights.

usage: IMPALA_HIP_LIB=<lib> python tools/bitwise_ab.py save <out.npz>
       python tools/bitwise_ab.py cmp <a.npz> <b.npz>"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def save(out):
    import torch
    import bench
    from impala_amd.engine import Engine
    from impala_amd.model import AtariPPOModel
    dev = torch.device("cuda:0")
    res = {}
    for dt in ("fp32", "bf16"):
        m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype=dt, seed=0)
        e = Engine(m, batch_size=64, rollout_length=20)
        batch = bench.synthetic_batch(64, 20, 15, 1234, dev)
        for s in range(4):
            e.train_step(*batch)
            torch.cuda.synchronize()
            res[f"{dt}_params_{s}"] = m.flat.cpu().numpy().copy()
            res[f"{dt}_metrics_{s}"] = e.metrics.cpu().numpy().copy()
        e.close()
    np.savez(out, **res)
    print("saved", out, len(res), "arrays")


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        same = np.array_equal(A[k].view(np.uint32), B[k].view(np.uint32))
        if not same:
            bad += 1
            d = np.abs(A[k].astype(np.float64) - B[k].astype(np.float64))
            print(f"DIFF {k}: {int((d > 0).sum())} elements, max {d.max():.3g}")
    print("bitwise equal" if bad == 0 else f"{bad} arrays differ", f"({len(A.files)} compared)")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2])
    else:
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3]) else 0)
