"""Measure how far the HIP fp32 learner step is from the reference arithmetic at BASELINE sizes.

For C1 (B=8) and C2 (B=64), T=20, one synthetic batch: the HIP fp32 step (with the fused head's
own V-trace exported through impala_set_debug_vtrace), the fp32 oracle (torch CPU, op for op
as agents/impala/learning.py:140-177), the same oracle with torch's native CPU convolutions
(oneDNN off: at C2 oneDNN's fp32 convolution weight gradients are ~1.6e-3 rel-L2 from float64)
and the same oracle in float64.  Prints one JSON line per config with the achieved errors HIP-vs-fp32, HIP-vs-fp64 and fp32-vs-fp64, from which the
tolerances in tests/test_gpu_parity_full.py are set.  Test infrastructure: uses oracle/.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ref_cpu  # noqa: E402

NAMES = ("loss", "entropy", "td", "pg", "kl", "ratio", "grad_norm")


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-30)


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def max_rel(a, b, floor):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), floor)))


def probe(B, T=20, A=15, seed=1234, steps=3):
    from impala_amd.engine import Engine
    from impala_amd.model import AtariPPOModel
    dev = torch.device("cuda:0")
    batch = ref_cpu.synthetic_batch(B, T, A, seed=seed)
    flat0 = ref_cpu.flat_params(ref_cpu.make_model(0))
    # fp32 oracle, step 1 captured
    ref = ref_cpu.make_model(0)
    opt = ref_cpu.make_optimizer(ref)
    cap32 = {}
    tb = [torch.from_numpy(x) for x in batch]
    met32 = {k: float(v) for k, v in ref_cpu.train_step(ref, opt, tb, collated=True,
                                                         capture=cap32).items()}
    g32 = ref_cpu.flat_grads(ref)
    p32_1 = ref_cpu.flat_params(ref)
    for _ in range(steps - 1):
        ref_cpu.train_step(ref, opt, tb, collated=True)
    p32_3 = ref_cpu.flat_params(ref)
    # fp32 with torch's native CPU convolutions (oneDNN off)
    with torch.backends.mkldnn.flags(enabled=False):
        refn = ref_cpu.make_model(0)
        optn = ref_cpu.make_optimizer(refn)
        met_n = {k: float(v) for k, v in ref_cpu.train_step(refn, optn, tb, collated=True).items()}
        gn = ref_cpu.flat_grads(refn)
    # fp64
    cap64 = {}
    p64_1, g64, met64 = ref_cpu.train_step_fp64(flat0, batch, A, steps=1, capture=cap64)
    # HIP fp32
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32")
    m.load_flat(flat0)
    e = Engine(m, batch_size=B, rollout_length=T)
    m._train_engine = e
    dbg = e.debug_vtrace()
    db = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in batch]
    e.train_step(*db)
    torch.cuda.synchronize()
    mh = e.metrics.cpu().numpy()[:7].astype(np.float64)
    gh = m.flat_grad.cpu().numpy()
    ph_1 = m.flat.cpu().numpy()
    vt = {k: v.cpu().numpy().copy() for k, v in dbg.items()}
    for _ in range(steps - 1):
        e.train_step(*db)
    torch.cuda.synchronize()
    ph_3 = m.flat.cpu().numpy()
    out = {"B": B, "T": T, "metrics": {}, "vtrace": {}}
    for i, k in enumerate(NAMES):
        key = "train/" + k
        out["metrics"][k] = {"hip": float(mh[i]), "fp32": met32[key], "fp64": met64[key],
                             "hip_vs_fp32": rel(mh[i], met32[key]),
                             "hip_vs_fp64": rel(mh[i], met64[key]),
                             "fp32_vs_fp64": rel(met32[key], met64[key]),
                             "hip_vs_native": rel(mh[i], met_n[key]),
                             "native_vs_fp64": rel(met_n[key], met64[key])}
    for k in ("adv", "err", "q", "rho"):
        h, r32, r64 = vt[k], cap32[k].numpy(), cap64[k].numpy()
        scale = float(np.sqrt(np.mean(r64 ** 2)))
        out["vtrace"][k] = {
            "rms": scale,
            "hip_vs_fp32_maxabs": float(np.max(np.abs(h - r32))),
            "hip_vs_fp32_maxrel_floor1e-3": max_rel(h, r32, 1e-3 * scale),
            "hip_vs_fp32_rel_l2": rel_l2(h, r32),
            "hip_vs_fp64_rel_l2": rel_l2(h, r64),
            "fp32_vs_fp64_rel_l2": rel_l2(r32, r64),
            "fp32_vs_fp64_maxabs": float(np.max(np.abs(r32 - r64))),
        }
    out["grads"] = {"hip_vs_fp32_rel_l2": rel_l2(gh, g32), "hip_vs_fp64_rel_l2": rel_l2(gh, g64),
                    "fp32_vs_fp64_rel_l2": rel_l2(g32, g64), "hip_vs_native_rel_l2": rel_l2(gh, gn),
                    "native_vs_fp64_rel_l2": rel_l2(gn, g64)}
    out["params"] = {"step1_hip_vs_fp32_maxabs": float(np.max(np.abs(ph_1 - p32_1))),
                     "step1_hip_vs_fp64_maxabs": float(np.max(np.abs(ph_1 - p64_1))),
                     "step1_fp32_vs_fp64_maxabs": float(np.max(np.abs(p32_1 - p64_1))),
                     f"step{steps}_hip_vs_fp32_maxabs": float(np.max(np.abs(ph_3 - p32_3)))}
    return out


if __name__ == "__main__":
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    for B in [int(x) for x in (sys.argv[1:] or ["8", "64"])]:
        print(json.dumps(probe(B)), flush=True)
