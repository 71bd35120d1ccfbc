"""Build the HIP extension in-tree: ``python -m impala_amd.build``.

Compiles ``impala_amd/csrc/{impala,sac}.hip`` for gfx950 into ``impala_amd/libimpala_hip.so`` with
hipcc (cross-compiles without a GPU).  The .so is git-ignored and travels with the tree.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC_DIR = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libimpala_hip.so")
# A/B build: also compiles the measured-slower alternative kernels (csrc/common.h IMPALA_AB);
# loaded only when IMPALA_HIP_LIB points at it
OUT_AB = os.path.join(HERE, "libimpala_hip_ab.so")
ARCH = os.environ.get("IMPALA_OFFLOAD_ARCH", "gfx950")


def sources():
    return sorted(os.path.join(SRC_DIR, f) for f in os.listdir(SRC_DIR)
                  if f.endswith((".hip", ".h")))


def hip_units():
    """The translation units linked into the one library (impala.hip: IMPALA / PPO learner,
    sac.hip: SAC learner)."""
    return [os.path.join(SRC_DIR, f) for f in ("impala.hip", "sac.hip")]


def needs_build(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    inc = os.path.join(os.path.dirname(HERE), "include")
    deps = sources() + [os.path.join(inc, f) for f in os.listdir(inc)]
    return any(os.path.getmtime(s) > t for s in deps if os.path.exists(s))


def build(force: bool = False, verbose: bool = True, ab: bool = False) -> str:
    """Compile the product library (or, ab=True, the A/B library with the measured-slower
    alternative kernels) in-tree."""
    out = OUT_AB if ab else OUT
    if not force and not needs_build(out):
        return out
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    tmp = out + ".tmp"
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-Wno-unused-function"] + (["-DIMPALA_AB=1"] if ab else [])
    # the units compile in parallel (sac.hip dominates), then one link
    objs, procs = [], []
    for src in hip_units():
        obj = os.path.join(HERE, os.path.basename(src) + (".ab.o" if ab else ".o"))
        objs.append(obj)
        cmd = [hipcc] + flags + ["-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((cmd, subprocess.Popen(cmd)))
    failed = [cmd for cmd, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    if os.path.exists(tmp):
        os.remove(tmp)
    subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs,
                   check=True)
    os.replace(tmp, out)
    for obj in objs:
        os.remove(obj)
    return out


if __name__ == "__main__":
    print("built", build(force="--force" in sys.argv, ab="--ab" in sys.argv))
