#!/usr/bin/env python3
"""Round 6: the product library built with other LLVM scheduling options (whole-library A/B
against the default build; timing only, the arithmetic is unchanged).  Writes
build_variants/libimpala_hip_<name>.so and prints each build's scratch (spill) bytes for the
learner kernels.  usage: python tools/build_flag_variants.py"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from impala_amd import build  # noqa: E402

VARIANTS = {
    "maxilp": ["-mllvm", "--amdgpu-sched-strategy=max-ilp"],
    "memclause": ["-mllvm", "--amdgpu-sched-strategy=max-memory-clause"],
    "trackers": ["-mllvm", "--amdgpu-use-amdgpu-trackers"],
    "bias0": ["-mllvm", "--amdgpu-schedule-metric-bias=0"],
}


def main():
    out_dir = os.path.join(HERE, "build_variants")
    os.makedirs(out_dir, exist_ok=True)
    base = [f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-function"]
    for name, extra in VARIANTS.items():
        objs = []
        for src in build.hip_units():
            obj = os.path.join(out_dir, f"{os.path.basename(src)}.{name}.o")
            subprocess.run(["hipcc"] + base + extra + ["-c", "-o", obj, src], check=True)
            objs.append(obj)
        so = os.path.join(out_dir, f"libimpala_hip_{name}.so")
        subprocess.run(["hipcc", f"--offload-arch={build.ARCH}", "-shared", "-fPIC", "-o", so] + objs,
                       check=True)
        for o in objs:
            os.remove(o)
        asm = subprocess.run(["hipcc"] + base + extra + ["--cuda-device-only", "-S", "-o", "-",
                                                          os.path.join(build.SRC_DIR, "impala.hip")],
                             check=True, capture_output=True, text=True).stdout
        spills = re.findall(r"; ScratchSize: (\d+)", asm)
        print(name, so, "kernels with scratch:", sum(1 for s in spills if int(s) > 0), flush=True)


if __name__ == "__main__":
    main()
