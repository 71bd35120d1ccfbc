#!/usr/bin/env python3
"""Diagnostic builds: compile copies of csrc/ with source edits (phase knock-outs) into
build_variants/<name>.so; run them on the GPU with IMPALA_HIP_LIB=build_variants/<name>.so.
usage: tools/variants.py <spec.py>   where spec.py defines VARIANTS = {name: [(file, old, new), ...]}
"""
import os, runpy, shutil, subprocess, sys, tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build_variants")


def build(name, edits):
    tmp = tempfile.mkdtemp(prefix="var_")
    src = os.path.join(tmp, "impala_amd", "csrc")
    shutil.copytree(os.path.join(ROOT, "impala_amd", "csrc"), src)
    os.symlink(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    for f, old, new in edits:
        p = os.path.join(src, f)
        s = open(p).read()
        assert old in s, (name, f, old[:60])
        open(p, "w").write(s.replace(old, new))
    os.makedirs(OUT, exist_ok=True)
    out = os.path.join(OUT, name + ".so")
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "include"), "-o", out, os.path.join(src, "impala.hip"),
           os.path.join(src, "sac.hip")]
    subprocess.run(cmd, check=True)
    shutil.rmtree(tmp)
    return out


if __name__ == "__main__":
    spec = runpy.run_path(sys.argv[1])
    procs = []
    for name, edits in spec["VARIANTS"].items():
        print("built", build(name, edits), flush=True)
