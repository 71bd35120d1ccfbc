"""The staging ring's host side on the CPU (impala_amd/csrc/hostpool.h): the collate thread
pool, the streaming copy and the staging thread (impala_stage_rows / _async), compiled with
ROCm's clang++ and run; no GPU involved."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_hostpool_pool_copy_and_stager(tmp_path):
    cxx = shutil.which("clang++", path="/opt/rocm/lib/llvm/bin") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no clang++")
    exe = tmp_path / "hostpool_check"
    subprocess.run([cxx, "-O2", "-std=c++17", "-pthread", "-o", str(exe),
                    os.path.join(HERE, "hostpool_check.cpp")], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "hostpool ok" in r.stdout, r.stderr
