"""bench.py's rank launcher: `bench.py --gpus N` outside torch.distributed.run
starts N ranks itself; under a launcher WORLD_SIZE must equal --gpus."""
import argparse
import subprocess
import sys

import pytest

import bench


def _args(gpus):
    return argparse.Namespace(gpus=gpus)


def test_launch_cmd_shape():
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "20", "--warmup", "5"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    assert "--master-port=29555" in cmd
    assert cmd[-7].endswith("bench.py")
    assert cmd[-6:] == ["--gpus", "8", "--steps", "20", "--warmup", "5"]


def test_single_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.maybe_launch_ranks(_args(1), []) is None


def test_world_size_mismatch_exits(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit):
        bench.maybe_launch_ranks(_args(8), [])
    monkeypatch.setenv("WORLD_SIZE", "8")
    assert bench.maybe_launch_ranks(_args(8), []) is None


def test_multi_gpu_spawns_child_and_relays_status(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    class R:
        returncode = 3

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    rc = bench.maybe_launch_ranks(_args(4), ["--gpus", "4"])
    assert rc == 3
    assert "--nproc-per-node=4" in seen["cmd"]


def test_host_cpu_budget():
    h = bench.host_cpu_info()
    assert 1 <= h["baseline_threads"] <= h["physical_cores_allowed"] <= h["cpus_allowed"]
