"""bench.py's rank launcher: `bench.py --gpus N` outside torch.distributed.run
starts N ranks itself; under a launcher WORLD_SIZE must equal --gpus."""
import argparse
import os
import subprocess
import sys

import pytest

import bench

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _args(gpus):
    return argparse.Namespace(gpus=gpus)


def test_launch_cmd_shape():
    """The launcher binds its own rendezvous port (c10d store on port 0, 127.0.0.1): no port
    number is picked before the socket that uses it exists."""
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "20", "--warmup", "5"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--standalone" in cmd
    assert "--local-addr=127.0.0.1" in cmd
    assert not any(c.startswith("--master-port") for c in cmd)
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


def test_dp_variant_record_shape():
    """The N-GPU sub-record: every arrangement timed, the native ones with the
    communicator's rank count, each with the cross-rank and cross-variant bitwise checks."""
    assert [v[0] for v in bench.DP_VARIANTS] == ["c10d_1bucket", "native_1bucket",
                                                 "native_2bucket"]
    rec = bench.dp_variant_record("native_1bucket", 0.05, 200, 1280, 8, nranks=8,
                                  replicas_equal=True, equal_to_default=True)
    assert rec == {"ms_per_step": 0.25, "value": 8 * 1280 * 200 / 0.05,
                   "replicas_bitwise_equal": True, "rccl_nranks": 8,
                   "bitwise_equal_to_c10d_1bucket": True}
    base = bench.dp_variant_record("c10d_1bucket", 0.05, 200, 1280, 8, replicas_equal=True)
    assert "rccl_nranks" not in base and "bitwise_equal_to_c10d_1bucket" not in base


def test_frac_mix_of_the_executed_instruction_mix():
    """conv1's FLOPs count three times at the bf16 rate in the fp32 step, the
    rest at the fp32 rate; the step's floor is ~108 us at C2 (84.3 ns per frame)."""
    w = bench.kernel_work(4)
    mix = bench.kernel_mix("ln_conv3_conv2_dgrad_conv1_wgrad", w, "fp32")
    assert mix["bf16"] == 3 * bench.CONV1_FLOPS
    assert mix["fp32"] + bench.CONV1_FLOPS == w["ln_conv3_conv2_dgrad_conv1_wgrad"][0]
    assert abs(bench.mix_floor_s(mix, 1280) * 1e6 - 33.13) < 0.05
    assert bench.kernel_mix("fc_fwd", w, "fp32") == {"fp32": w["fc_fwd"][0], "bf16": 0}
    assert bench.kernel_mix("fc_fwd", bench.kernel_work(2), "bf16")["fp32"] == 0
    sr = bench.step_roofline(5.08e6, bench.STEP_FLOPS_PER_FRAME, "fp32")
    assert abs(sr["mix_per_frame"]["floor_us_per_frame"] * 1280 - 107.9) < 0.2
    assert abs(sr["frac_mix"] - 0.428) < 0.002


def _fingerprint_worker(rank, world, store, q):
    import os
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    x = torch.arange(1000, dtype=torch.float32) / 7
    same = bench.replicas_bitwise_equal(x, dist)
    if rank == 1:
        x[123] = torch.nextafter(x[123], torch.tensor(1e9))
    differ = bench.replicas_bitwise_equal(x, dist)
    q.put((rank, same, differ))
    dist.destroy_process_group()


def test_replicas_bitwise_equal_over_gloo(tmp_path):
    """The cross-rank check the N-GPU record carries, at world size 2 on the CPU: equal
    buffers agree, a one-ulp difference on one rank is caught."""
    import multiprocessing as mp
    store = str(tmp_path / "store")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_fingerprint_worker, args=(r, 2, store, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert res == [(0, True, False), (1, True, False)]


def _settle_worker(rank, world, store, q):
    import os
    import time

    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    calls = [0]

    def step():  # a collective per step, and rank-dependent step times
        calls[0] += 1
        t = torch.ones(1)
        dist.all_reduce(t)
        time.sleep(0.001 * (1 + 3 * rank))

    n = bench.settle(step, 60.0, dist, torch.device("cpu"))
    t = torch.tensor([float(n)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # would hang if the ranks' step counts differed
    q.put((rank, n, calls[0], int(t.item())))
    dist.destroy_process_group()


def test_settle_keeps_ranks_in_lockstep_over_gloo(tmp_path):
    """bench.settle (the untimed clock-settling steps before each timed region) runs the same
    number of steps on every rank when ranks run at different speeds: each step holds a
    collective, so a per-rank time check would leave one rank in an all-reduce alone."""
    import multiprocessing as mp
    store = str(tmp_path / "store")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_settle_worker, args=(r, 2, store, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    (r0, n0, c0, m0), (r1, n1, c1, m1) = res
    assert n0 == n1 == c0 == c1 == m0 == m1 and n0 >= 10 and n0 % 10 == 0


def test_step_time_stats_finds_the_stall():
    """The per-step statistics bench.py reports beside `value` (the median step):
    one 7.3 ms step among 0.3 ms steps -- the host-staged stall of the r04 driver record --
    is its max and its only slow step, and leaves the median alone."""
    ms = [0.30] * 20
    ms[2] = 7.3
    s = bench.step_time_stats(ms)
    assert s["ms_per_step_median"] == 0.3 and s["ms_per_step_max"] == 7.3
    assert s["slow_steps"] == [2] and len(s["step_ms"]) == 20
    assert abs(s["steps_sum_ms"] - (19 * 0.3 + 7.3)) < 1e-9
    assert "step_ms" not in bench.step_time_stats([1.0] * 300)


def test_stdout_carries_only_the_json_line():
    """bench.py claims fd 1 before any GPU / RCCL work: whatever is printed to stdout afterwards
    (RCCL's version banner at communicator init, library prints) goes to stderr, and stdout
    holds exactly the one JSON line the driver parses."""
    import subprocess
    code = ("import os, sys; sys.path.insert(0, %r); import bench; bench.claim_stdout(); "
            "os.write(1, b'RCCL version : x\\n'); print('noise', flush=True); "
            "bench.emit_line('{\"metric\": 1}')") % (HERE,)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout == '{"metric": 1}\n'
    assert "RCCL version" in r.stderr and "noise" in r.stderr
