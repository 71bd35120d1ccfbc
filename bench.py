#!/usr/bin/env python3
"""Learner throughput bench: env-frames/s of the IMPALA learner step on MI355X
(``--algo ppo`` / ``--algo sac``: the PPO / SAC learner steps of BASELINE configs 4 / 5).

``python bench.py --gpus N --steps K --warmup W``.  N > 1: one rank per GPU.  Under
torch.distributed.run (WORLD_SIZE set) it must equal --gpus; run directly with --gpus N > 1 it
starts ``python -m torch.distributed.run --nproc-per-node N`` itself as a child process (before
anything touches the GPU) and exits with the child's status.

Workload = BASELINE.json configs[1]: IMPALA procgen learner, B=64 trajectories x T=20 steps
per replica, 15 actions, obs (3,64,64) u8.  The headline (`value`, `dtype`) is the fp32 step --
the reference learner's own arithmetic (agents/impala/learning.py:140-177 in torch's default
fp32; MFMA f32-in/f32-accumulate, exact fp32 products); the bf16-operand mode (fp32 accumulation,
fp32 master weights) is reported beside it as the ``bf16_mode`` sub-record.  One step = the
full learner update (NatureCNN forward, log-softmax, V-trace, losses, backward, [RCCL gradient all-reduce], clip_grad_norm_(0.5), Adam) on a synthetic batch that
is resident in HBM before the timed region.  Multi-GPU: data-parallel
replicas, B=64 per GPU (weak scaling), one flat fp32 gradient bucket all-reduced over RCCL.

Also reported, all from the same run:
* ``roofline`` / ``roofline_top2``: the two kernels with algorithmic work that take longest
  (chosen from every kernel's average over --steps untimed steps, ``kernel_us``), each timed
  live by hipExtLaunchKernel start/stop events (the kernel's own begin / end stamps, the
  duration rocprofv3's kernel trace reports) over a second run of --steps steps right after
  the timed region: algorithmic FLOPs or bytes / that duration vs the dense MFMA or HBM peak,
  plus the PMC-measured HBM traffic per launch from the newest matching
  profiles/*/summary.json.  The stamped run is separate because an event pair on a launch
  costs the step ≈4.7 µs (tools/stamp_cost.py: 105 µs unstamped, 115 µs with two kernels
  stamped, 143 µs with all eight); its step time is reported as ``ms_per_step_stamped``;
* ``step_roofline``: SURVEY.md §8(d)'s step-level figure, frames/s x 17.74 MFLOP/frame vs
  the dense MFMA peak;
* ``bf16_mode`` (``--dtype bf16``: ``fp32_parity_mode``): the same workload in the other
  operand precision;
* ``host_staged``: the PCIe-inclusive rate (batches from page-locked host memory), never
  ``value``;
* ``cpu_baseline``: the reference CPU learner (the oracle's torch-CPU restatement of
  agents/impala/learning.py:140-177) on this host's cores, with a 1-thread leg and the host's
  CPU share stated.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# Algorithmic work of each learner-step kernel, per frame of the batch plus a
# per-launch constant (weights): (FLOPs/frame, HBM bytes/frame, HBM bytes/launch).  Bytes count
# each operand once (compulsory traffic) at the compute type's width `es` (2 for bf16, 4 for
# fp32); activations channels-last, fp32 where the kernel keeps fp32 (z, dy, LN stats).
def kernel_work(es):
    obs, a1, a2, a3 = 12288, 225 * 32 * es, 36 * 64 * es, 1024 * es
    m1 = 225 * 4  # conv1 ReLU bit mask
    return {
        "conv1_fwd": (2 * 225 * 32 * 192, obs + a1 + m1, 32 * 192 * es),
        "conv2_fwd": (2 * 36 * 64 * 512, a1 + a2, 64 * 512 * es),
        "conv1_fwd_conv2_fwd": (2 * 225 * 32 * 192 + 2 * 36 * 64 * 512, obs + a1 + m1 + a2,
                                (32 * 192 + 64 * 512) * es),
        "conv3_fwd": (2 * 16 * 64 * 576, a2 + 2 * a3 + 8, 64 * 576 * es + 2 * 1024 * 4),
        # the trunk forward and the FC forward in one launch (flag hand-off of y)
        "conv123_fwd_fc_fwd": (2 * 225 * 32 * 192 + 2 * 36 * 64 * 512 + 2 * 16 * 64 * 576 +
                               2 * 256 * 1024,
                               obs + a1 + m1 + a2 + 2 * a3 + 8 + a3 + 256 * 4 + 256 * es,
                               (32 * 192 + 64 * 512 + 64 * 576 + 256 * 1024) * es + 2 * 1024 * 4),
        # the fused trunk forward: conv1 + conv2 per frame, conv3 + LayerNorm as its tail
        "conv1_conv2_conv3_fwd": (2 * 225 * 32 * 192 + 2 * 36 * 64 * 512 + 2 * 16 * 64 * 576,
                                  obs + a1 + m1 + a2 + 2 * a3 + 8,
                                  (32 * 192 + 64 * 512 + 64 * 576) * es + 2 * 1024 * 4),
        "fc_fwd": (2 * 256 * 1024, a3 + 256 * 4 + 256 * es, 256 * 1024 * es),
        "head_step": (2 * 3 * 16 * 256, 256 * es + 256 * 4 + 8 + 4 + 4 + 15 * 4 + 256 * es,
                      2 * 16 * 256 * es),
        "fc_dgrad": (2 * 256 * 1024, 256 * es + 1024 * 4, 256 * 1024 * es),
        "ln_bwd": (10 * 1024, 1024 * 4 + 2 * a3 + 8, 2 * 1024 * 4),
        "conv3_dgrad": (2 * 16 * 64 * 576, a3 + 2 * a2, 64 * 576 * es),
        "ln_bwd_conv3_dgrad": (2 * 16 * 64 * 576 + 10 * 1024, 1024 * 4 + 2 * a3 + 8 + 2 * a2,
                               64 * 576 * es + 1024 * 4 * 2),
        "conv2_dgrad_conv1_wgrad": (2 * 36 * 64 * 512 + 2 * 225 * 32 * 192, obs + a2 + m1,
                                    64 * 512 * es),
        # the two per-frame backward chains in one launch (dact2 written once, re-read once)
        "ln_conv3_conv2_dgrad_conv1_wgrad": (2 * 16 * 64 * 576 + 10 * 1024 + 2 * 36 * 64 * 512 +
                                             2 * 225 * 32 * 192,
                                             1024 * 4 + 2 * a3 + 8 + 3 * a2 + obs + m1,
                                             (64 * 576 + 64 * 512) * es + 1024 * 4 * 2),
        "fc_wgrad": (2 * 256 * 1024, 256 * es + a3, 0),
        # FC weight + input gradient in one launch (dz read once for both)
        "fc_wgrad_fc_dgrad": (2 * 2 * 256 * 1024, 256 * es + a3 + 1024 * 4, 256 * 1024 * es),
        "conv3_wgrad": (2 * 16 * 64 * 576, a3 + a2, 0),
        "conv2_wgrad": (2 * 36 * 64 * 512, a2 + a1, 0),
        "conv3_wgrad_conv2_wgrad": (2 * 16 * 64 * 576 + 2 * 36 * 64 * 512, a3 + 2 * a2 + a1, 0),
        # per-parameter traffic: grads, m, v, params read + written, shadow weight written
        "adam": (0, 0, 344_496 * (8 * 4 + es)),
        "reduce_grads": (0, 0, 0),
        # fused reduction + Adam: params, m, v read; grads, m, v, params written; shadow written
        # (the gradient slabs are an implementation artefact, not algorithmic bytes)
        "reduce_grads_adam": (0, 0, 344_496 * (7 * 4 + es)),
    }


STEP_FLOPS_PER_FRAME = 17_743_872  # fwd 6,836,224 + bwd 10,907,648 (no conv1 dgrad)

# The MFMA instruction mix the fp32 step executes.  conv1's image operand is
# bytes (exact in bf16) and its other operand (W1 in the forward, dY1 in the weight gradient) is
# split exactly into three bf16 terms, so conv1 runs as three v_mfma_f32_16x16x32_bf16 passes
# (conv1.h c1_load_w1, conv12_bwd_body_f32 group B); everything else runs on
# v_mfma_f32_16x16x4_f32.  Per kernel: {mfma type: (FLOPs executed per frame)} -- conv1's
# algorithmic FLOPs x 3 at the bf16 rate.  bf16 mode: every contraction on bf16 MFMA, once.
CONV1_FLOPS = 2 * 225 * 32 * 192  # per frame, forward or weight gradient
CONV1_PASSES_FP32 = 3


def kernel_mix(k, work, dtype):
    """-> {"fp32": FLOPs/frame on f32 MFMA, "bf16": FLOPs/frame on bf16 MFMA} for kernel k."""
    f = work[k][0]
    if dtype == "bf16":
        return {"fp32": 0, "bf16": f}
    c1 = CONV1_FLOPS if k in ("conv1_fwd", "conv1_fwd_conv2_fwd", "conv1_conv2_conv3_fwd",
                              "conv123_fwd_fc_fwd", "conv2_dgrad_conv1_wgrad",
                              "ln_conv3_conv2_dgrad_conv1_wgrad") else 0
    return {"fp32": f - c1, "bf16": CONV1_PASSES_FP32 * c1}


def mix_floor_s(mix, frames):
    """Time the executed instruction mix takes at the dense peaks of its MFMA types."""
    return frames * (mix["fp32"] / (PEAK_TFLOPS["fp32"] * 1e12) +
                     mix["bf16"] / (PEAK_TFLOPS["bf16"] * 1e12))


def step_mix(dtype):
    """The whole step's executed mix per frame: conv1 forward + conv1 weight gradient."""
    if dtype == "bf16":
        return {"fp32": 0, "bf16": STEP_FLOPS_PER_FRAME}
    return {"fp32": STEP_FLOPS_PER_FRAME - 2 * CONV1_FLOPS,
            "bf16": CONV1_PASSES_FP32 * 2 * CONV1_FLOPS}
# PPO: same trunk, one loss head per transition (the heads' work is ~0.1 % of the total)
STEP_FLOPS_PER_FRAME_PPO = STEP_FLOPS_PER_FRAME
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}  # dense MFMA, MI355X_MICROARCH.md


def synthetic_batch(B, T, A, seed, device):
    """obs u8 uniform; a ~ U[0,A); r ~ N(0,1) clipped; g = 0.99*(u>0.05);
    mu ~ N(0,1).  Built on the host once, copied to HBM before timing."""
    return [torch.from_numpy(x).to(device) for x in _synthetic_np(B, T, A, seed)]


def synthetic_ppo_batch(N, A, seed, device):
    """PPO transitions: obs u8 uniform, a ~ U[0,A), v_target ~ N(0,1), pi_ref ~ 0.3 N(0,1)."""
    rng = np.random.default_rng(seed)
    obs = rng.integers(0, 256, size=(N, 3, 64, 64), dtype=np.uint8)
    act = rng.integers(0, A, size=(N,), dtype=np.int64)
    tgt = rng.standard_normal(N).astype(np.float32)
    mu = (0.3 * rng.standard_normal((N, A))).astype(np.float32)
    return [torch.from_numpy(x).to(device) for x in (obs, act, tgt, mu)]


def cpu_baseline_ppo(N, A, seconds, threads=None):
    """The reference PPO learner (oracle port of agents/ppo/learning.py:130-143)."""
    from oracle import ref_cpu
    if threads:
        torch.set_num_threads(threads)
    threads = torch.get_num_threads()
    batch = [torch.from_numpy(x) for x in ref_cpu.synthetic_ppo_batch(N, A, seed=4321)]
    model = ref_cpu.make_model(0, A)
    opt = ref_cpu.make_optimizer(model)
    for _ in range(2):
        ref_cpu.ppo_train_step(model, opt, batch)
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        ref_cpu.ppo_train_step(model, opt, batch)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"value": N / med, "unit": "env-frames/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} oracle PPO learner steps (N={N}, fp32 torch-CPU, "
                      f"{threads} threads) after 2 warm-up; median step {med * 1e3:.1f} ms"}


def cgroup_cpu_quota():
    """The CPU bandwidth quota of this process's cgroup in CPUs (cgroup v2 cpu.max, v1
    cfs_quota_us / cfs_period_us), or None when unlimited / unreadable."""
    try:
        rel = "/"
        for line in open("/proc/self/cgroup"):
            parts = line.strip().split(":", 2)
            if len(parts) == 3 and parts[0] == "0":
                rel = parts[2]
        for d in (os.path.join("/sys/fs/cgroup", rel.lstrip("/")), "/sys/fs/cgroup"):
            p = os.path.join(d, "cpu.max")
            if os.path.exists(p):
                q, per = open(p).read().split()[:2]
                return None if q == "max" else int(q) / int(per)
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except Exception:
        return None


def physical_cores(cpus):
    """Distinct (package, core) pairs among the logical CPUs `cpus`."""
    seen = set()
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            seen.add((open(base + "physical_package_id").read().strip(),
                      open(base + "core_id").read().strip()))
        except Exception:
            seen.add(("?", c))
    return len(seen)


def host_cpu_info():
    """CPU model, the CPUs this process may run on, their physical cores, the cgroup CPU quota,
    and the CPU budget the baseline uses: the quota when one is set (the box's share of a
    shared machine), else every physical core of the affinity set."""
    try:
        cpu = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":")[1].strip()
    except Exception:
        cpu = "unknown"
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except Exception:
        allowed = list(range(os.cpu_count() or 1))
    phys = physical_cores(allowed)
    quota = cgroup_cpu_quota()
    budget = max(1, int(quota)) if quota else phys
    budget = min(budget, phys)
    return {"cpu": cpu, "cpus_allowed": len(allowed), "physical_cores_allowed": phys,
            "cgroup_cpu_quota": quota, "cpus_machine": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "baseline_threads": budget,
            "budget_rule": "cgroup CPU quota if set, else all physical cores of the affinity set"}


def launch_cmd(nproc, argv):
    """The torch.distributed.run command `bench.py --gpus N` (N > 1, no WORLD_SIZE) runs as its
    child: one rank per GPU of this node; the launcher's c10d store binds a port itself on
    127.0.0.1 (--standalone), so no port is chosen before the socket that uses it exists."""
    return [sys.executable, "-m", "torch.distributed.run", "--standalone",
            "--local-addr=127.0.0.1", f"--nproc-per-node={nproc}",
            os.path.abspath(__file__)] + list(argv)


_JSON_FD = None


def claim_stdout():
    """From here on everything written to fd 1 -- RCCL's version banner at communicator init,
    anything a library prints -- goes to stderr; the original stdout is kept for the ONE JSON
    line (emit_line), which the driver parses."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def emit_line(line):
    """Write the result line to the stdout claim_stdout kept (or stdout)."""
    if _JSON_FD is None:
        print(line, flush=True)
    else:
        os.write(_JSON_FD, (line + "\n").encode())


def maybe_launch_ranks(args, argv):
    """--gpus N > 1 outside torch.distributed.run: start the N ranks as a child process (this
    process has not touched the GPU) and return its exit status; None = run in this process.
    Under a launcher WORLD_SIZE must equal --gpus (SystemExit otherwise)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
        return None
    if args.gpus <= 1:
        return None
    import subprocess
    cmd = launch_cmd(args.gpus, argv)
    print("bench.py: launching " + " ".join(cmd), file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def cpu_baseline(B, T, A, seconds, threads=None, warmup=2):
    """The reference CPU learner (oracle port of learning.py:140-177), timed on host cores."""
    from oracle import ref_cpu
    prev = torch.get_num_threads()
    if threads:
        torch.set_num_threads(threads)
    try:
        return _cpu_baseline(ref_cpu, B, T, A, seconds, warmup)
    finally:
        torch.set_num_threads(prev)


def _cpu_baseline(ref_cpu, B, T, A, seconds, warmup):
    threads = torch.get_num_threads()
    batch = [torch.from_numpy(x) for x in ref_cpu.synthetic_batch(B, T, A, seed=1234)]
    model = ref_cpu.make_model(0, A)
    opt = ref_cpu.make_optimizer(model)
    for _ in range(warmup):
        ref_cpu.train_step(model, opt, batch, collated=True)
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        ref_cpu.train_step(model, opt, batch, collated=True)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    cpu = host_cpu_info()["cpu"]
    return {"value": B * T / med, "unit": "env-frames/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} oracle learner steps (B={B},T={T},fp32 torch-CPU, "
                      f"{threads} threads, {cpu}) after {warmup} warm-up; median step "
                      f"{med * 1e3:.1f} ms"}


class StepClock:
    """Per-step device times of a timed region (SURVEY.md §8(d) defines the metric on the
    median step), from the library's device step clock (Engine.step_clock_*): the first kernel
    of every step stamps the device's 100 MHz clock as it starts, and one 1-thread kernel after
    the last step closes the region, so the steps tile the region's device time with no gaps
    and nothing is enqueued between them (a timing event per step cost the fp32 step ~1.4 %:
    tools/region_order.py, profiles/r05host).  Optionally the host's own per-iteration times
    (enqueue + any host wait inside the loop body)."""

    def __init__(self, eng, n, host=False):
        self.eng, self.n = eng, n
        self.host = [] if host else None
        self._t = None
        self.gc = []  # (generation, ms) of the Python collections inside the region (host=True)
        self._gc0 = None
        if host:
            gc.callbacks.append(self._on_gc)
        eng.step_clock_start(n)

    def _on_gc(self, phase, info):
        if phase == "start":
            self._gc0 = time.perf_counter()
        elif self._gc0 is not None:
            self.gc.append((info.get("generation", -1), (time.perf_counter() - self._gc0) * 1e3))
            self._gc0 = None

    def mark(self):
        """Before every step and after the last (host times only)."""
        if self.host is not None:
            t = time.perf_counter()
            if self._t is not None:
                self.host.append(t - self._t)
            self._t = t

    def close(self):
        """After the last step, inside the timed region: the closing stamp."""
        self.eng.step_clock_end()
        if self._on_gc in gc.callbacks:
            gc.callbacks.remove(self._on_gc)

    def summary(self, digits=4):
        """-> per-step statistics in ms (call after the region's final synchronize); the raw
        per-step times stay in ``self.ms``."""
        ms = self.ms = self.eng.step_clock_read()
        out = step_time_stats(ms, digits)
        out["step_clock"] = "device: the step's first kernel stamps s_memrealtime (100 MHz)"
        if self.host:
            h = np.array(self.host) * 1e3
            out["host_ms_per_iter_median"] = round(float(np.median(h)), digits)
            out["host_ms_per_iter_max"] = round(float(h.max()), digits)
            if len(h) <= 256:
                out["host_ms"] = [round(float(x), digits) for x in h]
            out["python_gc"] = {"collections": len(self.gc),
                                "by_generation": [sum(1 for g, _ in self.gc if g == k) for k in range(3)],
                                "ms": round(sum(t for _, t in self.gc), digits),
                                "max_ms": round(max((t for _, t in self.gc), default=0.0), digits)}
        return out


def step_time_stats(ms, digits=4):
    """Per-step statistics of a timed region's step times `ms` (milliseconds): median, min,
    max, p90, the indices of steps over twice the median, their sum, and (<= 256 steps) the
    steps themselves."""
    ms = np.asarray(ms, dtype=np.float64)
    med = float(np.median(ms))
    out = {"ms_per_step_median": round(med, digits),
           "ms_per_step_min": round(float(ms.min()), digits),
           "ms_per_step_max": round(float(ms.max()), digits),
           "ms_per_step_p90": round(float(np.percentile(ms, 90)), digits),
           "slow_steps": [int(i) for i in np.nonzero(ms > 2 * med)[0]],
           "steps_sum_ms": round(float(ms.sum()), digits)}
    if len(ms) <= 256:
        out["step_ms"] = [round(float(x), digits) for x in ms]
    return out


def step_stats(clock, dist, dev):
    """StepClock.summary(), with the per-step times taken as the element-wise max over ranks
    (the slowest rank sets every step) when data parallel, however many steps there are."""
    s = clock.summary()
    if dist is None:
        return s
    t = torch.tensor(clock.ms, device=dev, dtype=torch.float64)
    n = torch.tensor([t.numel(), -t.numel()], device=dev, dtype=torch.int64)
    dist.all_reduce(n, op=dist.ReduceOp.MAX)  # every rank sees the same max and min
    if int(n[0].item()) != -int(n[1].item()):
        raise RuntimeError("step clock: the ranks stamped different step counts")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s.update(step_time_stats(t.cpu().numpy()))
    s["over_ranks"] = "max per step"
    return s


def run_host_staged(eng, batch, args, dist, model, world):
    """The PCIe-inclusive rate (SURVEY.md §8(d) secondary bound; never `value`): every step's
    batch comes from page-locked host memory through the library's staging ring
    (impala_stage, 2 slots), the H2D copies of step k+1 overlapping the update on step k.
    The loop is ImpalaLearner._stage_host's: before a slot is restaged the host waits for the
    previous copy out of its host buffers (impala_stage_wait), which a producer refilling them
    has to do.  (Without that wait the host runs ahead of the GPU and the runtime stalls the
    SDMA copies for milliseconds every few dozen steps: 0.31-0.55 ms per step against a steady
    0.30 ms; tools/hs_loop.py, profiles/r04hs.)"""
    from impala_amd.distributed import compute_grads_allreduced, native_dp_buckets
    hosts = [[t.cpu().pin_memory() for t in batch] for _ in range(2)]
    eng.stage_init(2)

    def run(n, clock=None):
        eng.stage(0, *hosts[0])
        for k in range(n):
            s = k % 2
            if k + 1 < n:
                eng.stage_wait(1 - s)
                eng.stage(1 - s, *hosts[1 - s])
            b = eng.slot_batch(s)
            if clock is not None:
                clock.mark()
            if dist is None:
                eng.train_step(b)
            elif getattr(eng, "_dp", False):
                eng.dp_train_step(b, buckets=native_dp_buckets())
            else:
                compute_grads_allreduced(eng, (b,), model.flat_grad)
                eng.apply_update()
            eng.slot_release(s)
        if clock is not None:
            clock.mark()
            clock.close()

    run(max(args.warmup, 2))
    torch.cuda.synchronize()
    settled = settle(lambda: run(1), args.settle_ms, dist, model.flat.device)
    clock = StepClock(eng, args.steps, host=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, clock)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=model.flat.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    nbytes = sum(t.numel() * t.element_size() for t in hosts[0])
    st = step_stats(clock, dist, model.flat.device)
    return {"value": round(world * eng.frames * args.steps / elapsed, 1), "unit": "env-frames/s",
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "value_at_median": round(world * eng.frames / (st["ms_per_step_median"] * 1e-3), 1),
            **st, "settle": {"min_ms": args.settle_ms, "steps": settled},
            "h2d_bytes_per_step": nbytes,
            "h2d_GBps_per_gpu": round(nbytes * args.steps / elapsed / 1e9, 2),
            "note": "rollouts staged from page-locked host memory every step (impala_stage ring, "
                    "2 slots, obs over 2 SDMA streams, H2D overlapped with the previous update; "
                    "the learner's loop: a slot's previous copy is waited for before restaging "
                    "it); not `value`"}


def synthetic_trajectories(n, T, A, seed):
    """n trajectories in the reference's replay format ([s u8 (T,3,64,64), a i64 (T,1),
    r (T,1), g (T,1), mu (T,A)], agents/impala/learning.py:77-80) on the host, with the
    synthetic distributions of synthetic_batch."""
    obs, act, rew, disc, mu = (torch.from_numpy(x) for x in _synthetic_np(n, T, A, seed))
    return [[obs[i], act[i].view(T, 1), rew[i].view(T, 1), disc[i].view(T, 1), mu[i]]
            for i in range(n)]


def _synthetic_np(B, T, A, seed):
    rng = np.random.default_rng(seed)
    obs = rng.integers(0, 256, size=(B, T, 3, 64, 64), dtype=np.uint8)
    act = rng.integers(0, A, size=(B, T), dtype=np.int64)
    rew = np.clip(rng.standard_normal((B, T)), -10, 10).astype(np.float32)
    disc = (0.99 * (rng.random((B, T)) > 0.05)).astype(np.float32)
    mu = rng.standard_normal((B, T, A)).astype(np.float32)
    return obs, act, rew, disc, mu


LOOP_REPLAYS = ("device_replay", "host_list_replay")


def run_learner_loop(args, dev, headline_ms):
    """the loop the reference's caller runs, timed end to end --
    DistributedAgent.train (agents/distributed_agent.py:26-41: prepare, then train_step x K,
    float(v) of every metric) -> ImpalaLearner.train_step (learning.py:119-138: replay.sample(B),
    stage, _train_step, push every 4 steps, debug timings) -> a replay of 1000 trajectories
    (builder.py:30-36), for each replay the learner can be given:
    * device_replay     DeviceReplayBuffer: HBM ring, device-side gather of the sampled slots;
    * host_list_replay  ReplayBuffer: the reference's list of pageable CPU tensors, the rows
                        collated by the library's thread pool into a page-locked slot and
                        copied by SDMA (impala_stage_rows).
    Each with sync_every 1 (the reference: the metrics read every step) and 100; the learner
    prefetches two batches ahead (ImpalaLearner prefetch=2, the default).  Per-step device times
    from the step clock (each step's first learner kernel stamps it)."""
    from impala_amd.agent import DistributedAgent
    from impala_amd.learner import ImpalaLearner
    from impala_amd.model import AtariPPOModel
    from impala_amd.replay import DeviceReplayBuffer, ReplayBuffer
    B, T, A, cap = args.batch, args.rollout, args.actions, args.loop_capacity
    trajs = synthetic_trajectories(cap, T, A, 4242)
    makers = {"device_replay": lambda: DeviceReplayBuffer(cap, T, A, device=dev, seed=5),
              "host_list_replay": lambda: ReplayBuffer(cap, seed=5)}
    out = {"steps": args.loop_steps, "capacity": cap, "headline_ms_per_step": headline_ms,
           "note": "DistributedAgent.train -> ImpalaLearner.train_step -> replay.sample(B) on a "
                   "replay pre-filled with the capacity's synthetic trajectories; fp32 step; "
                   "wall ms per train_step (host sync on both sides of the loop), device step "
                   "clock per step"}
    for name in LOOP_REPLAYS:
        rb = makers[name]()
        for t in trajs:
            rb.append(t)
        torch.cuda.synchronize()
        m = AtariPPOModel((3, 64, 64), A, device=dev, dtype=args.dtype, seed=0)
        ln = ImpalaLearner(m, rb, batch_size=B, rollout_length=T, learning_starts=cap)
        rec = {}
        for sync in (1, 100):
            ag = DistributedAgent(None, ln, sync_every=sync)
            ag.train(args.loop_warmup if args.loop_warmup is not None else max(args.warmup, 5))
            torch.cuda.synchronize()
            clock = StepClock(ln.engine, args.loop_steps, host=True)
            step = ln.train_step

            def marked(step=step, clock=clock):
                clock.mark()
                return step()

            ln.train_step = marked
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ag.train(args.loop_steps)
            clock.mark()
            clock.close()
            torch.cuda.synchronize()
            elapsed = time.perf_counter() - t0
            ln.train_step = step
            st = clock.summary()
            st.pop("step_ms", None)
            st.pop("host_ms", None)
            ms = elapsed * 1e3 / args.loop_steps
            rec[f"sync_every_{sync}"] = {
                "ms_per_step": round(ms, 4), "value": round(B * T / (ms * 1e-3), 1),
                "ratio_to_headline": round(ms / headline_ms, 3), **st}
        out[name] = rec
        ln.engine.close()
        del ln, m, rb
        torch.cuda.synchronize()
    return out


def run_actor_act(args, dev, batch=128, calls=200):
    """actor-side batched inference, ``AtariPPOModel.act``
    (models/distributed_models.py:21-32: forward, argmax where deterministic, else a draw from
    softmax(logits); action, logits and value back on the host) on ``batch`` frames per call --
    the reference's inference batch (conf/config.yaml:28, <= 128) -- with the observations
    coming from host memory (the actors' page-locked buffers) and, for the kernel side alone,
    already in HBM.  Wall ms per call (host-synced by the .cpu() results), median of ``calls``."""
    from impala_amd.model import AtariPPOModel
    m = AtariPPOModel((3, 64, 64), args.actions, device=dev, dtype=args.dtype, seed=0)
    g = torch.Generator().manual_seed(77)
    obs_host = torch.randint(0, 256, (batch, 3, 64, 64), dtype=torch.uint8, generator=g).pin_memory()
    obs_dev = obs_host.to(dev)
    det = torch.zeros(batch, dtype=torch.bool)
    det[::4] = True  # a quarter of the actors in evaluation mode (per-frame argmax)
    out = {"batch": batch, "calls": calls, "dtype": args.dtype,
           "note": "wall ms per AtariPPOModel.act call (forward + argmax / softmax draw in one "
                   "HIP launch chain, impala_act), results copied to the host; median over calls"}
    for name, obs in (("host_obs", obs_host), ("device_obs", obs_dev)):
        for _ in range(20):
            m.act(obs, det)
        times = []
        for _ in range(calls):
            t0 = time.perf_counter()
            m.act(obs, det)
            times.append(time.perf_counter() - t0)
        med = float(np.median(times))
        out[name] = {"ms_per_call_median": round(med * 1e3, 4),
                     "ms_per_call_p90": round(float(np.percentile(times, 90)) * 1e3, 4),
                     "frames_per_s": round(batch / med, 1)}
    return out


PROFILE_NAMES = {"conv1_fwd": "Conv1Fwd", "conv1_fwd_conv2_fwd": "Conv12Fwd", "conv2_fwd": "Conv2Fwd", "conv3_fwd": "Conv3LnFwd",
                 "fc_fwd": "FcFwd", "heads_fwd": "HeadsFwd", "head_step": "head_step",
                 "fc_dgrad": "FcDgrad", "ln_bwd": "ln_bwd", "conv3_dgrad": "Conv3Dgrad",
                 "conv2_dgrad_conv1_wgrad": "Conv12Bwd", "ln_bwd_conv3_dgrad": "LnConv3Bwd", "fc_wgrad": "FcWgrad",
                 "conv3_wgrad": "Conv3Wgrad", "conv2_wgrad": "Conv2Wgrad",
                 "reduce_grads": "reduce_grads", "adam": "adam", "reduce_grads_adam": "reduce_adam",
                 "fc_wgrad_fc_dgrad": "FcBwd", "conv3_wgrad_conv2_wgrad": "Wgrad23",
                 "conv1_conv2_conv3_fwd": "Conv12Fwd", "ln_conv3_conv2_dgrad_conv1_wgrad": "LnConv12Bwd",
                 "conv123_fwd_fc_fwd": "FwdChain"}


SAC_PROFILE_NAMES = {"actor_chain": "actor_chain", "critic_loss_chain": "critic_loss_chain"}


def profiled_kernel(kernel, dtype, names=None, algo="impala"):
    """The newest committed rocprofv3 summary record of `kernel` for the same algorithm and
    dtype (profiles/<tag>/summary.json, "algo" defaulting to impala) that carries PMC HBM bytes
    -> (record, tag), or (None, None).  Newest = the latest "created" stamp
    (tools/summarize_profile.py); summaries without one are older, ordered by tag (r05r6 <
    r06a)."""
    root = os.path.join(HERE, "profiles")
    if not os.path.isdir(root):
        return None, None
    found = []
    for tag in sorted(os.listdir(root)):
        p = os.path.join(root, tag, "summary.json")
        if not os.path.exists(p):
            continue
        try:
            js = json.load(open(p))
        except Exception:
            continue
        if js.get("dtype", "bf16") != dtype or js.get("algo", "impala") != algo:
            continue
        for k in js.get("kernels", []):
            if k.get("kernel") == (names or PROFILE_NAMES).get(kernel) and k.get("hbm_bytes"):
                found.append((str(js.get("created", "")), tag, k))
    if not found:
        return None, None
    _, tag, k = max(found, key=lambda f: (f[0], f[1]))
    return k, tag


def profiled_traffic(kernel, dtype, names=None, algo="impala"):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), or None."""
    rec, tag = profiled_kernel(kernel, dtype, names, algo)
    return (float(rec["hbm_bytes"]), tag) if rec else (None, None)


# ----------------------------------------------------------------------------- SAC
def sac_phase_work(D, K, es, H=256):
    """Algorithmic work of each SAC learner-step launch (sac.hip kPhase): (FLOPs/transition,
    HBM bytes/transition, HBM bytes/launch), unpadded dims, each operand counted once."""
    DK = D + K
    act = H * es  # one hidden row
    w2 = H * H * es
    w = {
        "pack": (0, (2 * D + K) * 4 + (3 * D + 2 * DK) * es, 0),
        "fwd_l1": (2 * H * (2 * D + 2 * DK), (2 * D + DK) * es + 4 * act + 3 * act,
                   H * (2 * D + 2 * DK) * es),
        "fwd_l2": (4 * 2 * H * H, 4 * act + 4 * act + 3 * act, 4 * w2),
        "heads": (2 * 2 * H * 2 * K + 2 * 2 * H, 4 * act + 4 * K * 4 * 2, 0),
        "target_critic_l1": (2 * 2 * H * DK, DK * es + 2 * act, 2 * H * DK * es),
        "target_critic_l2": (2 * 2 * H * H, 4 * act, 2 * w2),
        "critic_loss": (4 * 2 * H, 4 * act + 4 * act, 0),
        "critic_bwd_l2": (2 * 2 * H * H + 2 * 2 * H * (H + 1) + 2 * 2 * (H + 1),
                          2 * 3 * act + 2 * 2 * act + 2 * (act + es), 2 * w2 + 2 * (H * H + 2 * H + 1) * 4),
        "critic_wgrad_l1": (2 * 2 * H * (DK + 1), 2 * act + (DK + 1) * es, 2 * H * (DK + 1) * 4),
        "actor_q_l1": (2 * 2 * H * DK, DK * es + 2 * act, 2 * H * DK * es),
        "actor_q_l2": (2 * 2 * H * H, 4 * act, 2 * w2),
        "actor_loss": (2 * 2 * H, 4 * act, 0),
        "actor_q_dgrad": (2 * 2 * H * H, 6 * act, 2 * w2),
        "actor_head_bwd": (2 * 2 * H * K + 2 * H * 2 * K, 3 * act + 2 * act + 2 * K * es, 0),
        "actor_bwd_l2": (2 * H * H + 2 * H * (H + 1) + 2 * 2 * K * (H + 1),
                         3 * act + 2 * act + 2 * K * es + act, w2 + (H * H + H + 2 * K * (H + 1)) * 4),
        "actor_wgrad_l1": (2 * H * (D + 1), act + (D + 1) * es, H * (D + 1) * 4),
        "alpha_fwd_l1": (2 * H * D, D * es + act, H * D * es),
        "alpha_fwd_l2": (2 * H * H, 2 * act, w2),
        "alpha_head": (2 * H * 2 * K, act + K * 4, 0),
        "critic_adam": (0, 0, 2 * (H * DK + H * H + 3 * H + 1) * (10 * 4 + 3 * es)),
        "actor_adam": (0, 0, (H * D + H * H + 2 * H + 2 * K * (H + 1)) * (10 * 4 + 3 * es)),
        "finalize": (0, 0, 0),
    }
    # fused path (sac_fused.h): per-row-block chains; a chain's intermediate rows stay in LDS,
    # so its bytes are the unfused phases' minus those hand-offs (approximated by their sum)
    dgrad2 = 2 * H * H
    w["critic_fwd_chain"] = sum_work(w, ("fwd_l1", "fwd_l2", "heads"))
    w["critic_loss_chain"] = sum_work(w, ("target_critic_l1", "target_critic_l2", "critic_loss"),
                                      (2 * dgrad2, 4 * act, 2 * w2))
    w["critic_wgrad"] = sum_work(w, ("critic_wgrad_l1",),
                                 (2 * 2 * H * (H + 1) + 2 * 2 * (H + 1), 4 * act + 2 * (act + es),
                                  2 * (H * H + 2 * H + 1) * 4))
    w["actor_chain"] = sum_work(w, ("actor_q_l1", "actor_q_l2", "actor_loss", "actor_q_dgrad",
                                    "actor_head_bwd"), (dgrad2, 2 * act, w2))
    w["actor_wgrad"] = sum_work(w, ("actor_wgrad_l1",),
                                (2 * H * (H + 1) + 2 * 2 * K * (H + 1), 3 * act + 2 * K * es,
                                 (H * H + H + 2 * K * (H + 1)) * 4))
    w["alpha_chain"] = sum_work(w, ("alpha_fwd_l1", "alpha_fwd_l2", "alpha_head"))
    return w


def sum_work(w, names, extra=(0, 0, 0)):
    return tuple(sum(w[n][i] for n in names) + extra[i] for i in range(3))


def cpu_baseline_sac(N, D, K, seconds):
    """The reference SAC learner step (oracle port of agents/sac/learning.py:146-265)."""
    from oracle import sac_cpu
    threads = torch.get_num_threads()
    actor, critic = sac_cpu.make_models(D, K, seed=0)
    st = sac_cpu.SACState(actor, critic)
    s, a, r, s1, d = (torch.from_numpy(x) for x in sac_cpu.synthetic_batch(N, D, K, seed=99))
    probs = torch.full((N,), 1.0 / 1000)
    g = torch.Generator().manual_seed(0)

    def one():
        eps3 = [torch.randn(N, K, generator=g) for _ in range(3)]
        sac_cpu.train_step(st, (s, a, r, s1, d), probs, eps3)

    for _ in range(2):
        one()
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"value": N / med, "unit": "transitions/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} oracle SAC learner steps (N={N}, D={D}, K={K}, fp32 "
                      f"torch-CPU, {threads} threads) after 2 warm-up; median step {med * 1e3:.2f} ms"}


def run_sac(args):
    """SAC learner step (BASELINE config 5): critic + actor + alpha updates and both Polyak
    averages on N sampled transitions, sampled on the device from an HBM replay each step."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist = None
    if world > 1:  # independent replicas (the reference's SAC learner does not shard)
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    from impala_amd.sac import DeviceTransitionReplay, SACEngine, SoftActor, SoftCritic
    N, D, K = args.batch, args.obs_dim, args.act_dim
    torch.manual_seed(0)
    critic = SoftCritic((D,), (K,), device=dev)
    actor = SoftActor((D,), (K,), device=dev, dtype=args.dtype)
    tactor = actor.clone_to(dev)
    eng = SACEngine(actor, critic, tactor, batch_size=N, dtype=args.dtype, seed=rank)
    actor._train_engine = eng
    critic._engine = eng
    # HBM replay of 1e6 transitions (conf/agent/sac.yaml replay_buffer_size), filled before timing
    cap = args.replay
    rb = DeviceTransitionReplay(cap, device=dev, seed=1000 + rank)
    g = torch.Generator(device=dev).manual_seed(7 + rank)
    rb.extend([torch.randn(cap, D, device=dev, generator=g),
               torch.rand(cap, K, device=dev, generator=g) * 2 - 1,
               torch.randn(cap, device=dev, generator=g),
               torch.randn(cap, D, device=dev, generator=g),
               torch.rand(cap, device=dev, generator=g) < 0.05])
    prio = torch.zeros(N, dtype=torch.float32, device=dev)

    def step():
        _, (s, a, r, s1, d), p = rb.sample(N, copy=False)
        eng.train_step(s, a, r, s1, d, probabilities=p, priorities=prio)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    work = sac_phase_work(D, K, 2 if args.dtype == "bf16" else 4)
    names = eng.phase_names()
    probe = {}
    rk = args.roofline_kernel
    if rk is None:
        for i, kname in enumerate(names):
            eng.timer_start(i, 3)
            for _ in range(3):
                step()
            ms, n = eng.timer_read()
            if n:
                probe[kname] = ms / n
        rk = max((k for k in probe if work[k][0]), key=probe.get)
    torch.cuda.synchronize()
    # timed region: the production mode (each step one hipGraph replay, sampling included)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the dominant launch's duration: HIP events around it on its stream, over as many steps
    # again (an armed timer launches directly -- a graph replay cannot carry per-launch events)
    eng.timer_start(names.index(rk), args.steps)
    for _ in range(args.steps):
        step()
    k_ms, k_n = eng.timer_read()
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    met = eng.metrics.cpu().numpy()
    if not np.all(np.isfinite(met)):
        raise RuntimeError(f"non-finite metrics {met}")
    value = world * N * args.steps / elapsed
    k_avg_ms = k_ms / max(k_n, 1)
    fpt, bpt, bpl = work[rk]
    flops, nbytes = fpt * N, bpt * N + bpl
    t_s = k_avg_ms * 1e-3
    if flops / (PEAK_TFLOPS[args.dtype] * 1e12) >= nbytes / (PEAK_HBM_GBS * 1e9):
        bound, unit, achieved, peak = "mfma", "TFLOP/s", flops / t_s / 1e12, PEAK_TFLOPS[args.dtype]
    else:
        bound, unit, achieved, peak = "hbm", "GB/s", nbytes / t_s / 1e9, PEAK_HBM_GBS
    traffic, tsrc = profiled_traffic(rk, args.dtype, SAC_PROFILE_NAMES, algo="sac")
    traffic_src = (f"profiles/{tsrc}/summary.json (rocprofv3 PMC FETCH_SIZE*2+WRITE_SIZE, "
                   "bytes per launch)") if tsrc else None
    # per-step algorithmic flops: the phases that ran (probe), else the fused step's phases
    ran = probe or ("critic_fwd_chain", "critic_loss_chain", "critic_wgrad", "actor_chain",
                    "actor_wgrad", "alpha_chain")
    step_flops = sum(work[k][0] for k in ran) * N
    out = {
        "metric": "SAC learner transitions/sec (agents/sac, BASELINE config 5)",
        "value": round(value, 1), "unit": "transitions/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": f"synthetic transitions (s, s1 ~ N(0,1), a ~ U(-1,1), r ~ N(0,1), 5% done) in a "
                f"{cap}-transition HBM replay, sampled on the device each step; reference init (seed 0)",
        "config": {"workload": f"SAC learner step (twin Q, tanh-Normal actor, alpha tuning, Polyak "
                               f"0.005), obs {D}, action {K}, N={N} transitions/GPU",
                   "global_batch": N * world, "parallelism": f"replicas{world}"},
        "roofline": {"bound": bound, "kernel": rk, "achieved": round(achieved, 3), "peak": peak,
                     "unit": unit, "frac": round(achieved / peak, 5), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "algorithmic": {"flops": flops, "bytes": nbytes},
                     "avg_launch_us": round(k_avg_ms * 1e3, 2), "launches": k_n,
                     "timing": "separate event-timed pass of --steps direct-launch steps"},
        "step_gflop": round(step_flops / 1e9, 3),
    }
    if probe:
        out["kernel_probe_us"] = {k: round(v * 1e3, 2) for k, v in sorted(probe.items(), key=lambda kv: -kv[1])}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_sac(N, D, K, args.cpu_seconds)
    if rank == 0:
        emit_line(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64, help="trajectories per GPU")
    ap.add_argument("--rollout", type=int, default=20)
    ap.add_argument("--actions", type=int, default=15)
    ap.add_argument("--dtype", default="fp32", choices=["bf16", "fp32"],
                    help="operand precision of the headline step (fp32 = the reference's)")
    ap.add_argument("--roofline-kernel", default=None)
    ap.add_argument("--settle-ms", type=float, default=250.0,
                    help="untimed steps for at least this much wall time (device synced) right "
                         "before each timed region, after the --warmup steps: the GPU clock "
                         "ramps over tens of ms of steady work (profiles/r05b), which a "
                         "20-step region would otherwise sample mid-ramp")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-seconds-1t", type=float, default=8.0,
                    help="sample length of the 1-thread CPU baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: host_cpu_info()['baseline_threads'])")
    ap.add_argument("--no-alt-line", "--no-fp32-line", dest="no_alt_line", action="store_true",
                    help="skip the other-precision sub-record (bf16_mode / fp32_parity_mode)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dp-variants", action="store_true",
                    help="N > 1: skip timing / cross-checking every all-reduce arrangement")
    ap.add_argument("--no-host-staged", action="store_true",
                    help="skip the PCIe-inclusive pass (host batches through impala_stage)")
    ap.add_argument("--no-step-clock", action="store_true",
                    help="time the headline region without the device step clock (per-step "
                         "times then unreported): the graph-replay A/B (IMPALA_GRAPH=1)")
    ap.add_argument("--no-learner-loop", action="store_true",
                    help="skip the drop-in loop sub-record (DistributedAgent -> ImpalaLearner "
                         "-> replay, N=1 IMPALA only)")
    ap.add_argument("--loop-steps", type=int, default=100,
                    help="train_steps per learner_loop record")
    ap.add_argument("--no-actor-act", action="store_true",
                    help="skip the actor inference sub-record (AtariPPOModel.act, N=1 IMPALA only)")
    ap.add_argument("--loop-warmup", type=int, default=None,
                    help="untimed train_steps before each learner_loop record (default: "
                         "max(--warmup, 5))")
    ap.add_argument("--loop-capacity", type=int, default=1000,
                    help="replay capacity of the learner_loop records (builder.py:30-36)")
    ap.add_argument("--algo", default="impala", choices=["impala", "ppo", "sac"],
                    help="ppo: PPO learner step (BASELINE config 4) on --batch transitions "
                         "(default 256, conf/agent/ppo.yaml); sac: SAC learner step (config 5, "
                         "--batch default 256 as conf/agent/sac.yaml, HalfCheetah dims 17/6)")
    ap.add_argument("--obs-dim", type=int, default=17)
    ap.add_argument("--act-dim", type=int, default=6)
    ap.add_argument("--replay", type=int, default=1_000_000)
    args = ap.parse_args()
    rc = maybe_launch_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    claim_stdout()  # (a rank process: RCCL prints its banner to stdout at the first collective)
    if args.algo == "sac":
        if args.batch == 64:
            args.batch = 256
        return run_sac(args)
    ppo = args.algo == "ppo"
    if ppo:
        if args.batch == 64:
            args.batch = 256
        args.rollout = 1

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist = None
    # IMPALA_BENCH_DIST=1: the data-parallel path (RCCL group, bucketed all-reduce, barriers,
    # max over ranks) also at world size 1, to rehearse the N-GPU code on one GPU
    if world > 1 or os.environ.get("IMPALA_BENCH_DIST") == "1":
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from impala_amd.distributed import (compute_grads_allreduced, native_dp_buckets,
                                        native_dp_enabled)
    from impala_amd.engine import Engine
    from impala_amd.model import AtariPPOModel

    B, T, A = args.batch, args.rollout, args.actions
    model = AtariPPOModel((3, 64, 64), A, device=dev, dtype=args.dtype, seed=0)
    eng = Engine(model, batch_size=B, rollout_length=T, world_size=world,
                 algo=args.algo)
    model._train_engine = eng
    if ppo:
        batch = synthetic_ppo_batch(B, A, 4321 + rank, dev)
    else:
        batch = synthetic_batch(B, T, A, 1234 + rank, dev)
    if dist is not None:  # identical initial weights on every replica
        dist.broadcast(model.flat, 0)
        model.params_changed()

    # data parallel: the learner's default (torch.distributed all-reduce) unless
    # IMPALA_DP_NATIVE=1 selects the library's own RCCL communicator (impala_dp_train_step);
    # every variant is timed and cross-checked in dp_variants below
    native_dp = dist is not None and native_dp_enabled()
    dp_buckets = native_dp_buckets() if native_dp else None

    def make_step(e, m):
        if native_dp:
            e.dp_init()

        def step():
            if dist is None:
                e.train_step(*batch)
            elif native_dp:
                e.dp_train_step(*batch, buckets=dp_buckets)
            else:
                compute_grads_allreduced(e, batch, m.flat_grad)
                e.apply_update()
        return step

    step = make_step(eng, model)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    work = kernel_work(2 if args.dtype == "bf16" else 4)
    kernel_us, top = select_kernels(eng, step, work, args)
    settled = settle(step, args.settle_ms, dist, dev)
    # --no-step-clock: the headline region without the device step clock, so that
    # IMPALA_GRAPH=1 runs it as graph replays (an armed clock makes steps launch directly)
    clock = None if args.no_step_clock else StepClock(eng, args.steps)
    elapsed, _ = timed_steps(eng, step, [], args, dist, dev, clock)  # the headline: no kernel stamps
    steps_stat = step_stats(clock, dist, dev) if clock is not None else {
        "ms_per_step_median": elapsed * 1e3 / args.steps, "step_clock": "off (--no-step-clock)"}
    # the stamped run for the roofline kernels' live durations, after its own settle: the
    # regions 5-10 ms after a settle ends run 5-7 % slow (tools/region_order.py, profiles/r05host)
    settle(step, args.settle_ms, dist, dev)
    elapsed_st, k_times = timed_steps(eng, step, top, args, dist, dev)
    met = eng.metrics.cpu().numpy()
    if not np.all(np.isfinite(met)):
        raise RuntimeError(f"non-finite metrics {met}")

    frames = world * B * T * args.steps
    value = frames / elapsed
    ms_step = elapsed * 1e3 / args.steps
    algo = args.algo
    rooflines = [kernel_roofline(k, k_times[k], work, B * T, args.dtype, algo) for k in top]
    metric = "learner env-frames/sec (IMPALA procgen T=20 B=64) at 1/2/4/8 MI355X"
    workload = f"IMPALA procgen learner step, NatureCNN actor-critic, B={B}/GPU T={T} A={A}, " \
               f"global B={B * world}"
    if ppo:
        metric = "PPO learner transitions/sec (procgen, NatureCNN, BASELINE config 4)"
        workload = f"PPO learner step (clip 0.1), NatureCNN actor-critic, N={B} transitions/GPU"
    step_flops_pf = STEP_FLOPS_PER_FRAME if not ppo else STEP_FLOPS_PER_FRAME_PPO
    out = {
        "metric": metric,
        "value": round(value, 1), "unit": "env-frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "algo": algo,
        "data": "synthetic rollouts resident in HBM (obs u8 uniform, BASELINE.md §3); "
                "random-init weights (reference layer_init_truncated, seed 0)",
        "config": {"workload": workload,
                   "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}",
                   "allreduce": (None if dist is None else
                                 f"native RCCL communicator, {dp_buckets} bucket(s)" if native_dp
                                 else "torch.distributed (c10d) RCCL")},
        "roofline": rooflines[0],
        "roofline_top2": rooflines,
        "step_roofline": step_roofline(value / world, step_flops_pf, args.dtype),
        "kernel_us": kernel_us,
        **steps_stat,
        "value_at_median": round(world * B * T / (steps_stat["ms_per_step_median"] * 1e-3), 1),
        "step_times": "device step clock (StepClock): each step's first kernel stamps the "
                      "device clock; no event or marker between the headline region's steps",
        "ms_per_step_stamped": round(elapsed_st * 1e3 / args.steps, 4),
        "settle": {"min_ms": args.settle_ms, "steps": settled},
    }
    if not args.no_alt_line:
        alt = "fp32" if args.dtype == "bf16" else "bf16"
        out["fp32_parity_mode" if alt == "fp32" else "bf16_mode"] = alt_line(
            alt, args, B, T, A, dev, dist, world, make_step, ppo)
    if native_dp:
        out["config"]["rccl_nranks"] = eng.dp_nranks
    if dist is not None and not args.no_dp_variants:
        # a sub-record: an error in it (raised on every rank alike, e.g. RCCL not loadable for
        # the native communicator) is recorded instead of losing the line
        try:
            out["dp_variants"] = dp_variants(args, B, T, A, dev, dist, world, batch)
        except Exception as ex:  # noqa: BLE001
            out["dp_variants"] = {"error": f"{type(ex).__name__}: {ex}"[:300]}
    # the drop-in loop before host_staged: its engines are closed afterwards.  A process's
    # streams share GPU_MAX_HW_QUEUES (4) hardware queues; when every handle had its own copy
    # streams, the loop's copies ran 0.42 instead of 0.30-0.32 ms per step beside the headline
    # engine's ring (profiles/r06w).  The copy streams are now one set per device (r06x)
    if world == 1 and dist is None and not ppo and not args.no_learner_loop:
        out["learner_loop"] = run_learner_loop(args, dev, round(ms_step, 4))
    if world == 1 and dist is None and not ppo and not args.no_actor_act:
        out["actor_act"] = run_actor_act(args, dev)
    if not args.no_host_staged:
        out["host_staged"] = run_host_staged(eng, batch, args, dist, model, world)
        if "learner_loop" in out and "host_list_replay" in out["learner_loop"]:
            # the host-list loop against the same process's host-staged step
            hs = out["host_staged"]["ms_per_step"]
            for rec in out["learner_loop"]["host_list_replay"].values():
                rec["ratio_to_host_staged"] = round(rec["ms_per_step"] / hs, 3)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if ppo:
            out["cpu_baseline"] = cpu_baseline_ppo(B, A, args.cpu_seconds,
                                                   args.cpu_threads or host_cpu_info()["baseline_threads"])
        else:
            host = host_cpu_info()
            cb = cpu_baseline(B, T, A, args.cpu_seconds, threads=args.cpu_threads or host["baseline_threads"])
            cb["host"] = host
            cb["single_thread"] = cpu_baseline(B, T, A, args.cpu_seconds_1t, threads=1, warmup=1)
            out["cpu_baseline"] = cb
    if rank == 0:
        emit_line(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


DP_VARIANTS = (("c10d_1bucket", False, 1), ("native_1bucket", True, 1),
               ("native_2bucket", True, 2))


def params_fingerprint(flat):
    """An exact fingerprint of a float32 buffer: its bit patterns summed with position
    weights in int64 (equal buffers give equal fingerprints; -0.0 and 0.0 differ)."""
    bits = flat.contiguous().view(torch.int32).to(torch.int64)
    w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
    return int((bits * w).sum().item())


def replicas_bitwise_equal(flat, dist):
    """True when every rank holds the same parameters (its fingerprint's max == min over
    ranks)."""
    fp = params_fingerprint(flat)
    t = torch.tensor([fp, -fp], dtype=torch.int64, device=flat.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(int(t[0].item()) == -int(t[1].item()))


def dp_variant_record(name, elapsed, steps, frames_per_step, world, nranks=None,
                      replicas_equal=None, equal_to_default=None):
    """One dp_variants entry (shape checked by tests/test_bench_launch.py)."""
    rec = {"ms_per_step": round(elapsed * 1e3 / steps, 4),
           "value": round(world * frames_per_step * steps / elapsed, 1),
           "replicas_bitwise_equal": replicas_equal}
    if nranks is not None:
        rec["rccl_nranks"] = nranks
    if equal_to_default is not None:
        rec["bitwise_equal_to_c10d_1bucket"] = equal_to_default
    return rec


def dp_variants(args, B, T, A, dev, dist, world, batch):
    """Multi-GPU only: every all-reduce arrangement of the data-parallel step, each from the
    same seed-0 weights on the same per-rank batch for warmup + steps steps: the timed steps'
    ms / value (max over ranks), the RCCL communicator's rank count (ncclCommCount) for the
    native ones, whether the replicas ended bit-identical (fingerprint max == min over ranks)
    and whether each native arrangement ended bit-identical to the c10d default."""
    from impala_amd.distributed import compute_grads_allreduced
    from impala_amd.engine import Engine
    from impala_amd.model import AtariPPOModel
    out, finals = {}, {}

    def all_ok(err):
        """Every rank learns whether any rank failed its local part (MIN of the ok flags), so
        that all ranks leave together instead of some entering a collective alone."""
        ok = torch.tensor([0 if err else 1], dtype=torch.int64, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        return bool(ok.item())

    for name, native, buckets in DP_VARIANTS:
        err = None
        try:
            m = AtariPPOModel((3, 64, 64), A, device=dev, dtype=args.dtype, seed=0)
            e = Engine(m, batch_size=B, rollout_length=T, world_size=world, algo=args.algo)
            m._train_engine = e
        except Exception as ex:  # noqa: BLE001 -- e.g. out of memory for the extra engine
            err = f"{type(ex).__name__}: {ex}"[:300]
        if not all_ok(err):
            out[name] = {"error": err or "failed on another rank"}
            break
        dist.broadcast(m.flat, 0)
        m.params_changed()
        if native:
            e.dp_init()

        def step(e=e, m=m, native=native, buckets=buckets):
            if native:
                e.dp_train_step(*batch, buckets=buckets)
            else:
                compute_grads_allreduced(e, batch, m.flat_grad, buckets=buckets)
                e.apply_update()

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        elapsed, _ = timed_steps(e, step, [], args, dist, dev)
        torch.cuda.synchronize()
        finals[name] = m.flat.clone()
        same = None
        if name != DP_VARIANTS[0][0]:
            same = torch.tensor([int(torch.equal(m.flat, finals[DP_VARIANTS[0][0]]))],
                                dtype=torch.int64, device=dev)
            dist.all_reduce(same, op=dist.ReduceOp.MIN)
            same = bool(same.item())
        out[name] = dp_variant_record(name, elapsed, args.steps, B * T, world,
                                      e.dp_nranks if native else None,
                                      replicas_bitwise_equal(m.flat, dist), same)
        e.close()
    return out


def select_kernels(eng, step, work, args):
    """Average duration of every kernel over --steps untimed steps (all kernel timers armed at
    once; each launch stamped by hipExtLaunchKernel events), and the two with algorithmic work
    that take longest -> (per-kernel us table, [dominant, second])."""
    names = [k for k in eng.kernel_names()]
    for k in names:
        eng.timer_start(k, args.steps)
    for _ in range(args.steps):
        step()
    avg = {}
    for k in names:
        ms, n = eng.timer_read(k)
        if n:
            avg[k] = ms / n
    table = {k: round(v * 1e3, 2) for k, v in sorted(avg.items(), key=lambda kv: -kv[1])}
    if args.roofline_kernel:
        top = [args.roofline_kernel]
    else:
        ranked = [k for k in sorted(avg, key=avg.get, reverse=True) if k in work and work[k][0]]
        top = ranked[:2]
    return table, top


def timed_steps(eng, step, kernels, args, dist, dev, clock=None):
    """The timed region: --steps steps between barriers + device syncs; the given kernels' own
    durations are stamped live (hipExtLaunchKernel events on their launch stream).  With a
    StepClock (armed before the region), its closing stamp is enqueued after the last step."""
    for k in kernels:
        eng.timer_start(k, args.steps)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if clock is None:
        for _ in range(args.steps):
            step()
    else:
        for _ in range(args.steps):
            clock.mark()
            step()
        clock.mark()
        clock.close()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    k_times = {k: eng.timer_read(k) for k in kernels}
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, k_times


def settle(step, min_ms, dist=None, dev=None, max_steps=20000):
    """Untimed steps until `min_ms` of wall time has passed (device synced): the GPU's clocks
    and the runtime's lazily created queues settle before a short timed region.  Data parallel:
    every rank runs the same number of steps (each step holds collectives), rank 0's clock
    deciding after every 10 (a broadcast of its flag).  Returns the number of steps run."""
    if min_ms <= 0:
        return 0
    n = 0
    t_end = time.perf_counter() + min_ms * 1e-3
    flag = torch.zeros(1, dtype=torch.int32, device=dev) if dist is not None else None
    while n < max_steps:
        for _ in range(10):
            step()
        n += 10
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        done = time.perf_counter() >= t_end
        if dist is not None:
            flag.fill_(int(done))
            dist.broadcast(flag, 0)
            done = bool(flag.item())
        if done:
            break
    return n


def kernel_roofline(k, timing, work, frames, dtype, algo):
    """Roofline of one kernel: the bound is whichever of MFMA time and HBM time of its
    algorithmic work is larger; `achieved` = that work / the kernel's average duration."""
    ms, n = timing
    k_avg_ms = ms / max(n, 1)
    fpf, bpf, bpl = work[k]
    flops, nbytes = fpf * frames, bpf * frames + bpl
    t_s = k_avg_ms * 1e-3
    if flops / (PEAK_TFLOPS[dtype] * 1e12) >= nbytes / (PEAK_HBM_GBS * 1e9):
        bound, unit, achieved, peak = "mfma", "TFLOP/s", flops / t_s / 1e12, PEAK_TFLOPS[dtype]
    else:
        bound, unit, achieved, peak = "hbm", "GB/s", nbytes / t_s / 1e9, PEAK_HBM_GBS
    rec, tsrc = profiled_kernel(k, dtype, algo=algo)
    traffic = float(rec["hbm_bytes"]) if rec else None
    mix = kernel_mix(k, work, dtype)
    floor = mix_floor_s(mix, frames)
    # the same fraction from the committed rocprofv3 kernel-trace average (a reader can
    # reproduce it from profiles/<tag>/summary.json; the profiler's runs clock each launch a
    # few % longer than the live stamps of an unprofiled run)
    prof = None
    if rec and rec.get("avg_us"):
        pt = float(rec["avg_us"]) * 1e-6
        ach = (flops / pt / 1e12) if bound == "mfma" else (nbytes / pt / 1e9)
        prof = {"avg_us": round(float(rec["avg_us"]), 2), "frac": round(ach / peak, 4),
                "source": f"profiles/{tsrc}/summary.json (rocprofv3 --kernel-trace --stats avg)"}
    return {"bound": bound, "kernel": k, "achieved": round(achieved, 2), "peak": peak,
            "unit": unit, "frac": round(achieved / peak, 4),
            # against the instruction mix the kernel executes (kernel_mix): the time its MFMAs
            # take at the dense peak of their own type / the measured duration
            "frac_mix": round(floor / t_s, 4),
            "mix": {"fp32_mfma_flops": mix["fp32"] * frames, "bf16_mfma_flops": mix["bf16"] * frames,
                    "floor_us": round(floor * 1e6, 2)},
            "traffic": traffic,
            "traffic_source": (f"profiles/{tsrc}/summary.json (rocprofv3 PMC FETCH_SIZE*2+"
                               "WRITE_SIZE, bytes per launch)") if tsrc else None,
            "algorithmic": {"flops": flops, "bytes": nbytes},
            "avg_launch_us": round(k_avg_ms * 1e3, 2), "launches": n,
            "rocprof": prof,
            "timing": "hipExtLaunchKernel start/stop events (kernel begin/end stamps) over the "
                      "timed steps"}


def step_roofline(frames_per_s_per_gpu, flops_per_frame, dtype):
    """the whole step against the dense MFMA peak (frames/s x algorithmic
    FLOPs per frame, per GPU)."""
    ach = frames_per_s_per_gpu * flops_per_frame / 1e12
    mix = step_mix(dtype)
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_TFLOPS[dtype],
            "unit": "TFLOP/s", "frac": round(ach / PEAK_TFLOPS[dtype], 4),
            "flops_per_frame": flops_per_frame,
            # the executed mix's floor per frame x frames/s (= floor / measured step time)
            "frac_mix": round(mix_floor_s(mix, 1) * frames_per_s_per_gpu, 4),
            "mix_per_frame": {"fp32_mfma_flops": mix["fp32"], "bf16_mfma_flops": mix["bf16"],
                              "floor_us_per_frame": round(mix_floor_s(mix, 1) * 1e6, 6)}}


def alt_line(dtype, args, B, T, A, dev, dist, world, make_step, ppo):
    """The same workload in the other operand precision, in the same run: value, step
    roofline and the dominant kernel's roofline (`bf16_mode` beside an fp32 headline)."""
    from impala_amd.engine import Engine
    from impala_amd.model import AtariPPOModel
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype=dtype, seed=0)
    e = Engine(m, batch_size=B, rollout_length=T, world_size=world, algo=args.algo)
    m._train_engine = e
    if dist is not None:
        dist.broadcast(m.flat, 0)
        m.params_changed()
    step = make_step(e, m)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    work = kernel_work(2 if dtype == "bf16" else 4)
    table, top = select_kernels(e, step, work, argparse.Namespace(steps=args.steps,
                                                                   roofline_kernel=None))
    settled = settle(step, args.settle_ms, dist, dev)
    clock = StepClock(e, args.steps)
    elapsed, _ = timed_steps(e, step, [], args, dist, dev, clock)
    st = step_stats(clock, dist, dev)
    settle(step, args.settle_ms, dist, dev)
    elapsed_st, k_times = timed_steps(e, step, top[:1], args, dist, dev)
    value = world * B * T * args.steps / elapsed
    out = {"dtype": dtype, "value": round(value, 1), "unit": "env-frames/s",
           "ms_per_step": round(elapsed * 1e3 / args.steps, 4), **st,
           "value_at_median": round(world * B * T / (st["ms_per_step_median"] * 1e-3), 1),
           "settle": {"min_ms": args.settle_ms, "steps": settled},
           "ms_per_step_stamped": round(elapsed_st * 1e3 / args.steps, 4),
           "step_roofline": step_roofline(value / world, STEP_FLOPS_PER_FRAME if not ppo
                                          else STEP_FLOPS_PER_FRAME_PPO, dtype),
           "roofline": kernel_roofline(top[0], k_times[top[0]], work, B * T, dtype, args.algo),
           "kernel_us": table}
    e.close()
    return out


if __name__ == "__main__":
    main()
