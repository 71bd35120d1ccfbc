"""Data-parallel learner replicas: one process per GPU, RCCL over xGMI.

Trajectories are independent and every loss term is a mean over (B, T-1) or (B, T), so with
equal shards the mean of the replicas' gradients IS the full-batch gradient.

Default: the torch.distributed path below.  Opt-in on RCCL groups (IMPALA_DP_NATIVE=1,
``native_dp_enabled``): the library's own communicator (``Engine.dp_init``,
``impala_dp_train_step``) enqueues the whole step -- backward, in-place ncclAllReduce of the
gradient buckets on its side stream, update -- with no host round trip.  Each replica:
``impala_compute_grads`` (the whole backward) -> ``all_reduce(sum)`` of the flat fp32 gradient
(bucketed variants: ``compute_grads_allreduced``) -> ``impala_apply_update`` (x 1/world,
global-norm clip on the reduced gradient -- identical on every replica -- and Adam).  Weights therefore stay bit-identical
across replicas (checked by ``params_checksum``).
"""
from __future__ import annotations

import os
from typing import Tuple

import torch


def env_rank() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init_process_group(backend: str = "nccl", init_method: str | None = None):
    """Initialise the default group from the environment (MASTER_ADDR=127.0.0.1 on one node).
    ``nccl`` is RCCL on ROCm; ``gloo`` for CPU tests.  ``init_method`` (e.g. a ``file://``
    store) replaces the MASTER_ADDR / MASTER_PORT rendezvous."""
    import torch.distributed as dist
    rank, local_rank, world = env_rank()
    if init_method is None:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {} if init_method is None else {"init_method": init_method}
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local_rank), **kw)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return dist.group.WORLD


def shard_range(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous equal shard [start, stop) of the global trajectory batch for `rank`."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} not divisible by world size {world}")
    per = global_batch // world
    return rank * per, (rank + 1) * per


def allreduce_grads(flat_grad: torch.Tensor, group=None) -> None:
    """Sum the flat gradient bucket over replicas (the 1/world factor is applied in Adam)."""
    import torch.distributed as dist
    dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=group)


def compute_grads_allreduced(engine, batch, flat_grad: torch.Tensor, group=None,
                             buckets: int | None = None) -> None:
    """Local gradients of `batch` summed over replicas.  The caller's stream waits for the
    collectives before it continues (apply_update).

    One bucket (default): the whole backward, then one all-reduce of the flat fp32 gradient
    (1.38 MB).  Measured at world size 1 (RCCL group of one, host-time A/B recorded in
    `profiles/r02j/dp_hosttime.txt`): 114-130 us per step (bench: 0.1132 ms) against 105 us
    for the fused single-replica step, while every bucketed arrangement costs more than the
    overlap it can buy: each extra all-reduce adds a pair of cross-stream dependencies (~12 us of GPU idle
    each pair) and ~15-30 us of host time in c10d, which leaves the GPU waiting on the host.
    Two buckets (``buckets=2`` or IMPALA_DP_BUCKETS=2): FC + heads (1.07 MB) all-reduced after
    part 2 while part 6 (the fused per-frame backward and the conv weight gradients) runs,
    then conv1 .. LayerNorm (0.31 MB): 142 us at world size 1.  Three buckets (the unfused
    kernels): FC + heads after part 2, conv3 + LayerNorm after part 3, conv1 + conv2 after
    part 4."""
    import torch.distributed as dist
    if buckets is None:
        buckets = int(os.environ.get("IMPALA_DP_BUCKETS", "1"))
    if buckets not in (1, 2, 3):
        raise ValueError(f"gradient buckets must be 1, 2 or 3 (IMPALA_DP_BUCKETS), got {buckets}")
    if buckets == 1:
        engine.compute_grads(*batch)
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=group)
        return
    engine.compute_grads_part(2, *batch)
    off_fc, off = engine.bucket_offset_fc, engine.bucket_offset
    w_fc = dist.all_reduce(flat_grad[off_fc:], op=dist.ReduceOp.SUM, group=group, async_op=True)
    if buckets == 2:
        engine.compute_grads_part(6, *batch)
        w_rest = dist.all_reduce(flat_grad[:off_fc], op=dist.ReduceOp.SUM, group=group,
                                 async_op=True)
        w_fc.wait()
        w_rest.wait()
        return
    engine.compute_grads_part(3, *batch)
    w_c3 = dist.all_reduce(flat_grad[off:off_fc], op=dist.ReduceOp.SUM, group=group,
                           async_op=True)
    engine.compute_grads_part(4, *batch)
    w_c12 = dist.all_reduce(flat_grad[:off], op=dist.ReduceOp.SUM, group=group, async_op=True)
    w_fc.wait()
    w_c3.wait()
    w_c12.wait()


def native_dp_enabled(group=None) -> bool:
    """Opt-in (IMPALA_DP_NATIVE=1, RCCL groups only): the library's own RCCL communicator
    (``Engine.dp_init`` / ``dp_train_step``) drives the data-parallel step.  The default is the
    torch.distributed (c10d) all-reduce of ``compute_grads_allreduced``: the native path has
    run on one rank only (bitwise equal to ``train_step`` there), and stays opt-in until a
    multi-GPU run shows its replicas bit-identical to each other and to the c10d step
    (``bench.py --gpus N`` records both checks, ``dp_variants``)."""
    import torch.distributed as dist
    if os.environ.get("IMPALA_DP_NATIVE", "0") != "1":
        return False
    return dist.get_backend(group) == "nccl"


def native_dp_buckets() -> int:
    """Gradient buckets of the native step (IMPALA_DP_BUCKETS).  Default 1: the whole backward,
    then one in-place ncclAllReduce on the compute stream -- at world size 1 the step costs
    what the single-replica step does (fp32 0.3135 vs 0.3132 ms, bf16 0.1047 vs 0.1041 ms;
    the c10d all-reduce: 0.3233 / 0.1129 ms; profiles/r03e/dp_native.txt).  2: the FC + heads
    gradient (1.07 MB) all-reduced on the handle's side stream while the per-frame backward
    runs -- its three cross-stream event dependencies cost 36-40 us per step on this platform
    (0.3495 / 0.1446 ms at world size 1), more than the 8-GPU all-reduce it could hide."""
    b = int(os.environ.get("IMPALA_DP_BUCKETS", "1"))
    if b not in (1, 2):
        raise ValueError(f"native data-parallel buckets must be 1 or 2 (IMPALA_DP_BUCKETS), got {b}")
    return b


def params_checksum(flat: torch.Tensor) -> float:
    return float(flat.double().sum().item())
