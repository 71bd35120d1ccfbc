"""Data-parallel learner replicas: one process per GPU, RCCL over xGMI.

Trajectories are independent and every loss term is a mean over (B, T-1) or (B, T), so with
equal shards the mean of the replicas' gradients IS the full-batch gradient.  Each replica:
``impala_compute_grads_part`` 2 / 6, each followed by an async ``all_reduce(sum)`` of the
gradient bucket it finalised (FC + heads, then conv1 .. LayerNorm), so the larger bucket
travels while the backward continues -> ``impala_apply_update`` (x 1/world, global-norm clip on the reduced
gradient -- identical on every replica -- and Adam).  Weights therefore stay bit-identical
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


def init_process_group(backend: str = "nccl"):
    """Initialise the default group from the environment (MASTER_ADDR=127.0.0.1 on one node).
    ``nccl`` is RCCL on ROCm; ``gloo`` for CPU tests."""
    import torch.distributed as dist
    rank, local_rank, world = env_rank()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
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
                             buckets: int = 2) -> None:
    """Local gradients of `batch` summed over replicas, in buckets, each all-reduced as soon as
    the backward has finalised it so that it runs on the collective stream beside the rest of
    the backward.  Two buckets (default): FC + heads (1.07 MB, after part 2: heads step, FC
    weight and input gradients) overlaps part 6 (the fused per-frame LayerNorm / conv3 / conv2
    backward and the conv3 + conv2 weight gradients, ~60 us); conv1 .. LayerNorm (0.31 MB)
    follows it.  Three buckets (the unfused kernels): FC + heads after part 2, conv3 +
    LayerNorm after part 3, conv1 + conv2 after part 4.  The caller's stream waits for all of
    them before it continues (apply_update)."""
    import torch.distributed as dist
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


def params_checksum(flat: torch.Tensor) -> float:
    return float(flat.double().sum().item())
