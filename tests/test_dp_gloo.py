"""Data-parallel learner logic on CPU with gloo, world_size 2:
mean of shard gradients (all-reduce SUM / world) == full-batch gradient, and replicas stay
bit-identical after the clipped Adam update.  The HIP path does exactly this arithmetic
(impala_compute_grads -> all_reduce -> impala_apply_update with 1/world)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from impala_amd.distributed import allreduce_grads, init_process_group, shard_range, params_checksum
    from oracle import ref_cpu
    init_process_group("gloo")
    B, T, A = 4, 6, 15
    full = [torch.from_numpy(x) for x in ref_cpu.synthetic_batch(B, T, A, seed=77)]
    lo, hi = shard_range(B, world, rank)
    shard = [x[lo:hi] for x in full]
    m = ref_cpu.make_model(0, A)
    g_local = torch.from_numpy(ref_cpu.local_grads(m, shard))
    allreduce_grads(g_local)
    g_mean = g_local / world
    # apply the DP update on this replica: clip on the reduced gradient, then Adam
    off = 0
    for p in m.parameters():
        n = p.numel()
        p.grad = g_mean[off:off + n].view_as(p).clone()
        off += n
    torch.nn.utils.clip_grad_norm_(m.parameters(), 0.5)
    opt = ref_cpu.make_optimizer(m)
    opt.step()
    np.save(os.path.join(out_dir, f"g{rank}.npy"), g_mean.numpy())
    np.save(os.path.join(out_dir, f"p{rank}.npy"), ref_cpu.flat_params(m))
    ck = torch.tensor([params_checksum(torch.from_numpy(ref_cpu.flat_params(m)))], dtype=torch.float64)
    cks = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(cks, ck)
    assert all(float(c) == float(cks[0]) for c in cks)
    dist.barrier()
    dist.destroy_process_group()


def test_dp_shard_gradients_equal_full_batch(tmp_path):
    from oracle import ref_cpu
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    full = [torch.from_numpy(x) for x in ref_cpu.synthetic_batch(4, 6, 15, seed=77)]
    m = ref_cpu.make_model(0, 15)
    g_full = ref_cpu.local_grads(m, full)
    g0, g1 = np.load(tmp_path / "g0.npy"), np.load(tmp_path / "g1.npy")
    np.testing.assert_array_equal(g0, g1)
    rel = np.linalg.norm(g0 - g_full) / np.linalg.norm(g_full)
    assert rel < 1e-5, rel
    np.testing.assert_array_equal(np.load(tmp_path / "p0.npy"), np.load(tmp_path / "p1.npy"))
