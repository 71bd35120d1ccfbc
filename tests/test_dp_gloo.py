"""Data-parallel learner logic on CPU with gloo: mean of shard gradients
(all-reduce SUM / world) == full-batch gradient, and replicas stay bit-identical after the
clipped Adam update.  The HIP path does exactly this arithmetic (impala_compute_grads ->
all_reduce -> impala_apply_update with 1/world).

Two shapes: world 2 at B=4, T=6 in fp32, and C3's replica count -- world 8, B=8 per replica,
T=20 (global B=64) -- in float64, where the only difference between the mean of the 8 shard
gradients and the B=64 gradient is the summation order: bound 1e-12 rel-L2 (measured 4.8e-15)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _batch(B, T, A, seed, f64):
    from oracle import ref_cpu
    b = [torch.from_numpy(x) for x in ref_cpu.synthetic_batch(B, T, A, seed=seed)]
    if f64:
        b = [x.double() if x.is_floating_point() else x for x in b]
    return b


def _model(A, f64):
    from oracle import ref_cpu
    m = ref_cpu.make_model(0, A)
    return m.double() if f64 else m


def _worker(rank, world, out_dir, B=4, T=6, f64=False):
    # rendezvous through a file store in the test's own directory: no TCP port to pick
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    if f64:  # obs / 255. follows the default dtype
        torch.set_default_dtype(torch.float64)
    from impala_amd.distributed import allreduce_grads, init_process_group, shard_range, params_checksum
    from oracle import ref_cpu
    init_process_group("gloo", init_method=f"file://{os.path.join(out_dir, 'store')}")
    A = 15
    full = _batch(B, T, A, 77, f64)
    lo, hi = shard_range(B, world, rank)
    shard = [x[lo:hi] for x in full]
    m = _model(A, f64)
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


@pytest.mark.parametrize("world,B,T,f64,tol", [(2, 4, 6, False, 1e-5), (8, 64, 20, True, 1e-12)],
                         ids=["w2_B4_T6_fp32", "w8_B64_T20_fp64"])
def test_dp_shard_gradients_equal_full_batch(tmp_path, world, B, T, f64, tol):
    from oracle import ref_cpu
    mp.spawn(_worker, args=(world, str(tmp_path), B, T, f64), nprocs=world,
             join=True)
    prev, prev_dt = torch.get_num_threads(), torch.get_default_dtype()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if f64:
        torch.set_default_dtype(torch.float64)
    try:
        full = _batch(B, T, 15, 77, f64)
        m = _model(15, f64)
        g_full = ref_cpu.local_grads(m, full)
        # one learner on the whole batch: clip on the full-batch gradient, then Adam
        torch.nn.utils.clip_grad_norm_(m.parameters(), 0.5)
        ref_cpu.make_optimizer(m).step()
        p_full = ref_cpu.flat_params(m)
    finally:
        torch.set_num_threads(prev)
        torch.set_default_dtype(prev_dt)
    gs = [np.load(tmp_path / f"g{r}.npy") for r in range(world)]
    ps = [np.load(tmp_path / f"p{r}.npy") for r in range(world)]
    for r in range(1, world):  # replicas bit-identical after all-reduce, clip and Adam
        np.testing.assert_array_equal(gs[r], gs[0])
        np.testing.assert_array_equal(ps[r], ps[0])
    rel = np.linalg.norm(gs[0] - g_full) / np.linalg.norm(g_full)
    print(f"DP {world}x: shard-mean vs full-batch grad rel-L2 {rel:.3e}")
    assert rel < tol, rel
    # params after one Adam step: within a small fraction of the lr (1e-4) of the full-batch step
    dp = float(np.abs(ps[0] - p_full).max())
    assert dp < (1e-9 if f64 else 1e-6), dp
