#!/usr/bin/env python3
"""Host cost of the data-parallel step at world size 1 (RCCL group of one): enqueue time per
step and the host time of each piece (compute parts, c10d all_reduce calls, waits, update)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29547")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
import torch
import torch.distributed as dist
from bench import synthetic_batch
from impala_amd.distributed import compute_grads_allreduced
from impala_amd.engine import Engine
from impala_amd.model import AtariPPOModel

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
B, T, A = 64, 20, 15
model = AtariPPOModel((3, 64, 64), A, device=dev, dtype="bf16", seed=0)
eng = Engine(model, batch_size=B, rollout_length=T, world_size=1)
model._train_engine = eng
batch = synthetic_batch(B, T, A, 1234, dev)


def step():
    compute_grads_allreduced(eng, batch, model.flat_grad)
    eng.apply_update()


for _ in range(20):
    step()
torch.cuda.synchronize()
n = 200
t0 = time.perf_counter()
for _ in range(n):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"dp step: enqueue {1e6 * (t1 - t0) / n:.1f} us/step, total {1e6 * (t2 - t0) / n:.1f} us/step")
# pieces, host time only
g = model.flat_grad
acc = {"part2": 0.0, "part6": 0.0, "ar_fc": 0.0, "ar_rest": 0.0, "waits": 0.0, "update": 0.0}
for _ in range(n):
    a = time.perf_counter(); eng.compute_grads_part(2, *batch)
    b = time.perf_counter(); eng.compute_grads_part(6, *batch)
    c = time.perf_counter(); w1 = dist.all_reduce(g[eng.bucket_offset_fc:], async_op=True)
    d = time.perf_counter(); w2 = dist.all_reduce(g[:eng.bucket_offset_fc], async_op=True)
    e = time.perf_counter(); w1.wait(); w2.wait()
    f = time.perf_counter(); eng.apply_update()
    h = time.perf_counter()
    for k, v in zip(acc, (b - a, c - b, d - c, e - d, f - e, h - f)):
        acc[k] += v
    torch.cuda.synchronize()
print("host us per call: " + ", ".join(f"{k} {1e6 * v / n:.1f}" for k, v in acc.items()))
# variants of the bucketing / stream arrangement (total per step)
def old_two():
    eng.compute_grads_part(2, *batch)
    w1 = dist.all_reduce(g[eng.bucket_offset_fc:], async_op=True)
    eng.compute_grads_part(6, *batch)
    w2 = dist.all_reduce(g[:eng.bucket_offset_fc], async_op=True)
    w1.wait(); w2.wait()
    eng.apply_update()


def one_bucket():
    eng.compute_grads_part(2, *batch)
    eng.compute_grads_part(6, *batch)
    dist.all_reduce(g)
    eng.apply_update()


def no_collective():
    eng.compute_grads_part(2, *batch)
    eng.compute_grads_part(6, *batch)
    eng.apply_update()


side = torch.cuda.Stream(device=dev)
ev2, ev6 = torch.cuda.Event(), torch.cuda.Event()


def side_sync():
    main = torch.cuda.current_stream()
    eng.compute_grads_part(2, *batch)
    ev2.record(main)
    eng.compute_grads_part(6, *batch)
    ev6.record(main)
    with torch.cuda.stream(side):
        side.wait_event(ev2)
        dist.all_reduce(g[eng.bucket_offset_fc:])
        side.wait_event(ev6)
        dist.all_reduce(g[:eng.bucket_offset_fc])
    main.wait_stream(side)
    eng.apply_update()


def two_bucket():
    compute_grads_allreduced(eng, batch, model.flat_grad, buckets=2)
    eng.apply_update()


for name, fn in (("side stream, blocking-call collectives", side_sync), ("default (one bucket)", step),
                 ("compute_grads_allreduced buckets=2", two_bucket), ("two-bucket, all_reduce after each part", old_two),
                 ("one bucket at the end", one_bucket), ("parts + update, no collective", no_collective)):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{name}: enqueue {1e6 * (t1 - t0) / n:.1f}, total {1e6 * (time.perf_counter() - t0) / n:.1f} us/step")
# single-GPU step for comparison
for _ in range(20):
    eng.train_step(*batch)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    eng.train_step(*batch)
torch.cuda.synchronize()
print(f"train_step total {1e6 * (time.perf_counter() - t0) / n:.1f} us/step")
dist.destroy_process_group()
