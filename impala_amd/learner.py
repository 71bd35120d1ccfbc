"""ImpalaLearner — drop-in for ``agents/impala/learning.py:86-177`` on MI355X.

Same constructor signature, same ``prepare`` / ``train_step`` / ``connect`` behaviour, same
metric keys; ``_train_step`` is one HIP call (forward, V-trace, loss, backward, clip, Adam —
``impala_train_step``) or, for data-parallel replicas, ``impala_compute_grads`` + an RCCL
all-reduce of the flat gradient + ``impala_apply_update``.
"""
from __future__ import annotations

import collections
import os
import time
from dataclasses import dataclass
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch

from impala_amd import _lib
from impala_amd.core import Learner
from impala_amd.engine import Engine
from impala_amd.replay import RowSample


@dataclass
class ImpalaAdam:
    """Optimizer descriptor: torch.optim.Adam(lr, eps) of agents/impala/builder.py:43-44,
    executed by the fused HIP clip+Adam kernel over the model's flat parameter buffer."""
    lr: float = 1e-4
    eps: float = 1e-5
    betas: Tuple[float, float] = (0.9, 0.999)

    @staticmethod
    def from_torch(opt: torch.optim.Optimizer) -> "ImpalaAdam":
        if not isinstance(opt, torch.optim.Adam):
            raise TypeError("the HIP learner implements torch.optim.Adam only")
        g = opt.param_groups[0]
        if g.get("weight_decay", 0) or g.get("amsgrad", False) or g.get("maximize", False):
            raise ValueError("weight_decay / amsgrad / maximize are not used by the reference")
        return ImpalaAdam(lr=float(g["lr"]), eps=float(g["eps"]), betas=tuple(g["betas"]))


def _collate(batch, device) -> Tuple[torch.Tensor, ...]:
    """learning.py:123,142: list of B trajectories [s, a, r, g, mu] -> (B,T,...) device tensors.
    Accepts an already collated tuple (DeviceReplayBuffer.sample) unchanged."""
    if isinstance(batch, (tuple, list)) and len(batch) == 5 and isinstance(batch[0], torch.Tensor) \
            and batch[0].dim() == 5:
        return tuple(t if t.device == device else t.to(device, non_blocking=True) for t in batch)
    fields = []
    for j in range(5):
        xs = [item[j] for item in batch]
        if xs[0].device.type == "cpu":
            host = torch.stack(xs)
            if torch.cuda.is_available():
                host = host.pin_memory()
            t = host.to(device, non_blocking=True)
        else:
            t = torch.stack([x.to(device) for x in xs])
        if j in (1, 2, 3) and t.dim() == 3:
            t = t.squeeze(-1)
        fields.append(t.contiguous())
    obs, act, rew, disc, mu = fields
    return obs, act.to(torch.int64), rew.float(), disc.float(), mu.float()


# rows of the page-locked metrics ring: a step's host row is valid until the step
# HOST_METRICS_RING later is enqueued (DistributedAgent reads every sync_every < this)
HOST_METRICS_RING = 1024


@dataclass
class HostMetrics:
    """Where a step's metrics vector also lands in host memory (impala_set_metrics_host): the
    ring row (a numpy view of 16 floats; word 15 is the ready word the step's Adam kernel sets),
    the stream the step ran on, the learner and the step's index."""
    row: "np.ndarray"
    stream: "torch.cuda.Stream"
    learner: "ImpalaLearner"
    index: int

    def values(self):
        """-> the row's NUM_METRICS floats once the step's Adam kernel has stored them (its
        ready word; a short spin, then a stream synchronize), or None when the row has been
        handed to a later step since, or was never written (the caller then reads the device
        vector)."""
        if self.learner._step_count - self.index > HOST_METRICS_RING - 1:
            return None
        ready = self.row.view(np.uint32)
        if ready[15] == 0:
            t_end = time.perf_counter() + 2e-3
            while ready[15] == 0 and time.perf_counter() < t_end:
                pass
            if ready[15] == 0:
                self.stream.synchronize()
                if ready[15] == 0:
                    return None
        return self.row[:_lib.NUM_METRICS].tolist()


class StepMetrics(dict):
    """The metrics dict train_step returns (learning.py:161-174: key -> device scalar), with
    ``host``: the step's HostMetrics, or None."""
    host: Optional[HostMetrics] = None


class ImpalaLearner(Learner):
    def __init__(self, model, replay_buffer, optimizer=None, batch_size: int = 8,
                 max_grad_norm: float = 0.5, entropy_coeff: float = 0.01,
                 learning_starts: Optional[int] = None, model_push_period: int = 4,
                 rollout_length: int = 20, dtype: Optional[str] = None,
                 process_group=None, world_size: Optional[int] = None,
                 vtrace_grad_mode: Optional[str] = None, prefetch: int = 2):
        """The reference's constructor (learning.py:88-96) plus keyword-only extensions:
        ``rollout_length``, ``dtype`` ("fp32" | "bf16"), the data-parallel ``process_group`` /
        ``world_size``, ``vtrace_grad_mode`` -- what the V-trace backward treats as constant
        (``_lib.VTRACE_GRAD_MODES``; default "sg_advantage": targets and pg advantages constant,
        SURVEY.md §8(c); "sg_targets" / "sg_none" for rlax's stop_target_gradients=True / False
        with the advantage live) -- and ``prefetch``: the batches sampled and staged ahead,
        right after a step is enqueued (default 2), so the sampling, the host collate and the
        H2D copies of the next steps run while the GPU computes (the reference's replay client
        prefetches its samples the same way, conf/config.yaml ``prefetch: 5``); host batches
        then use prefetch + 1 staging slots.  0 samples inside each train_step, as
        learning.py:121 does."""
        self._model = model
        self._replay_buffer = replay_buffer
        if optimizer is None:
            optimizer = ImpalaAdam()
        elif isinstance(optimizer, torch.optim.Optimizer):
            optimizer = ImpalaAdam.from_torch(optimizer)
        self._optimizer = optimizer
        self._batch_size = batch_size
        self._max_grad_norm = max_grad_norm
        self._entropy_coeff = entropy_coeff
        self._learning_starts = learning_starts
        self._model_push_period = model_push_period
        self._rollout_length = rollout_length
        self._pg = process_group
        self._native_dp = None  # decided at the first data-parallel step (distributed.py)
        if world_size is None:
            world_size = 1
            if process_group is not None:
                import torch.distributed as dist
                world_size = dist.get_world_size(process_group)
        self._world_size = int(world_size)
        self._device = None
        self._prefetch = max(0, int(prefetch))
        # the prefetched (batch, slot, n_samples, sample seconds), oldest first
        self._queue = collections.deque()
        self._mhost = None  # the page-locked metrics ring (_host_row), False off the GPU
        self._rows_ok = None  # _rows_in_place
        self._next_m = None  # (the next step's metrics vector, the stream it was made on)
        self._ring = None  # (replay, Engine.ring_batch of its arrays)
        self._step_count = 0
        self._step_counter = 0
        self.can_train = True
        self._engine = Engine(model, batch_size=batch_size, rollout_length=rollout_length,
                              dtype=dtype, lr=optimizer.lr, eps=optimizer.eps,
                              betas=optimizer.betas, max_grad_norm=max_grad_norm,
                              entropy_coeff=entropy_coeff, world_size=self._world_size,
                              vtrace_grad_mode=vtrace_grad_mode)
        model._train_engine = self._engine

    @property
    def engine(self) -> Engine:
        return self._engine

    def device(self) -> torch.device:
        if self._device is None:
            self._device = self._model.flat.device
        return self._device

    @property
    def samples_per_step(self) -> int:
        """Environment frames one train_step consumes (DistributedAgent.train's total without
        a controller)."""
        return self._batch_size * self._rollout_length

    def prepare(self):  # learning.py:116-117
        self._replay_buffer.warm_up(self._learning_starts)

    def _row_key(self):
        """The (dtypes, byte sizes) of one trajectory's fields impala_stage_rows copies: obs u8
        (T,3,64,64), actions i64 (T,1), rewards / discounts f32 (T,1), logits f32 (T,A)."""
        T, A = self._rollout_length, self._engine.num_actions
        return ((torch.uint8, torch.int64, torch.float32, torch.float32, torch.float32),
                (T * 3 * 64 * 64, T * 8, T * 4, T * 4, T * A * 4))

    def _stage_host(self, batch):
        """learning.py:121-123,142 for host trajectories, staged through the library's H2D ring
        (two slots: the copies of step k+1 wait only for the step that last read the slot).
        A batch that carries its rows' host addresses (ReplayBuffer.sample's RowBatch) is
        staged by impala_stage_rows: the library's thread pool collates the rows into the slot's
        page-locked block, then the SDMA copies; any other list of trajectories is collated into
        this slot's page-locked buffers (one torch.stack per field) and staged by impala_stage.
        -> the slot (its device batch: Engine.slot_batch, on the stream that runs the step).
        Row batches return before their host collate: impala_stage_rows_async hands it to the
        library's staging thread, so with the prefetch it runs beside this thread's enqueue of
        the step and the device's work."""
        e = self._engine
        if getattr(e, "n_slots", 0) == 0:
            e.stage_init(max(2, self._prefetch + 1))  # the prefetched batches + the step's
            self._host_bufs = [None] * e.n_slots
            self._row_batches = [None] * e.n_slots
        self._slot = slot = (getattr(self, "_slot", -1) + 1) % e.n_slots
        e.stage_wait(slot)  # the previous copies out of this slot's host memory are done
        rows = getattr(batch, "row_ptrs", None)
        if rows is not None and len(batch) == e.batch_size and batch.row_key == self._row_key():
            # the library's staging thread collates and enqueues (slot_batch waits for it); the
            # rows stay alive until the slot is restaged, after its copies are done
            e.stage_rows(slot, rows, background=True)
            self._row_batches[slot] = batch
            return slot
        if self._host_bufs[slot] is None:
            B, T, A = self._batch_size, self._rollout_length, e.num_actions
            pin = torch.cuda.is_available()
            self._host_bufs[slot] = (
                torch.empty(B, T, 3, 64, 64, dtype=torch.uint8, pin_memory=pin),
                torch.empty(B, T, dtype=torch.int64, pin_memory=pin),
                torch.empty(B, T, dtype=torch.float32, pin_memory=pin),
                torch.empty(B, T, dtype=torch.float32, pin_memory=pin),
                torch.empty(B, T, A, dtype=torch.float32, pin_memory=pin))
        bufs = self._host_bufs[slot]
        if len(batch) != bufs[0].shape[0]:
            raise ValueError(f"replay returned {len(batch)} trajectories, expected {bufs[0].shape[0]}")
        for j, buf in enumerate(bufs):
            xs = [item[j] for item in batch]
            try:  # one collate per field (learning.py:142 torch.stack), into the pinned buffer
                torch.stack(xs, out=buf.view((len(xs),) + tuple(xs[0].shape)))
            except (RuntimeError, TypeError):  # other dtype / shape spelling: per trajectory
                for i, x in enumerate(xs):
                    buf[i].copy_(x.reshape(buf.shape[1:]))
        e.stage(slot, *bufs)
        return slot

    def _fetch(self):
        """learning.py:121-123: replay.sample(B) and its staging -> (a device batch for
        _train_step, or None when it sits in a staging slot; the slot or None; frames; seconds
        spent).  Host batches are staged (copies enqueued) here; their slot's device views are
        taken by _resolve on the thread that runs the step."""
        t0 = time.perf_counter()
        if self._rows_in_place():
            # the sampled slots only: the step reads them from the ring in place
            # (Engine.train_step_rows), no gather
            _, rs, _ = self._replay_buffer.sample_rows(self._batch_size)
            return (rs,), None, self._batch_size * self._rollout_length, time.perf_counter() - t0, None
        _, batch, _ = self._replay_buffer.sample(self._batch_size)
        slot = None
        if isinstance(batch, list) and batch and isinstance(batch[0][0], torch.Tensor) \
                and batch[0][0].device.type == "cpu":
            slot = self._stage_host(batch)
            batch = None
            n_samples = self._batch_size * self._rollout_length
        else:
            tensors = _collate(batch, self.device())
            n_samples = self._batch_size * tensors[0].shape[1]
            # checked and turned into the library's batch struct here, off the path from the
            # previous step's metrics read to this step's first launch; the tensors stay
            # referenced by the queue entry until the step is enqueued
            return (self._engine._batch(*tensors),), None, n_samples, time.perf_counter() - t0, tensors
        return batch, slot, n_samples, time.perf_counter() - t0, None

    def _resolve(self, item):
        batch, slot, n_samples, sample_s, keep = item
        if slot is not None:  # the step's stream waits for the slot's copies
            batch = (self._engine.slot_batch(slot),)
        return batch, slot, n_samples, sample_s, keep

    def _rows_in_place(self) -> bool:
        """Whether the learner's steps read a DeviceReplayBuffer's slots in place
        (IMPALA_REPLAY_ROWS=0 turns it off; world size 1 only, batch <= 256; a handle that turns
        out not to support it -- A/B kernel knobs -- falls back to gathers for good)."""
        if self._rows_ok is None:
            from impala_amd.replay import DeviceReplayBuffer
            self._rows_ok = (isinstance(self._replay_buffer, DeviceReplayBuffer) and
                             self._world_size == 1 and self._batch_size <= 256 and
                             self._replay_buffer.T == self._rollout_length and
                             os.environ.get("IMPALA_REPLAY_ROWS", "1") != "0")
        return self._rows_ok

    def _refill(self):
        """Sample and stage batches until `prefetch` are queued (a device replay's gathers go on
        the learner's stream behind this step; host batches' collates and copies are handed to
        the library's staging thread, which runs them back to back).  A replay that cannot give
        a batch now is asked again by the next call, synchronously when nothing is queued
        (raising there if it still cannot)."""
        while len(self._queue) < self._prefetch:
            try:
                self._queue.append(self._fetch())
            except Exception:  # noqa: BLE001 -- re-raised by a later call's own sample
                break

    def _take_next(self):
        return self._queue.popleft() if self._queue else self._fetch()

    def train_step(self):  # learning.py:119-138
        t0 = time.perf_counter()
        batch, slot, n_samples, sample_s, keep = self._resolve(self._take_next())
        t1 = time.perf_counter()
        metrics = self._train_step(batch)
        del keep  # (the device batch's tensors: enqueued now, stream-ordered from here)
        if slot is not None:
            self._engine.slot_release(slot)
        t2 = time.perf_counter()
        self._refill()  # the next steps' batches, while this step runs on the device
        if self._engine.device.type == "cuda":  # the next step's metrics vector, made now
            self._next_m = (torch.empty(_lib.NUM_METRICS, dtype=torch.float32, device=self._engine.device),
                            torch.cuda.current_stream(self._engine.device))
        update_time = 0
        self._step_count += 1
        self._step_counter = self._step_count
        if self._step_count % self._model_push_period == 0:
            start = time.perf_counter()
            self._model.push()
            update_time = time.perf_counter() - start
        # same definitions (and units) as the reference, learning.py:133-137 (the sample time
        # is this batch's own, also when it was prefetched by the previous call)
        metrics["debug/replay_sample_per_second"] = (n_samples / (max(sample_s, 1e-9) * 1000))
        metrics["debug/gradient_per_second"] = (n_samples / ((t2 - t1) * 1000))
        metrics["debug/total_time"] = (time.perf_counter() - t0) * 1000
        metrics["debug/forward_dt"] = (t2 - t1) * 1000 / self._batch_size
        metrics["debug/update_time"] = update_time
        return metrics

    def _host_row(self):
        """This step's row of the page-locked metrics ring (impala_set_metrics_host) as (tensor,
        numpy view) with its ready word cleared, or None off the GPU."""
        if self._mhost is None:
            if self._engine.device.type != "cuda":
                self._mhost = False
            else:
                t = torch.zeros(HOST_METRICS_RING, 16, dtype=torch.float32, pin_memory=True)
                self._mhost = (t, t.numpy(), [r for r in t])  # (numpy view and rows share t)
        if self._mhost is False:
            return None
        i = self._step_count % HOST_METRICS_RING
        t, tn, rows = self._mhost
        tn[i].view(np.uint32)[15] = 0  # the ready word, set again by this step's Adam kernel
        return rows[i], tn[i]

    def _train_step(self, batch) -> Dict[str, torch.Tensor]:  # learning.py:140-177
        e = self._engine
        # this step's metrics go to a vector of its own, which the returned values are views
        # of (impala_set_metrics: no device copy after the step), and to a row of a page-locked
        # ring that the step's last kernel writes (impala_set_metrics_host)
        cur = torch.cuda.current_stream(e.device) if e.device.type == "cuda" else None
        m, self._next_m = self._next_m, None
        if m is None or m[1] != cur:  # (made on another stream: not reused across streams)
            m = (torch.empty(_lib.NUM_METRICS, dtype=torch.float32, device=e.device), cur)
        m = m[0]
        hr = self._host_row()
        e._bind_metrics(m, None if hr is None else hr[0])
        if len(batch) == 1 and isinstance(batch[0], RowSample):
            rs = batch[0]
            try:
                if self._ring is None or self._ring[0] is not rs.replay:  # checked once per replay
                    self._ring = (rs.replay,) + e.ring_batch(rs.replay.fields)
                _, rb_, cap = self._ring
                rs.replay.read_rows(rs, lambda fields, idx, st: e._train_step_rows(rb_, cap, idx, st),
                                    cur)
            except _lib.Unsupported:  # not on the default kernels: gather, for good
                self._rows_ok = False
                e.train_step(*rs.gather())
        elif self._world_size == 1:
            e.train_step(*batch)
        else:
            from .distributed import (compute_grads_allreduced, native_dp_buckets,
                                      native_dp_enabled)
            if self._native_dp is None:
                native = native_dp_enabled(self._pg)
                if native:
                    e.dp_init(self._pg)  # raises before the path is chosen if RCCL fails
                self._native_dp = native
            if self._native_dp:
                e.dp_train_step(*batch, buckets=native_dp_buckets())
            else:
                compute_grads_allreduced(e, batch, self._model.flat_grad, group=self._pg)
                e.apply_update()
        # device scalars, views of the step's metrics vector: float(v) synchronises lazily;
        # DistributedAgent reads the host row once the step's Adam kernel has set its ready word
        # (agent._read_values), or moves all of a step's values with one copy
        out = StepMetrics(zip(_lib.METRIC_NAMES, m.unbind(0)))
        if hr is not None:  # (no event per step: its marker left a 6 us gap, profiles/r06lt)
            out.host = HostMetrics(hr[1], cur, self, self._step_count)
        return out

    # ---------------------------------------------------------------- checkpoint
    def optimizer_state(self) -> dict:
        return {"step": int(self._engine.metrics[7].item()), "exp_avg": self._engine.exp_avg.clone(),
                "exp_avg_sq": self._engine.exp_avg_sq.clone()}

    def load_optimizer_state(self, st: dict) -> None:
        self._engine.exp_avg.copy_(st["exp_avg"])
        self._engine.exp_avg_sq.copy_(st["exp_avg_sq"])
        self._engine.set_step(int(st["step"]))
