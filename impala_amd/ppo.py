"""PPOLearner — drop-in for ``agents/ppo/learning.py:78-143`` on MI355X.

Same constructor (``model, replay_buffer, optimizer, batch_size=256, max_grad_norm=0.5,
entropy_coeff=0.01, learning_starts=None, model_push_period=8``), ``prepare`` /
``train_step`` behaviour and metric keys (``train/{loss,entropy,td,pg,target,kl,ratio}``,
``train_step/grad_norm``, ``debug/*``).  ``_train_step`` is one HIP call on a PPO handle
(``impala_ppo_train_step``: the shared CNN forward, the fused PPO head -- clipped surrogate,
½·td², entropy, KL -- the shared backward, clip and Adam), or for data-parallel replicas the
data-parallel gradient path of ``distributed.compute_grads_allreduced``.

The batch is flat transitions ``(s u8 [N,3,64,64], a i64 [N], v_target f32 [N], pi_ref
logits f32 [N,A])`` -- the order ``_train_step`` unpacks (learning.py:132).  The reference
actor's target computation (``rlego.lambda_returns``, learning.py:64-69) cannot run as shipped
(``values`` is undefined there), so targets arrive with the batch exactly as the learner
expects them.
"""
from __future__ import annotations

import time
from typing import Dict, Optional

import torch

from impala_amd import _lib
from impala_amd.core import Learner
from impala_amd.engine import Engine
from impala_amd.learner import ImpalaAdam


def collate_transitions(batch, device):
    """CircularBuffer(collate_fn=torch.cat) semantics (agents/ppo/builder.py:30-35): a list of
    transition items ``[s, a, target, pi_ref]`` (each with a leading dim, or without one) ->
    4 contiguous device tensors; an already-collated 4-tuple is moved as is."""
    if isinstance(batch, (tuple, list)) and len(batch) == 4 and isinstance(batch[0], torch.Tensor) \
            and batch[0].dim() == 4:
        fields = list(batch)
    else:
        fields = []
        for j in range(4):
            xs = [item[j] for item in batch]
            xs = [x if x.dim() > (3 if j == 0 else (1 if j == 3 else 0)) else x.unsqueeze(0)
                  for x in xs]
            fields.append(torch.cat(xs))
    out = []
    for j, t in enumerate(fields):
        if t.device != device:
            if t.device.type == "cpu" and torch.cuda.is_available():
                t = t.pin_memory()
            t = t.to(device, non_blocking=True)
        out.append(t.contiguous())
    s, a, tgt, mu = out
    return (s, a.reshape(-1).to(torch.int64), tgt.reshape(-1).float(),
            mu.reshape(s.shape[0], -1).float())


class PPOLearner(Learner):
    def __init__(self, model, replay_buffer, optimizer=None, batch_size: int = 256,
                 max_grad_norm: float = 0.5, entropy_coeff: float = 0.01,
                 learning_starts: Optional[int] = None, model_push_period: int = 8,
                 clip_coeff: float = 0.1, dtype: Optional[str] = None, process_group=None,
                 world_size: Optional[int] = None):
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
        self._pg = process_group
        self._native_dp = None  # decided at the first data-parallel step (distributed.py)
        if world_size is None:
            world_size = 1
            if process_group is not None:
                import torch.distributed as dist
                world_size = dist.get_world_size(process_group)
        self._world_size = int(world_size)
        self._device = None
        self._step_counter = 0
        self.can_train = False
        # losses.ppo_loss's clip_coeff default (losses.py:131): the learner never overrides it
        self._engine = Engine(model, batch_size=batch_size, algo="ppo", ppo_clip=clip_coeff,
                              dtype=dtype, lr=optimizer.lr, eps=optimizer.eps,
                              betas=optimizer.betas, max_grad_norm=max_grad_norm,
                              entropy_coeff=entropy_coeff, world_size=self._world_size)
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
        return self._batch_size

    def prepare(self):  # learning.py:105-108
        if not self.can_train:
            self._replay_buffer.warm_up(self._learning_starts)
        self.can_train = True

    def train_step(self):  # learning.py:110-128
        t0 = time.perf_counter()
        _, batch, _ = self._replay_buffer.sample(self._batch_size)
        batch = collate_transitions(batch, self.device())
        t1 = time.perf_counter()
        metrics = self._train_step(batch)
        t2 = time.perf_counter()
        self._step_counter += 1
        update_time = 0
        if self._step_counter % self._model_push_period == 0:
            start = time.perf_counter()
            self._model.push()
            update_time = (time.perf_counter() - start) * 1000
        metrics["debug/replay_sample_per_second"] = (self._batch_size / ((t1 - t0) * 1000))
        metrics["debug/gradient_per_second"] = (self._batch_size / ((t2 - t1) * 1000))
        metrics["debug/total_time"] = (time.perf_counter() - t0) * 1000
        metrics["debug/forward_dt"] = (t2 - t1) * 1000
        metrics["debug/update_time"] = update_time
        return metrics

    def _train_step(self, batch) -> Dict[str, torch.Tensor]:  # learning.py:130-143
        e = self._engine
        # this step's metrics vector (impala_set_metrics), which the returned values are views of
        m = torch.empty(_lib.NUM_METRICS, dtype=torch.float32, device=e.device)
        e.bind_metrics(m)
        if self._world_size == 1:
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
        v = m.unbind(0)  # device scalars; float(v) synchronises lazily
        return {name: v[i] for name, i in _lib.PPO_METRIC_SLOTS}
