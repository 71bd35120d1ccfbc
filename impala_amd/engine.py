"""Engine: one HIP learner handle (``impala_learner*``) bound to a model's flat buffers.

Owns the Adam moments and the device metrics vector as torch tensors; the library owns its
activation / slab / kernel-layout-weight workspace.  All calls are asynchronous on torch's
current HIP stream (or an explicit one).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence, Tuple

import torch

from impala_amd import _lib
from impala_amd._lib import ImpalaBatch, ImpalaConfig, ImpalaRows, check, ptr, stream_ptr

DTYPES = {"fp32": _lib.IMPALA_DTYPE_F32, "f32": _lib.IMPALA_DTYPE_F32,
          "float32": _lib.IMPALA_DTYPE_F32, "bf16": _lib.IMPALA_DTYPE_BF16,
          "bfloat16": _lib.IMPALA_DTYPE_BF16}


class Engine:
    def __init__(self, model, batch_size: int, rollout_length: int = 20, dtype: Optional[str] = None,
                 lr: float = 1e-4, eps: float = 1e-5, betas: Tuple[float, float] = (0.9, 0.999),
                 max_grad_norm: float = 0.5, entropy_coeff: float = 0.01, world_size: int = 1,
                 vtrace_lambda: float = 1.0, clip_rho_threshold: float = 1.0,
                 clip_pg_rho_threshold: float = 1.0, inference_only: bool = False,
                 algo: str = "impala", ppo_clip: float = 0.1, vtrace_grad_mode=None):
        if model.flat.device.type != "cuda":
            raise RuntimeError("the IMPALA learner runs on the HIP path only (cuda device)")
        self.model = model
        self.device = model.flat.device
        if algo not in ("impala", "ppo"):
            raise ValueError(f"unknown algo {algo!r}")
        self.algo = algo
        self.batch_size = int(batch_size)
        # PPO learns from flat transitions (agents/ppo/learning.py:132): N = batch_size
        self.rollout_length = 1 if algo == "ppo" else int(rollout_length)
        self.num_actions = model.action_dim
        self.inference_only = inference_only
        dtype = dtype or model.compute_dtype
        if dtype not in DTYPES:
            raise ValueError(f"unknown dtype {dtype!r}")
        self.dtype = dtype
        L = _lib.lib()
        cfg = _lib.default_config()
        cfg.batch_size = self.batch_size
        cfg.rollout_length = self.rollout_length
        cfg.num_actions = self.num_actions
        cfg.dtype = DTYPES[dtype]
        cfg.lr, cfg.adam_eps = lr, eps
        cfg.adam_beta1, cfg.adam_beta2 = betas
        cfg.max_grad_norm = max_grad_norm
        cfg.entropy_coeff = entropy_coeff
        cfg.vtrace_lambda = vtrace_lambda
        cfg.clip_rho_threshold = clip_rho_threshold
        cfg.clip_pg_rho_threshold = clip_pg_rho_threshold
        cfg.world_size = int(world_size)
        cfg.algo = _lib.IMPALA_ALGO_PPO if algo == "ppo" else _lib.IMPALA_ALGO_IMPALA
        cfg.ppo_clip = float(ppo_clip)
        cfg.vtrace_grad_mode = _lib.vtrace_grad_mode(vtrace_grad_mode)
        self.cfg = cfg
        h = C.c_void_p()
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        check(L.impala_create(C.byref(cfg), idx, C.byref(h)), "impala_create")
        self._h = h
        n = model.flat.numel()
        assert n == _lib.param_count(self.num_actions)
        if inference_only:
            self.exp_avg = self.exp_avg_sq = self.metrics = None
            check(L.impala_bind_state(h, ptr(model.flat), None, None, None, None,
                                      stream_ptr(None)), "impala_bind_state")
        else:
            self.exp_avg = torch.zeros_like(model.flat)
            self.exp_avg_sq = torch.zeros_like(model.flat)
            self.metrics = torch.zeros(_lib.NUM_METRICS, dtype=torch.float32, device=self.device)
            check(L.impala_bind_state(h, ptr(model.flat), ptr(model.flat_grad), ptr(self.exp_avg),
                                      ptr(self.exp_avg_sq), ptr(self.metrics), stream_ptr(None)),
                  "impala_bind_state")
        self._version = model._version
        self._metrics_host = False  # impala_set_metrics_host bound (bind_metrics)
        self._dp = False  # dp_init ran: the handle has its own RCCL communicator

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.lib().impala_destroy(h)
            except Exception:
                pass
            self._h = None

    def __del__(self):
        self.close()

    @property
    def frames(self) -> int:
        return self.batch_size * self.rollout_length

    def refresh_weights(self, stream=None):
        check(_lib.lib().impala_refresh_weights(self._h, stream_ptr(stream)),
              "impala_refresh_weights")
        self._version = self.model._version

    def _sync_weights(self, stream=None):
        if self._version != self.model._version:
            self.refresh_weights(stream)

    def bind_metrics(self, metrics: torch.Tensor, host: Optional[torch.Tensor] = None):
        """The following steps write their metrics into `metrics` (a device float32 vector of
        NUM_METRICS, impala_set_metrics; no device work), which becomes ``self.metrics``; and,
        when `host` (a page-locked float32 CPU vector of NUM_METRICS) is given, also into
        `host` (impala_set_metrics_host: readable once an event recorded after the step has
        completed).  ``host=None`` stops the host copy."""
        if metrics.dtype != torch.float32 or metrics.device != self.device or \
                metrics.numel() < _lib.NUM_METRICS or not metrics.is_contiguous():
            raise ValueError(f"metrics must be a contiguous float32 vector of >= "
                             f"{_lib.NUM_METRICS} on {self.device}")
        if host is not None and (host.dtype != torch.float32 or host.device.type != "cpu" or
                                 host.numel() < _lib.NUM_METRICS or not host.is_contiguous()):
            raise ValueError(f"host metrics must be a contiguous float32 CPU vector of >= "
                             f"{_lib.NUM_METRICS}")
        self._bind_metrics(metrics, host)

    def _bind_metrics(self, metrics, host=None):
        """bind_metrics without the argument checks (for vectors the caller made to measure)."""
        L = _lib.lib()
        check(L.impala_set_metrics(self._h, metrics.data_ptr()), "impala_set_metrics")
        if host is not None or self._metrics_host:
            check(L.impala_set_metrics_host(self._h, None if host is None else host.data_ptr()),
                  "impala_set_metrics_host")
            self._metrics_host = host is not None
        self.metrics = metrics

    def set_step(self, step: int, stream=None):
        check(_lib.lib().impala_set_step(self._h, int(step), stream_ptr(stream)), "impala_set_step")

    def debug_vtrace(self, enable: bool = True):
        """Export the step's own V-trace from the fused head (impala_set_debug_vtrace): returns a
        dict of device views ``adv``, ``err``, ``q`` [B,T-1], ``rho`` and the values ``v`` [B,T] the
        scan ran on, refilled by every
        following training step; ``enable=False`` turns the export off (returns None)."""
        if not enable:
            check(_lib.lib().impala_set_debug_vtrace(self._h, None), "impala_set_debug_vtrace")
            self._vt_dbg = None
            return None
        B, T = self.batch_size, self.rollout_length
        L = T - 1
        buf = torch.zeros(3 * B * L + 2 * B * T, dtype=torch.float32, device=self.device)
        check(_lib.lib().impala_set_debug_vtrace(self._h, ptr(buf)), "impala_set_debug_vtrace")
        self._vt_dbg = buf  # keeps the buffer alive while the library writes into it
        BL = B * L
        return {"adv": buf[:BL].view(B, L), "err": buf[BL:2 * BL].view(B, L),
                "q": buf[2 * BL:3 * BL].view(B, L), "rho": buf[3 * BL:3 * BL + B * T].view(B, T),
                "v": buf[3 * BL + B * T:].view(B, T)}

    # ------------------------------------------------------------------ compute
    def forward(self, obs: torch.Tensor, stream=None):
        """obs u8 [N,3,64,64] (any N; chunked by the handle capacity) -> logits [N,A], v [N,1]."""
        if obs.dtype != torch.uint8 or obs.shape[-3:] != (3, 64, 64):
            raise ValueError("obs must be uint8 [..., 3, 64, 64]")
        obs = obs.reshape(-1, 3, 64, 64)
        if obs.device != self.device:
            obs = obs.to(self.device, non_blocking=True)
        obs = obs.contiguous()
        self._sync_weights(stream)
        n = obs.shape[0]
        logits = torch.empty(n, self.num_actions, dtype=torch.float32, device=self.device)
        values = torch.empty(n, 1, dtype=torch.float32, device=self.device)
        cap = self.frames
        L = _lib.lib()
        sp = stream_ptr(stream)
        for s in range(0, n, cap):
            e = min(n, s + cap)
            check(L.impala_forward(self._h, ptr(obs[s:e]), e - s, ptr(logits[s:e]), ptr(values[s:e]),
                                   sp), "impala_forward")
        return logits, values

    def act(self, obs: torch.Tensor, deterministic=False, seed: int = 0, counter: int = 0,
            stream=None):
        """models/distributed_models.py:21-32 on device (impala_act): obs u8 [N,3,64,64],
        deterministic a bool or a per-frame bool tensor -> (actions i64 [N,1], logits [N,A],
        v [N,1]); stochastic actions are draws from softmax(logits) keyed by (seed, counter,
        frame) -- pass a fresh counter per call."""
        if obs.dtype != torch.uint8 or obs.shape[-3:] != (3, 64, 64):
            raise ValueError("obs must be uint8 [..., 3, 64, 64]")
        obs = obs.reshape(-1, 3, 64, 64)
        if obs.device != self.device:
            obs = obs.to(self.device, non_blocking=True)
        obs = obs.contiguous()
        self._sync_weights(stream)
        n = obs.shape[0]
        det_all, det = 0, None
        if isinstance(deterministic, torch.Tensor):
            d = deterministic.reshape(-1).to(self.device)
            if d.numel() == 1:
                det_all = int(bool(d.item()))
            elif d.numel() == n:
                det = d.to(torch.uint8).contiguous()
            else:
                raise ValueError(f"deterministic flags: {d.numel()} for {n} frames")
        else:
            det_all = int(bool(deterministic))
        actions = torch.empty(n, 1, dtype=torch.int64, device=self.device)
        logits = torch.empty(n, self.num_actions, dtype=torch.float32, device=self.device)
        values = torch.empty(n, 1, dtype=torch.float32, device=self.device)
        cap = self.frames
        L = _lib.lib()
        sp = stream_ptr(stream)
        for s in range(0, n, cap):
            e = min(n, s + cap)
            # frame index within the call keys the draw: chunks offset the counter
            check(L.impala_act(self._h, ptr(obs[s:e]), e - s, ptr(det[s:e]) if det is not None else None,
                               det_all, int(seed), int(counter) * 1_000_003 + s, ptr(actions[s:e]),
                               ptr(logits[s:e]), ptr(values[s:e]), sp), "impala_act")
        return actions, logits, values

    def _batch(self, *batch, device=None) -> ImpalaBatch:
        """IMPALA: (obs u8 [B,T,3,64,64], actions i64 [B,T], rewards [B,T], discounts [B,T],
        behaviour logits [B,T,A]).  PPO: (obs u8 [N,3,64,64], actions i64 [N], value targets
        [N], behaviour logits [N,A]) -- passed to the library with rewards = targets.
        A single ImpalaBatch (a staging-ring slot, slot_batch) passes through unchanged."""
        if len(batch) == 1 and isinstance(batch[0], ImpalaBatch):
            return batch[0]
        device = self.device if device is None else torch.device(device)
        B, T, A = self.batch_size, self.rollout_length, self.num_actions
        if self.algo == "ppo":
            names = ("obs", "actions", "targets", "behaviour_logits")
            exp = (((B, 3, 64, 64), torch.uint8), ((B,), torch.int64), ((B,), torch.float32),
                   ((B, A), torch.float32))
        else:
            names = ("obs", "actions", "rewards", "discounts", "behaviour_logits")
            exp = (((B, T, 3, 64, 64), torch.uint8), ((B, T), torch.int64),
                   ((B, T), torch.float32), ((B, T), torch.float32), ((B, T, A), torch.float32))
        if len(batch) != len(names):
            raise ValueError(f"{self.algo} batch is {names}, got {len(batch)} tensors")
        for k, t, (shape, dt) in zip(names, batch, exp):
            if tuple(t.shape) != shape or t.dtype != dt:
                raise ValueError(f"{k}: expected {dt} {shape}, got {t.dtype} {tuple(t.shape)}")
            if t.device != device or not t.is_contiguous():
                raise ValueError(f"{k}: must be a contiguous tensor on {device}")
        if self.algo == "ppo":
            obs, actions, targets, mu = batch
            return ImpalaBatch(ptr(obs), ptr(actions), ptr(targets), None, ptr(mu))
        return ImpalaBatch(*[ptr(t) for t in batch])

    def train_step(self, *batch, stream=None):
        """Full update (world_size 1): IMPALA learning.py:140-177, PPO
        agents/ppo/learning.py:131-143 (the batch layout follows the handle's algo)."""
        b = self._batch(*batch)
        self._sync_weights(stream)
        check(_lib.lib().impala_train_step(self._h, C.byref(b), stream_ptr(stream)),
              "impala_train_step")
        self._updated()

    def ring_batch(self, ring):
        """Check a replay ring's five device arrays -- (obs u8 [C,T,3,64,64], actions i64 [C,T],
        rewards [C,T], discounts [C,T], behaviour logits [C,T,A]) -- once -> (the library's batch
        struct of their base addresses, C) for train_step_rows (the caller keeps the arrays)."""
        obs = ring[0]
        C_, T, A = obs.shape[0], self.rollout_length, self.num_actions
        exp = (((C_, T, 3, 64, 64), torch.uint8), ((C_, T), torch.int64), ((C_, T), torch.float32),
               ((C_, T), torch.float32), ((C_, T, A), torch.float32))
        if len(ring) != 5:
            raise ValueError("a ring is (obs, actions, rewards, discounts, behaviour logits)")
        for t, (shape, dt) in zip(ring, exp):
            if tuple(t.shape) != shape or t.dtype != dt or t.device != self.device or not t.is_contiguous():
                raise ValueError(f"ring field: expected contiguous {dt} {shape} on {self.device}, "
                                 f"got {t.dtype} {tuple(t.shape)} on {t.device}")
        return ImpalaBatch(*[ptr(t) for t in ring]), int(C_)

    def train_step_rows(self, ring, rows, stream=None):
        """The full update on the trajectories ``rows`` (host int64 slot indices, one per batch
        row) read in place from a replay ring -- the five device arrays, or ring_batch's result
        for them -- (impala_train_step_rows; bitwise the same step as train_step on the gathered
        batch).  Raises _lib.Unsupported when the handle does not run the default fused
        kernels."""
        import numpy as np
        b, cap = ring if isinstance(ring[0], ImpalaBatch) else self.ring_batch(ring)
        idx = rows if isinstance(rows, np.ndarray) and rows.dtype == np.int64 and \
            rows.flags.c_contiguous else np.ascontiguousarray(rows, dtype=np.int64)
        self._train_step_rows(b, cap, idx, stream)

    def _train_step_rows(self, b, cap, idx, stream):
        """train_step_rows on a ring_batch struct and a contiguous int64 index array."""
        if self._version != self.model._version:
            self.refresh_weights(stream)
        check(_lib.lib().impala_train_step_rows(self._h, b, idx.ctypes.data, idx.size, cap,
                                                stream_ptr(stream)),
              "impala_train_step_rows")
        self._updated()

    def compute_grads(self, *batch, stream=None):
        b = self._batch(*batch)
        self._sync_weights(stream)
        check(_lib.lib().impala_compute_grads(self._h, C.byref(b), stream_ptr(stream)),
              "impala_compute_grads")

    def compute_grads_part(self, part, *batch, stream=None):
        """A piece of compute_grads.  Two buckets: part 0 finishes grads[bucket_offset:]
        (conv3 .. heads), part 1 (same batch) grads[:bucket_offset] (conv1, conv2) and the
        metrics.  Three buckets: part 2 finishes grads[bucket_offset_fc:] (FC, heads), part 3
        grads[bucket_offset:bucket_offset_fc] (conv3, LayerNorm), part 4 = part 1.  Two buckets
        on the fused per-frame backward: part 2, then part 6 grads[:bucket_offset_fc] + metrics."""
        b = self._batch(*batch)
        if part in (0, 2):
            self._sync_weights(stream)
        check(_lib.lib().impala_compute_grads_part(self._h, C.byref(b), int(part),
                                                   stream_ptr(stream)),
              "impala_compute_grads_part")

    @property
    def bucket_offset(self) -> int:
        """First flat-gradient index of bucket 1 (all-reduced while part 1 runs)."""
        return int(_lib.lib().impala_grad_bucket_offset(self._h))

    @property
    def bucket_offset_fc(self) -> int:
        """First flat-gradient index of the FC + heads bucket (final after part 2)."""
        return int(_lib.lib().impala_grad_bucket_offset_fc(self._h))

    # ------------------------------------------------------------------ native data parallel
    def dp_init(self, group=None):
        """Give the handle its own RCCL communicator over the replicas of ``group`` (collective:
        every rank calls it).  Rank 0 of the group creates the 128-byte communicator id
        (impala_dp_unique_id), torch.distributed broadcasts it, every rank runs impala_dp_init."""
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        if world != self.cfg.world_size:
            raise ValueError(f"group has {world} ranks, the handle was created for "
                             f"world_size {self.cfg.world_size}")
        uid = torch.zeros(_lib.DP_ID_BYTES, dtype=torch.uint8)
        if rank == 0:
            check(_lib.lib().impala_dp_unique_id(ptr(uid)), "impala_dp_unique_id")
        on_dev = dist.get_backend(group) == "nccl"
        t = uid.to(self.device) if on_dev else uid
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast(t, src, group=group)
        uid = t.cpu() if on_dev else t
        check(_lib.lib().impala_dp_init(self._h, ptr(uid), world, rank), "impala_dp_init")
        self._dp = True

    @property
    def dp_nranks(self) -> int:
        """Rank count of the handle's RCCL communicator (ncclCommCount; 0 before dp_init)."""
        n = C.c_int()
        check(_lib.lib().impala_dp_nranks(self._h, C.byref(n)), "impala_dp_nranks")
        return int(n.value)

    def dp_train_step(self, *batch, buckets: int = 1, stream=None):
        """The whole data-parallel step on the handle's communicator (impala_dp_train_step):
        local gradients, in-place RCCL all-reduce (sum) on the compute stream -- ``buckets=2``:
        the FC + heads bucket on the handle's side stream, overlapped with the per-frame
        backward -- then clip + Adam on the summed gradient."""
        b = self._batch(*batch)
        self._sync_weights(stream)
        check(_lib.lib().impala_dp_train_step(self._h, C.byref(b), int(buckets),
                                              stream_ptr(stream)), "impala_dp_train_step")
        self._updated()

    def apply_update(self, stream=None):
        check(_lib.lib().impala_apply_update(self._h, stream_ptr(stream)), "impala_apply_update")
        self._updated()

    # ------------------------------------------------------------------ host staging ring
    def stage_init(self, nslots: int = 2):
        """Allocate `nslots` device batch slots (impala_stage_init)."""
        check(_lib.lib().impala_stage_init(self._h, int(nslots)), "impala_stage_init")
        self.n_slots = int(nslots)
        self._staged = [None] * self.n_slots

    def stage(self, slot: int, *host_batch):
        """Enqueue the H2D copies of a host batch (train_step's layout; page-locked memory for
        an asynchronous copy) into ring slot `slot`, after the last step that read the slot."""
        b = self._batch(*host_batch, device="cpu")
        check(_lib.lib().impala_stage(self._h, C.byref(b), int(slot)), "impala_stage")
        self._staged[slot] = host_batch  # the copies read these until stage_wait(slot)

    def stage_rows(self, slot: int, row_ptrs, background: bool = False):
        """Enqueue the H2D copies of B trajectories that are NOT collated (impala_stage_rows):
        ``row_ptrs`` = five arrays of B host addresses (numpy uint64, or sequences of ints),
        trajectory b's obs / actions / rewards / discounts / behaviour-logits rows (discounts
        None on PPO handles).  The rows must stay unchanged until stage_wait(slot).
        ``background``: the handle's staging thread does the host collate and the enqueue
        (impala_stage_rows_async); slot_batch / stage_wait wait for it."""
        import numpy as np
        arrs = [None if p is None else np.ascontiguousarray(p, dtype=np.uint64) for p in row_ptrs]
        B = self.batch_size
        for a in arrs:
            if a is not None and a.shape != (B,):
                raise ValueError(f"row pointer arrays must hold {B} addresses")
        rows = ImpalaRows(*[0 if a is None else a.ctypes.data for a in arrs])
        fn = "impala_stage_rows_async" if background else "impala_stage_rows"
        check(getattr(_lib.lib(), fn)(self._h, C.byref(rows), B, int(slot)), fn)
        self._staged[slot] = arrs

    def stage_wait(self, slot: int):
        """Block until the copies into `slot` are done (its host batch may be reused)."""
        check(_lib.lib().impala_stage_wait(self._h, int(slot)), "impala_stage_wait")
        self._staged[slot] = None

    def slot_batch(self, slot: int, stream=None) -> ImpalaBatch:
        """The slot's device batch for train_step / compute_grads*; `stream` (torch's current
        when None) waits for the slot's copies."""
        b = ImpalaBatch()
        check(_lib.lib().impala_slot_batch(self._h, int(slot), stream_ptr(stream), C.byref(b)),
              "impala_slot_batch")
        return b

    def slot_release(self, slot: int, stream=None):
        """The steps reading `slot` are enqueued on `stream`: the next stage() into it waits
        for them."""
        check(_lib.lib().impala_slot_release(self._h, int(slot), stream_ptr(stream)),
              "impala_slot_release")

    # ------------------------------------------------------------------ live launch timer
    @staticmethod
    def kernel_names():
        L = _lib.lib()
        return [L.impala_kernel_name(i).decode() for i in range(L.impala_kernel_count())]

    def timer_start(self, kernel: str, max_launches: int):
        kid = self.kernel_names().index(kernel)
        check(_lib.lib().impala_timer_start(self._h, kid, int(max_launches)), "impala_timer_start")

    def timer_read(self, kernel: Optional[str] = None):
        """-> (summed kernel duration in ms, launches) of `kernel` (default: the kernel armed
        last); disarms it.  Several kernels may be armed at once."""
        ms, n = C.c_float(), C.c_int()
        if kernel is None:
            check(_lib.lib().impala_timer_read(self._h, C.byref(ms), C.byref(n)),
                  "impala_timer_read")
        else:
            kid = self.kernel_names().index(kernel)
            check(_lib.lib().impala_timer_read_kernel(self._h, kid, C.byref(ms), C.byref(n)),
                  "impala_timer_read_kernel")
        return float(ms.value), int(n.value)

    # ------------------------------------------------------------------ device step clock
    def step_clock_start(self, n: int):
        """Arm the device step clock for the next `n` steps: each step's first kernel stamps
        the device's 100 MHz clock as it starts (impala_step_clock); nothing is enqueued
        between the steps."""
        self._clock = torch.zeros(int(n) + 1, dtype=torch.int64, device=self.device)
        self._clock_steps = None  # set by step_clock_end for this region
        check(_lib.lib().impala_step_clock(self._h, ptr(self._clock), int(n)), "impala_step_clock")

    def step_clock_end(self, stream=None):
        """Enqueue the stamp that closes the last armed step (a 1-thread kernel on `stream`)
        and disarm; no host sync."""
        k = C.c_int()
        check(_lib.lib().impala_step_clock_end(self._h, stream_ptr(stream), C.byref(k)),
              "impala_step_clock_end")
        self._clock_steps = k.value

    def step_clock_read(self):
        """-> the per-step device times in ms of the last clocked region (a host sync)."""
        if getattr(self, "_clock", None) is None or getattr(self, "_clock_steps", None) is None:
            raise RuntimeError("step_clock_read: no clocked region closed by step_clock_end")
        st = self._clock[: self._clock_steps + 1].cpu().tolist()
        self._clock_steps = None
        self._clock = None
        return [(b - a) * 1e-5 for a, b in zip(st, st[1:])]  # 10 ns ticks -> ms

    def _updated(self):
        # the Adam kernel rewrote params AND this handle's kernel-layout weights
        self.model._version += 1
        self._version = self.model._version


# ---------------------------------------------------------------------- standalone kernels
def vtrace(v_tm1, v_t, r_t, discount_t, rho_tm1, lambda_=1.0, clip_rho_threshold=1.0,
           clip_pg_rho_threshold=1.0, stream=None):
    """Batched V-trace on device tensors [B, L] -> (pg_advantage, td_error, q_estimate).
    Same return order as the reference's ``adv, err, _ = batched_vtrace(...)``."""
    ts = [t.contiguous().to(torch.float32) for t in (v_tm1, v_t, r_t, discount_t, rho_tm1)]
    if ts[0].dim() == 1:
        ts = [t.unsqueeze(0) for t in ts]
        squeeze = True
    else:
        squeeze = False
    B, Lh = ts[0].shape
    for t in ts:
        if t.shape != (B, Lh) or t.device.type != "cuda":
            raise ValueError("vtrace inputs must be [B, L] cuda tensors of one shape")
    adv, err, q = (torch.empty_like(ts[0]) for _ in range(3))
    check(_lib.lib().impala_vtrace(*[ptr(t) for t in ts], B, Lh, lambda_, clip_rho_threshold,
                                   clip_pg_rho_threshold, ptr(adv), ptr(err), ptr(q),
                                   stream_ptr(stream)), "impala_vtrace")
    if squeeze:
        return adv[0], err[0], q[0]
    return adv, err, q


def loss_head(logits, values, actions, rewards, discounts, mu, entropy_coeff=0.01, lambda_=1.0,
              clip_rho=1.0, clip_pg_rho=1.0, grad_mode=None, stream=None):
    """Fused loss head (learning.py:144-170) on device tensors; returns a dict.  ``grad_mode``:
    the V-trace gradient semantics (``_lib.VTRACE_GRAD_MODES``, default "sg_advantage")."""
    B, T, A = logits.shape
    dev = logits.device
    f = lambda t: t.contiguous().to(torch.float32)  # noqa: E731
    lg, v, r, g, m = f(logits), f(values), f(rewards), f(discounts), f(mu)
    a = actions.contiguous().to(torch.int64)
    dl = torch.empty_like(lg)
    dv = torch.empty_like(v)
    met = torch.empty(6, dtype=torch.float32, device=dev)
    adv = torch.empty(B, T - 1, dtype=torch.float32, device=dev)
    err, q = torch.empty_like(adv), torch.empty_like(adv)
    rho = torch.empty(B, T, dtype=torch.float32, device=dev)
    check(_lib.lib().impala_loss_head(ptr(lg), ptr(v), ptr(a), ptr(r), ptr(g), ptr(m), B, T, A,
                                      entropy_coeff, lambda_, clip_rho, clip_pg_rho,
                                      _lib.vtrace_grad_mode(grad_mode), ptr(dl),
                                      ptr(dv), ptr(met), ptr(adv), ptr(err), ptr(q), ptr(rho),
                                      stream_ptr(stream)), "impala_loss_head")
    return dict(dlogits=dl, dvalues=dv, metrics=met, adv=adv, err=err, q=q, rho=rho)


def ppo_loss_head(logits, values, actions, targets, mu, entropy_coeff=0.01, clip_coeff=0.1,
                  stream=None):
    """PPO loss head (losses.py:131-155) on device tensors [N, A] / [N]; returns a dict with
    dlogits, dvalues and metrics (loss, entropy, td, pg, kl, ratio, target)."""
    N, A = logits.shape
    f = lambda t: t.contiguous().to(torch.float32)  # noqa: E731
    lg, v, t, m = f(logits), f(values).reshape(N), f(targets).reshape(N), f(mu)
    a = actions.contiguous().to(torch.int64).reshape(N)
    dl = torch.empty_like(lg)
    dv = torch.empty_like(v)
    met = torch.empty(7, dtype=torch.float32, device=lg.device)
    check(_lib.lib().impala_ppo_loss_head(ptr(lg), ptr(v), ptr(a), ptr(t), ptr(m), N, A,
                                          entropy_coeff, clip_coeff, ptr(dl), ptr(dv), ptr(met),
                                          stream_ptr(stream)), "impala_ppo_loss_head")
    return dict(dlogits=dl, dvalues=dv, metrics=met)


def gather_rollouts(fields, idx, stream=None):
    """HIP gather of replay rows: ``[f[idx] for f in fields]`` for device tensors whose first
    dim indexes slots.  ``idx``: a device tensor (impala_gather_rows), or host indices -- a
    numpy array or CPU tensor -- passed in the launch arguments (impala_gather_rows_hidx: no
    index upload on the stream)."""
    import numpy as np
    host = not (isinstance(idx, torch.Tensor) and idx.device.type != "cpu")
    if host:
        idx = np.ascontiguousarray(idx.numpy() if isinstance(idx, torch.Tensor) else idx,
                                   dtype=np.int64)
        n = int(idx.size)
    else:
        idx = idx.to(torch.int64).contiguous()
        n = int(idx.numel())
    outs = [torch.empty((n,) + tuple(f.shape[1:]), dtype=f.dtype, device=f.device) for f in fields]
    k = len(fields)
    src = (C.c_void_p * k)(*[ptr(f) for f in fields])
    dst = (C.c_void_p * k)(*[ptr(o) for o in outs])
    rb = (C.c_size_t * k)(*[f[0].numel() * f.element_size() for f in fields])
    if host:
        check(_lib.lib().impala_gather_rows_hidx(src, dst, rb, k, idx.ctypes.data, n,
                                                 stream_ptr(stream)), "impala_gather_rows_hidx")
    else:
        check(_lib.lib().impala_gather_rows(src, dst, rb, k, ptr(idx), n, stream_ptr(stream)),
              "impala_gather_rows")
    return tuple(outs)
