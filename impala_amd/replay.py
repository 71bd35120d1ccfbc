"""Rollout storage feeding the learner.

Reference: ``agents/impala/builder.py:30-36`` builds ``ReplayBuffer(CircularBuffer(1000),
UniformSampler())``; actors ``async_append`` one trajectory ``[s, a, r, discount, logits]``
(``agents/impala/learning.py:71-80``); the learner calls ``warm_up(learning_starts)`` and
``sample(batch_size) -> (keys, batch, probs)`` (``learning.py:116-121``).

Two implementations with that interface:

* ``ReplayBuffer``        host memory, returns the reference's list-of-trajectories batch.
* ``DeviceReplayBuffer``  MI355X-first: the circular store lives in HBM (1000 x 247 KB =
  247 MB of 288 GB); an appended trajectory is written into a pinned-host staging ring and
  copied to its HBM slot with an async H2D on a side stream, so each trajectory crosses PCIe
  once however often it is replayed; ``sample`` gathers B slots on the device with the HIP
  gather kernel and returns the collated ``(B,T,...)`` batch already resident in HBM.
"""
from __future__ import annotations

import threading
import time
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


class ReplayBuffer:
    """CircularBuffer + UniformSampler semantics on the host (reference-compatible)."""

    def __init__(self, capacity: int = 1000, seed: Optional[int] = None):
        self.capacity = int(capacity)
        self._data: List[Optional[list]] = [None] * self.capacity
        self._keys = np.zeros(self.capacity, dtype=np.int64)
        self._next_key = 0
        self._size = 0
        self._cursor = 0
        self._rng = np.random.default_rng(seed)
        self._cv = threading.Condition()

    def __len__(self):
        return self._size

    def reset(self, seed: Optional[int] = None):
        self._rng = np.random.default_rng(seed)

    def append(self, item: Sequence[torch.Tensor]) -> int:
        with self._cv:
            slot = self._cursor
            self._data[slot] = list(item)
            key = self._next_key
            self._keys[slot] = key
            self._next_key += 1
            self._cursor = (self._cursor + 1) % self.capacity
            self._size = min(self._size + 1, self.capacity)
            self._cv.notify_all()
            return key

    def extend(self, items) -> List[int]:
        return [self.append(x) for x in items]

    async def async_append(self, item):
        return self.append(item)

    def warm_up(self, learning_starts: Optional[int] = None, timeout: float = 240.0) -> None:
        """Block until ``learning_starts`` items are stored (rlmeta ReplayBuffer.warm_up)."""
        if not learning_starts:
            return
        need = min(int(learning_starts), self.capacity)
        deadline = time.monotonic() + timeout
        with self._cv:
            while self._size < need:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError(f"replay warm_up: {self._size}/{need} after {timeout}s")
                self._cv.wait(left)

    def _indices(self, batch_size: int) -> np.ndarray:
        if self._size == 0:
            raise RuntimeError("sample from an empty replay buffer")
        replace = batch_size > self._size
        return self._rng.choice(self._size, size=batch_size, replace=replace)

    def sample(self, batch_size: int):
        with self._cv:
            idx = self._indices(batch_size)
            batch = [self._data[i] for i in idx]
            keys = self._keys[idx].copy()
        probs = np.full(batch_size, 1.0 / self._size)
        return keys, batch, probs


class DeviceReplayBuffer(ReplayBuffer):
    """HBM-resident circular rollout store with pinned-host staging (see module doc)."""

    # the most entries the page-locked index ring grows to (_indices_to_device) before sample()
    # waits for the oldest one's copy
    _IDX_RING_MAX = 64

    def __init__(self, capacity: int = 1000, rollout_length: int = 20, num_actions: int = 15,
                 device="cuda", seed: Optional[int] = None, staging_slots: int = 64):
        super().__init__(capacity, seed)
        self.device = torch.device(device)
        C, T, A = self.capacity, int(rollout_length), int(num_actions)
        self.T, self.A = T, A
        d = self.device
        self.obs = torch.empty(C, T, 3, 64, 64, dtype=torch.uint8, device=d)
        self.act = torch.zeros(C, T, dtype=torch.int64, device=d)
        self.rew = torch.zeros(C, T, dtype=torch.float32, device=d)
        self.disc = torch.zeros(C, T, dtype=torch.float32, device=d)
        self.mu = torch.zeros(C, T, A, dtype=torch.float32, device=d)
        S = int(staging_slots)
        pin = torch.cuda.is_available()
        self._st_obs = torch.empty(S, T, 3, 64, 64, dtype=torch.uint8, pin_memory=pin)
        self._st_small = torch.empty(S, T, 3 + A, dtype=torch.float32, pin_memory=pin)
        self._st_act = torch.empty(S, T, dtype=torch.int64, pin_memory=pin)
        self._st_events = [None] * S
        self._st_next = 0
        self._stream = torch.cuda.Stream(device=d)
        self._pending: List[torch.cuda.Event] = []
        # the last gather enqueued by sample(): an append must not overwrite a slot that a
        # queued gather still reads (gathers run in order on the learner's stream, so waiting
        # for the latest one covers every earlier read)
        self._last_read: Optional[torch.cuda.Event] = None
        # page-locked ring for the sampled slot indices: their H2D is a true asynchronous copy
        # (from pageable memory it would wait behind the learner stream's queued work while
        # sample() holds the lock); a ring entry is reused after its copy has run.  It starts
        # at 4 entries and grows when the learner's stream runs further ahead than that
        self._idx_buf: List[Optional[torch.Tensor]] = [None] * 4
        self._idx_ev: List[Optional[torch.cuda.Event]] = [None] * 4
        self._idx_next = 0

    def append(self, item: Sequence[torch.Tensor]) -> int:
        s, a, r, g, mu = item
        T = self.T
        with self._cv:
            j = self._st_next
            self._st_next = (j + 1) % len(self._st_events)
            ev = self._st_events[j]
            if ev is not None:
                ev.synchronize()  # staging slot reuse: its previous H2D has finished
            self._st_obs[j].copy_(s.reshape(T, 3, 64, 64))
            self._st_act[j].copy_(a.reshape(T))
            sm = self._st_small[j]
            sm[:, 0].copy_(r.reshape(T))
            sm[:, 1].copy_(g.reshape(T))
            sm[:, 3:].copy_(mu.reshape(T, self.A))
            slot = self._cursor
            with torch.cuda.stream(self._stream):
                if self._last_read is not None:
                    self._stream.wait_event(self._last_read)
                self.obs[slot].copy_(self._st_obs[j], non_blocking=True)
                self.act[slot].copy_(self._st_act[j], non_blocking=True)
                small = sm.to(self.device, non_blocking=True)
                self.rew[slot].copy_(small[:, 0])
                self.disc[slot].copy_(small[:, 1])
                self.mu[slot].copy_(small[:, 3:])
                ev = torch.cuda.Event()
                ev.record(self._stream)
            self._st_events[j] = ev
            self._pending.append(ev)
            key = self._next_key
            self._keys[slot] = key
            self._next_key += 1
            self._cursor = (slot + 1) % self.capacity
            self._size = min(self._size + 1, self.capacity)
            self._cv.notify_all()
            return key

    def _indices_to_device(self, idx: np.ndarray, stream) -> torch.Tensor:
        """Slot indices -> a device int64 tensor, copied on `stream` from a page-locked ring
        entry (asynchronous: nothing here waits for the stream's queued work).  Called with
        ``_cv`` held, so it never blocks on the device: when the next entry's previous copy is
        still queued (the learner runs more than the ring's length ahead), the ring grows by a
        fresh entry instead, up to ``_IDX_RING_MAX`` entries."""
        k = self._idx_next
        ev = self._idx_ev[k]
        if ev is not None and not ev.query():
            if len(self._idx_buf) < self._IDX_RING_MAX:
                # the busy entry (the oldest) moves one place on and stays next in line
                self._idx_buf.insert(k, None)
                self._idx_ev.insert(k, None)
                ev = None
            else:  # bounded: only a learner thousands of steps ahead reaches this
                ev.synchronize()
        self._idx_next = (k + 1) % len(self._idx_buf)
        n = len(idx)
        buf = self._idx_buf[k]
        if buf is None or buf.numel() < n:
            buf = torch.empty(n, dtype=torch.int64, pin_memory=torch.cuda.is_available())
            self._idx_buf[k] = buf
        host = buf[:n]
        host.copy_(torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64)))
        with torch.cuda.stream(stream):
            dev = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        self._idx_ev[k] = ev
        return dev

    def sample(self, batch_size: int, stream=None):
        """-> (keys, (obs, act, rew, disc, mu) collated on the device, probs).

        The lock is held from picking the slots until the gather's completion event is
        published as ``_last_read`` (both are asynchronous enqueues, so this is cheap): an
        append either lands before -- its H2D event is among the ``pending`` the gather waits
        for -- or after, and then its copy waits for this gather.  No append can slip between
        the two and overwrite a slot the gather is reading."""
        from impala_amd.engine import gather_rollouts
        cur = torch.cuda.current_stream(self.device) if stream is None else stream
        with self._cv:
            idx = self._indices(batch_size)
            keys = self._keys[idx].copy()
            pending, self._pending = self._pending, []
            for ev in pending:  # the learner's stream waits for every staged H2D
                cur.wait_event(ev)
            idx_t = self._indices_to_device(idx, cur)
            batch = gather_rollouts((self.obs, self.act, self.rew, self.disc, self.mu), idx_t,
                                    stream)
            read = torch.cuda.Event()
            read.record(cur)
            self._last_read = read
            size = self._size
        probs = np.full(batch_size, 1.0 / size)
        return keys, batch, probs
