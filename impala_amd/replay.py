"""Rollout storage feeding the learner.

Reference: ``agents/impala/builder.py:30-36`` builds ``ReplayBuffer(CircularBuffer(1000),
UniformSampler())``; actors ``async_append`` one trajectory ``[s, a, r, discount, logits]``
(``agents/impala/learning.py:71-80``); the learner calls ``warm_up(learning_starts)`` and
``sample(batch_size) -> (keys, batch, probs)`` (``learning.py:116-121``).

Two implementations with that interface:

* ``ReplayBuffer``        host memory, returns the reference's list-of-trajectories batch; the
  batch also carries the rows' host addresses, so the learner stages them with
  ``impala_stage_rows`` (the library's thread pool collates them into a page-locked slot).
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


def _row_info(item):
    """(host addresses, (dtypes, byte sizes)) of a trajectory's fields when every field is a
    contiguous CPU tensor, else None: what impala_stage_rows needs to read the rows in place."""
    if not all(isinstance(t, torch.Tensor) and t.device.type == "cpu" and t.is_contiguous()
               for t in item):
        return None
    return ([t.data_ptr() for t in item],
            (tuple(t.dtype for t in item), tuple(t.numel() * t.element_size() for t in item)))


class RowBatch(list):
    """The list of B trajectories a replay's ``sample`` returns (the reference's batch format),
    plus, when every sampled trajectory's fields are contiguous host tensors of one layout,
    ``row_ptrs`` -- per field the B rows' host addresses (numpy uint64) -- and ``row_key`` --
    the fields' (dtypes, byte sizes) -- for ``impala_stage_rows``.  The rows are the replay's
    own tensors: an append replaces a slot's list and never writes into a stored tensor, so a
    consumer that keeps the batch keeps its rows."""
    row_ptrs = None
    row_key = None


class ReplayBuffer:
    """CircularBuffer + UniformSampler semantics on the host (reference-compatible)."""

    def __init__(self, capacity: int = 1000, seed: Optional[int] = None):
        self.capacity = int(capacity)
        self._data: List[Optional[list]] = [None] * self.capacity
        # per slot: the fields' host addresses and layout key (_row_info), when known
        self._ptr_tab = np.zeros((self.capacity, 5), dtype=np.uint64)
        self._row_keys: List[Optional[tuple]] = [None] * self.capacity
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
            info = _row_info(self._data[slot]) if len(item) == 5 else None
            if info is None:
                self._row_keys[slot] = None
            else:
                self._ptr_tab[slot] = info[0]
                self._row_keys[slot] = info[1]
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
            batch = RowBatch(self._data[i] for i in idx)
            rk = {self._row_keys[i] for i in idx}
            if len(rk) == 1 and None not in rk:
                batch.row_key = rk.pop()
                batch.row_ptrs = tuple(np.ascontiguousarray(self._ptr_tab[idx, f]) for f in range(5))
            keys = self._keys[idx].copy()
        probs = np.full(batch_size, 1.0 / self._size)
        return keys, batch, probs


class RowSample:
    """DeviceReplayBuffer.sample_rows: the sampled slots (host int64), read in place."""
    __slots__ = ("replay", "idx")

    def __init__(self, replay, idx):
        self.replay, self.idx = replay, np.ascontiguousarray(idx, dtype=np.int64)

    def gather(self, stream=None):
        """The rows collated on the device (what ``sample`` returns), for a caller that cannot
        read them in place."""
        from impala_amd.engine import gather_rollouts
        return self.replay.read_rows(self, lambda fields, idx, st: gather_rollouts(fields, idx, st),
                                     stream)


class DeviceReplayBuffer(ReplayBuffer):
    """HBM-resident circular rollout store with pinned-host staging (see module doc)."""

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
        # An append must not overwrite a slot that a queued gather still reads.  sample() numbers
        # its gathers (_gen) and marks the slots each one reads (_slot_gen); an append into a
        # slot read by a gather not yet fenced records ONE event on the gathers' stream (it
        # follows every gather enqueued so far) and its copy waits for it; later appends into
        # slots read before that fence wait for the same event.  So the learner's stream gets
        # at most one event per sample, and none while nothing is appended.
        self._read_stream = None
        self._gen = 0
        self._slot_gen = np.zeros(self.capacity, dtype=np.int64)
        self._fence_gen = 0
        self._fence_ev: Optional[torch.cuda.Event] = None

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
                read_gen = int(self._slot_gen[slot])
                if read_gen > self._fence_gen:  # read by a gather not yet fenced
                    fence = torch.cuda.Event()
                    fence.record(self._read_stream)
                    self._fence_ev, self._fence_gen = fence, self._gen
                if read_gen > 0:
                    self._stream.wait_event(self._fence_ev)
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

    def sample_rows(self, batch_size: int):
        """-> (keys, RowSample, probs): the same draw as ``sample`` (the same generator call),
        without a gather -- the step reads the sampled slots in place
        (``read_rows`` / Engine.train_step_rows).  A slot overwritten between this call and
        the step is read with its new trajectory (the draw is of slots)."""
        with self._cv:
            idx = self._indices(batch_size)
            keys = self._keys[idx].copy()
            size = self._size
        return keys, RowSample(self, idx), np.full(batch_size, 1.0 / size)

    @property
    def fields(self):
        """The ring's five arrays (obs, actions, rewards, discounts, behaviour logits)."""
        return (self.obs, self.act, self.rew, self.disc, self.mu)

    def read_rows(self, rs: "RowSample", enqueue, stream=None):
        """Run ``enqueue(fields, idx, stream)`` -- which enqueues work reading the ring slots
        ``rs.idx`` on ``stream`` (the current stream when None) -- under the lock ``append``
        takes, after that stream waits for every staged append; then mark the slots as read by
        it (the fence an append into them waits for, as for a gather in ``sample``)."""
        cur = torch.cuda.current_stream(self.device) if stream is None else stream
        with self._cv:
            if self._pending:
                pending, self._pending = self._pending, []
                for ev in pending:
                    cur.wait_event(ev)
            out = enqueue(self.fields, rs.idx, cur)
            self._read_stream = cur
            self._gen += 1
            self._slot_gen[rs.idx] = self._gen
        return out

    def sample(self, batch_size: int, stream=None):
        """-> (keys, (obs, act, rew, disc, mu) collated on the device, probs).

        The sampled slot indices travel in the gather launch's own arguments
        (impala_gather_rows_hidx), so the learner's stream gets the gather and nothing else: no
        index upload, no event, and nothing here ever waits on the device.  The lock is held
        from picking the slots until the gather is enqueued and its slots marked with its
        generation: an append either lands before -- its H2D event is among the ``pending``
        the gather waits for -- or after, and then its copy waits for a fence event recorded
        behind this gather (see ``__init__``).  No append can slip between the two and
        overwrite a slot the gather is reading."""
        from impala_amd.engine import gather_rollouts
        cur = torch.cuda.current_stream(self.device) if stream is None else stream
        with self._cv:
            idx = self._indices(batch_size)
            keys = self._keys[idx].copy()
            pending, self._pending = self._pending, []
            for ev in pending:  # the learner's stream waits for every staged H2D
                cur.wait_event(ev)
            batch = gather_rollouts((self.obs, self.act, self.rew, self.disc, self.mu), idx,
                                    stream)
            self._read_stream = cur
            self._gen += 1
            self._slot_gen[idx] = self._gen
            size = self._size
        probs = np.full(batch_size, 1.0 / size)
        return keys, batch, probs
