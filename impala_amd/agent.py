"""DistributedAgent — the learner-side driver of ``agents/distributed_agent.py:15-59``.

``train(num_steps)``: ``learner.prepare()`` then ``learner.train_step()`` x num_steps, metric
aggregation and a log call every 100 steps, as the reference.  Improvement kept optional:
``sync_every`` > 1 converts the device metrics to floats only every k steps (the reference's
``float(v)`` per step is a host-device sync per step).  The rlmeta controller / eval loops
are out of scope: a controller object with the reference's interface may be passed in.
"""
from __future__ import annotations

import time
from collections import defaultdict
from typing import Callable, Dict, Optional

from impala_amd.core import Agent, Learner


class StatsDict:
    """Minimal rlmeta StatsDict: running mean/count/min/max per key."""

    def __init__(self):
        self._d = defaultdict(lambda: {"sum": 0.0, "count": 0, "min": float("inf"),
                                       "max": float("-inf")})

    def extend(self, kv: Dict[str, float]):
        for k, v in kv.items():
            s = self._d[k]
            s["sum"] += v
            s["count"] += 1
            s["min"] = min(s["min"], v)
            s["max"] = max(s["max"], v)

    def dict(self):
        return {k: {"mean": s["sum"] / max(s["count"], 1), "count": s["count"], "min": s["min"],
                    "max": s["max"]} for k, s in self._d.items()}


class DistributedAgent(Agent):
    def __init__(self, controller, learner: Learner, writer: Optional[Callable] = None,
                 sync_every: int = 1):
        self._controller = controller
        self._learner = learner
        self._writer = writer
        self._stats_dict = StatsDict()
        self._start_time = time.perf_counter()
        self._sync_every = max(1, int(sync_every))

    def set_phase(self, phase=None):
        if self._controller is not None:
            self._controller.set_phase(phase=phase)

    def _log(self, d):
        if self._writer is not None:
            self._writer(d)

    def train(self, num_steps: int) -> int:
        if self._controller is not None:
            self._controller.set_phase("TRAIN")
        self._learner.prepare()
        pending = []
        for local_steps in range(num_steps):
            metrics = self._learner.train_step()
            pending.append(metrics)
            if len(pending) >= self._sync_every or local_steps == num_steps - 1:
                for m in pending:
                    self._stats_dict.extend({k: float(v) for k, v in m.items()})
                pending = []
            if local_steps % 100 == 0:
                self._log({k: float(v) for k, v in metrics.items()})
        return num_steps

    def eval(self, num_episodes: Optional[int] = None, keep_training_loops: bool = True):
        if self._controller is None:
            raise NotImplementedError("evaluation needs the actor/controller side (out of scope)")
        raise NotImplementedError

    def connect(self):
        if self._controller is not None and hasattr(self._controller, "connect"):
            self._controller.connect()
        self._learner.connect()

    @property
    def stats(self):
        return self._stats_dict
