"""DistributedAgent — the learner-side driver of ``agents/distributed_agent.py:15-68``.

``train(num_steps)``: ``controller.set_phase(Phase.TRAIN)``, ``learner.prepare()``, then
``learner.train_step()`` x num_steps with every metric folded into the stats dict and a log
call every 100 steps; afterwards the controller's TRAIN episode statistics give
``total_samples`` (mean episode length x episode count), logged with
``debug/samples_per_second`` and the ``train_envs/*`` means, and returned -- as the reference.
``eval`` runs the reference's controller protocol.  The device metrics of a step reach the host
in one copy (the reference's ``float(v)`` per value is one synchronising copy each), and the
optional ``sync_every`` > 1 converts them only every k steps, all k in one copy.  The rlmeta controller itself is out of scope: any object with
its interface (set_phase, reset_phase, count, stats, connect) may be passed in.
"""
from __future__ import annotations

import enum
import time
from collections import defaultdict
from typing import Callable, Dict, List, Optional

import torch

from impala_amd.core import Agent, Learner


class Phase(enum.IntFlag):
    """rlmeta.core.controller.Phase (the controller's phase flags)."""
    NONE = 0
    TRAIN = 1
    EVAL = 2
    BOTH = 3


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


def _host_floats(pending: List[Dict]) -> List[Dict[str, float]]:
    """``{k: float(v)}`` for every metrics dict of ``pending`` (distributed_agent.py:31), with
    one device-to-host copy for all of them: device scalars that are views of one metrics
    vector (ImpalaLearner._train_step) are read from a single stacked copy of those vectors,
    instead of one synchronising copy per value.  Anything else goes through float(v)."""
    return _to_dicts(*_read_values(pending))


def _read_values(pending: List[Dict]):
    """The synchronising half of _host_floats: the one device-to-host copy -> (pending, host
    rows by base id); _to_dicts builds the float dicts from them later.  Metrics dicts that
    carry their step's host row (ImpalaLearner's StepMetrics) are read from it as soon as the
    step's Adam kernel has set the row's ready word (HostMetrics.values), with no copy enqueued
    behind the work queued since."""
    host = {}
    rest = []
    for m in pending:
        hm = getattr(m, "host", None)
        vals = hm.values() if hm is not None else None
        base = next(iter(m.values()))._base if vals is not None and m else None
        if vals is not None and base is not None:
            host[id(base)] = (base, vals)
        else:
            rest.append(m)
    if not rest:
        return pending, host
    host.update(_copy_values(rest))
    return pending, host


def _copy_values(pending: List[Dict]):
    bases = {}
    for m in pending:
        for v in m.values():
            if isinstance(v, torch.Tensor) and v.dim() == 0 and v._base is not None \
                    and v.device.type != "cpu":
                b = v._base
                if b.dim() == 1 and b.is_contiguous():
                    bases.setdefault(id(b), b)
    host = {}
    if bases:
        bl = list(bases.values())
        if len(bl) == 1:  # one step's vector: copy it as it is (no stacking kernel)
            rows = [bl[0].cpu().tolist()]
        elif len({(b.numel(), b.dtype, b.device) for b in bl}) == 1:
            rows = torch.stack(bl).cpu().tolist()
        else:
            rows = [b.cpu().tolist() for b in bl]
        host = {id(b): (b, r) for b, r in zip(bl, rows)}
    return host


def _to_dicts(pending: List[Dict], host) -> List[Dict[str, float]]:
    out = []
    for m in pending:
        d = {}
        for k, v in m.items():
            hb = host.get(id(v._base)) if isinstance(v, torch.Tensor) and v._base is not None else None
            if hb is not None:
                b, r = hb
                d[k] = float(r[v.storage_offset() - b.storage_offset()])
            else:
                d[k] = float(v)
        out.append(d)
    return out


class DistributedAgent(Agent):
    def __init__(self, controller, learner: Learner, writer=None, sync_every: int = 1):
        self._controller = controller
        self._learner = learner
        self._writer = writer
        self._stats_dict = StatsDict()
        self._start_time = time.perf_counter()
        self._sync_every = max(1, int(sync_every))

    def set_phase(self, phase=Phase.TRAIN):
        if self._controller is not None:
            self._controller.set_phase(phase=phase)

    def _log(self, d):
        """The reference logs through ``writer.run.log`` (a wandb run); a plain callable works
        too."""
        w = self._writer
        if w is None:
            return
        run = getattr(w, "run", None)
        if run is not None and hasattr(run, "log"):
            run.log(d)
        elif callable(w):
            w(d)

    def train(self, num_steps: int):
        if self._controller is not None:
            self._controller.set_phase(Phase.TRAIN)
        self._learner.prepare()
        pending = []
        read = None  # values read at the last sync, turned into floats after the next enqueue
        for local_steps in range(num_steps):
            metrics = self._learner.train_step()
            if read is not None:
                # the previous sync's floats, booked now that this step is enqueued: the device
                # then runs while the host builds them (the values and order are unchanged)
                for d in _to_dicts(*read):
                    self._stats_dict.extend(d)
                read = None
            pending.append(metrics)
            if len(pending) >= self._sync_every or local_steps == num_steps - 1:
                read = _read_values(pending)  # the sync: every pending value on the host
                pending = []
            if local_steps % 100 == 0:
                just_read = read is not None and read[0][-1] is metrics
                self._log(_to_dicts(*read)[-1] if just_read else _host_floats([metrics])[0])
        if read is not None:
            for d in _to_dicts(*read):
                self._stats_dict.extend(d)
        if self._controller is None:
            # no actor side to ask: the frames this learner consumed
            total_samples = float(num_steps * getattr(self._learner, "samples_per_step", 0))
        else:
            remote = self._controller.stats(Phase.TRAIN).dict()
            total_samples = remote["episode_length"]["mean"] * remote["episode_length"]["count"]
        delta = total_samples / (time.perf_counter() - self._start_time)
        self._log({"debug/total_samples": total_samples})
        if self._controller is not None:
            self._log({f"train_envs/{k.replace('/', '_')}": v["mean"] for k, v in remote.items()})
        self._log({"debug/samples_per_second": delta})
        return total_samples

    def eval(self, num_episodes: Optional[int] = None, keep_training_loops: bool = True):
        """distributed_agent.py:44-56: switch the controller to EVAL (or BOTH), wait until
        ``num_episodes`` evaluation episodes are counted, log and return their stats."""
        if self._controller is None:
            raise RuntimeError("eval needs a controller (the actor side is out of scope)")
        self._controller.set_phase(Phase.BOTH if keep_training_loops else Phase.EVAL)
        self._controller.reset_phase(Phase.EVAL, limit=num_episodes)
        while self._controller.count(Phase.EVAL) < num_episodes:
            time.sleep(1)
        stats = self._controller.stats(Phase.EVAL)
        self._log({f"eval_envs/{k.replace('/', '_')}": v["mean"] for k, v in stats.dict().items()})
        return stats

    def connect(self):
        if self._controller is not None and hasattr(self._controller, "connect"):
            self._controller.connect()
        self._learner.connect()

    @property
    def stats(self):
        return self._stats_dict
