"""Plugin ABCs of the reference (``agents/core.py:12-91``), without the rlmeta dependency.

``Learner.connect`` keeps the reference behaviour: every attribute that has a ``connect``
method and is marked remote (``_is_remote = True``) is connected (rlmeta ``Remote`` objects in
the reference, ``agents/core.py:59-63``).
"""
from __future__ import annotations

import abc
from typing import Optional


def _connect_remotes(obj) -> None:
    for name in dir(obj):
        try:
            attr = getattr(obj, name)
        except Exception:
            continue
        if getattr(attr, "_is_remote", False) and callable(getattr(attr, "connect", None)):
            attr.connect()


class Agent(abc.ABC):  # agents/core.py:12-20
    @abc.abstractmethod
    def train(self, num_steps: int) -> None:
        ...

    @abc.abstractmethod
    def eval(self, num_episodes: int, keep_training_loops: bool) -> None:
        ...


class Actor(abc.ABC):  # agents/core.py:23-46
    def connect(self) -> None:
        _connect_remotes(self)

    @abc.abstractmethod
    async def async_act(self, timestep):
        ...

    @abc.abstractmethod
    async def async_observe_init(self, timestep) -> None:
        ...

    @abc.abstractmethod
    async def async_observe(self, action, next_timestep) -> None:
        ...

    @abc.abstractmethod
    async def async_update(self) -> None:
        ...


class Learner(abc.ABC):  # agents/core.py:49-65
    _step_counter: int
    can_train: bool = False

    @abc.abstractmethod
    def train_step(self):
        ...

    @abc.abstractmethod
    def prepare(self):
        ...

    def connect(self) -> None:
        _connect_remotes(self)


class Builder(abc.ABC):  # agents/core.py:68-91
    @abc.abstractmethod
    def make_replay(self):
        ...

    @abc.abstractmethod
    def make_actor(self, model, rb=None, deterministic: bool = False):
        ...

    @abc.abstractmethod
    def make_learner(self, model, rb):
        ...

    @abc.abstractmethod
    def make_network(self, env_spec):
        ...

    @property
    def actor_model(self):
        return getattr(self, "_actor_model", None)

    @property
    def learner_model(self):
        return getattr(self, "_learner_model", None)
