"""ImpalaBuilder / ImpalaActor — mirror ``agents/impala/builder.py:24-59`` and
``agents/impala/learning.py:29-83`` on the HIP learner.

The actor side (CPU procgen envs, rlmeta loops/RPC) is out of scope;
``ImpalaActor`` keeps the reference's trajectory format so in-process actors can feed the
replay: ``[s (T,3,64,64) u8, a (T,1) i64, r (T,1) f32, discount (T,1) f32, logits (T,A) f32]``
with ``discount = (not done) * gamma`` (``learning.py:77-80``).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from impala_amd.core import Actor, Builder
from impala_amd.learner import ImpalaAdam, ImpalaLearner
from impala_amd.model import AtariPPOModel
from impala_amd.replay import DeviceReplayBuffer, ReplayBuffer


class ImpalaActor(Actor):
    def __init__(self, model, replay_buffer=None, deterministic_policy: bool = False,
                 gamma: float = 0.99, lambda_: float = 0.95, rollout_length: int = 20):
        self._gamma = gamma
        self._lambda = lambda_  # stored, unused — as the reference
        self._deterministic_policy = torch.tensor([deterministic_policy])
        self._model = model
        self._replay_buffer = replay_buffer
        self._rollout_length = rollout_length
        self._trajectory: List[tuple] = []
        self._last_transition = None

    def act(self, timestep):
        obs = timestep.observation if hasattr(timestep, "observation") else timestep[0]
        action, logpi, v = self._model.act(obs, self._deterministic_policy)
        return action, {"logpi": logpi, "v": v}

    async def async_act(self, timestep):
        return self.act(timestep)

    async def async_observe_init(self, timestep) -> None:
        if self._replay_buffer is None:
            return
        self._last_transition = timestep

    def observe(self, action, next_timestep) -> None:
        if self._replay_buffer is None:
            return
        obs = self._last_transition[0]
        act, info = action
        next_obs, reward, done = next_timestep[0], next_timestep[1], next_timestep[2]
        self._trajectory.append((torch.as_tensor(obs), torch.as_tensor(act).reshape(1),
                                 torch.as_tensor(reward, dtype=torch.float32).reshape(1),
                                 torch.as_tensor(done).reshape(1),
                                 torch.as_tensor(info["logpi"]).reshape(-1)))
        self._last_transition = next_timestep
        if len(self._trajectory) == self._rollout_length:
            self.update()

    async def async_observe(self, action, next_timestep) -> None:
        self.observe(action, next_timestep)

    def update(self) -> None:
        if self._replay_buffer is None or not self._trajectory:
            return
        self._replay_buffer.append(self._make_replay())

    async def async_update(self) -> None:
        self.update()

    def _make_replay(self):  # learning.py:77-80
        s, a, r, d, pi_ref = (torch.stack(x) for x in zip(*self._trajectory))
        self._trajectory = []
        discount_t = torch.logical_not(d) * self._gamma
        return [s, a.to(torch.int64), r, discount_t.to(torch.float32), pi_ref.to(torch.float32)]


class ImpalaActorFactory:
    def __init__(self, model, rb, deterministic: bool, rollout_length: int = 20):
        self._args = (model, rb, deterministic)
        self._rollout_length = rollout_length

    def __call__(self, index: int) -> Actor:
        m, rb, det = self._args
        return ImpalaActor(m, rb, det, rollout_length=self._rollout_length)


class ImpalaBuilder(Builder):
    def __init__(self, cfg):
        self.cfg = cfg
        self._learner_model = None
        self._actor_model = None

    def _learner_cfg(self, key, default):
        lc = self.cfg.get("learner", {}) if isinstance(self.cfg, dict) else getattr(self.cfg, "learner", {})
        return lc.get(key, default) if lc else default

    def make_replay(self):  # builder.py:30-36
        cap = self.cfg.agent.replay_buffer_size
        seed = self.cfg.training.seed
        kind = self._learner_cfg("replay", "device")
        A = self._learner_model.action_dim if self._learner_model is not None else 15
        if kind == "device" and torch.cuda.is_available():
            dev = self.cfg.distributed.train_device
            return DeviceReplayBuffer(cap, self.cfg.agent.rollout_length, A, device=dev, seed=seed)
        return ReplayBuffer(cap, seed=seed)

    def make_actor(self, model, rb=None, deterministic: bool = False):  # builder.py:38-40
        # the reference always builds stochastic actors (its `deterministic` is ignored)
        return ImpalaActorFactory(model, rb, False, self.cfg.agent.rollout_length)

    def make_learner(self, model, rb):  # builder.py:42-49
        opt = ImpalaAdam(lr=float(self.cfg.agent.optimizer.lr),
                         eps=float(self.cfg.agent.optimizer.eps))
        kw = {}
        if self._learner_cfg("honour_yaml_hparams", False):
            kw = dict(max_grad_norm=float(self.cfg.agent.max_grad_norm),
                      entropy_coeff=float(self.cfg.agent.entropy_cost),
                      model_push_period=int(self.cfg.agent.model_push_period))
        pg = None
        ws = int(self._learner_cfg("world_size", 1))
        if ws > 1:
            import torch.distributed as dist
            pg = dist.group.WORLD
        return ImpalaLearner(self._learner_model if model is None else model, rb, opt,
                             batch_size=self.cfg.agent.batch_size,
                             learning_starts=self.cfg.agent.learning_starts,
                             rollout_length=self.cfg.agent.rollout_length,
                             dtype=self._learner_cfg("dtype", None), process_group=pg,
                             world_size=ws,
                             vtrace_grad_mode=self._learner_cfg("vtrace_grad_mode", None),
                             prefetch=min(2, max(0, int(self.cfg.training.get("prefetch", 2) or 0))),
                             **kw)

    def make_network(self, env_spec=None):  # builder.py:51-59
        obs_shape, n_act = (3, 64, 64), 15
        if env_spec is not None:
            obs_shape = tuple(env_spec.observation_space.shape)
            n_act = int(env_spec.action_space.n)
        model = AtariPPOModel(obs_shape, n_act, device=self.cfg.distributed.train_device,
                              dtype=self._learner_cfg("dtype", "fp32"))
        self._learner_model = model
        actor_model = model.clone_to(self.cfg.distributed.infer_device)
        self._actor_model = actor_model
        model.downstream = actor_model  # push() publishes the learner weights here
        return model


class PPOBuilder(Builder):
    """agents/ppo/builder.py:24-53 on the HIP learner."""

    def __init__(self, cfg):
        self.cfg = cfg
        self._learner_model = None
        self._actor_model = None

    def make_replay(self):  # builder.py:30-36: CircularBuffer(size, torch.cat) + UniformSampler
        return ReplayBuffer(self.cfg.agent.replay_buffer_size, seed=self.cfg.training.seed)

    def make_actor(self, model, rb=None, deterministic: bool = False):  # builder.py:38-39
        # PPOActorRemote._make_replay (agents/ppo/learning.py:65-69) references an undefined
        # `values`; the actor side is out of scope here
        raise NotImplementedError("PPO actors are not part of the MI355X learner path")

    def make_learner(self, model, rb):  # builder.py:41-44: PPOLearner(model, rb, optimizer)
        from impala_amd.ppo import PPOLearner
        opt = ImpalaAdam(lr=float(self.cfg.agent.optimizer.lr),
                         eps=float(self.cfg.agent.optimizer.eps))
        dtype = None
        lc = self.cfg.get("learner", {}) if isinstance(self.cfg, dict) else getattr(self.cfg, "learner", {})
        if lc:
            dtype = lc.get("dtype", None)
        # the reference passes no cfg to the learner: constructor defaults (batch 256, clip 0.5,
        # entropy 0.01, push period 8) apply, whatever conf/agent/ppo.yaml says
        return PPOLearner(self._learner_model if model is None else model, rb, opt, dtype=dtype)

    def make_network(self, env_spec=None):  # builder.py:46-53
        obs_shape, n_act = (3, 64, 64), 15
        if env_spec is not None:
            obs_shape = tuple(env_spec.observation_space.shape)
            n_act = int(env_spec.action_space.n)
        model = AtariPPOModel(obs_shape, n_act, device=self.cfg.distributed.train_device,
                              dtype="fp32")
        self._learner_model = model
        self._actor_model = model.clone_to(self.cfg.distributed.infer_device)
        model.downstream = self._actor_model
        return model
