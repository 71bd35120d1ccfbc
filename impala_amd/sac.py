"""SAC on MI355X — drop-in for ``models/sac_model.py``, ``agents/sac/learning.py`` and
``agents/sac/builder.py`` (BASELINE config 5).

* ``SoftActor`` / ``SoftCritic``: the reference modules' parameter names, shapes and init
  (``layer_init_uniform``, scale 0.33, built in the reference's construction order so a given
  torch seed gives the same weights), with every parameter a VIEW into one flat fp32 buffer
  per network (``flat``, ``flat_grad``; the target critic in ``target_flat``; ``log_alpha`` in
  ``la_buf[0]``).  ``forward`` / ``act`` / ``policy`` / ``target`` run on the HIP path only.
* ``SACEngine``: one ``sac_learner`` handle (``include/sac_hip.h``) bound to those buffers plus
  the optimizer moments and the target actor.
* ``SACLearner``: ``agents/sac/learning.py:93-193`` — same constructor, ``prepare`` /
  ``train_step`` behaviour and metric keys.  The critic step, actor step, alpha step and both
  Polyak updates are ONE ``sac_train_step`` call (a replayed hipGraph of 22 launches).
* ``DeviceTransitionReplay``: ``ReplayBuffer(CircularBuffer(size), UniformSampler())`` of
  ``builder.py:30-36`` with the store in HBM and sampling + gather on the device
  (``sac_sample``): "replay-buffer GPU sampling" of BASELINE config 5.
* ``SACActor`` / ``SACBuilder``: ``SACActorRemote`` (``learning.py:15-57``) and ``SACBuilder``.
"""
from __future__ import annotations

import copy
import ctypes as C
import math
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

from impala_amd import _lib
from impala_amd.core import Actor, Builder, Learner
from impala_amd.model import picklable_state, rebind_views

HIDDEN = 256
LOG_STD_MAX = 2
LOG_STD_MIN = -5


def _prod(shape) -> int:
    return int(np.prod(shape)) if isinstance(shape, (tuple, list)) else int(shape)


def actor_specs(D: int, K: int) -> List[Tuple[str, Tuple[int, ...]]]:
    """SoftActor.parameters() order (sac_model.py:92-139,181-188)."""
    return [("actor.body.body.0.weight", (HIDDEN, D)), ("actor.body.body.0.bias", (HIDDEN,)),
            ("actor.body.body.2.weight", (HIDDEN, HIDDEN)), ("actor.body.body.2.bias", (HIDDEN,)),
            ("actor.head.fc_mean.weight", (K, HIDDEN)), ("actor.head.fc_mean.bias", (K,)),
            ("actor.head.fc_logstd.weight", (K, HIDDEN)), ("actor.head.fc_logstd.bias", (K,))]


def critic_specs(prefix: str, D: int, K: int) -> List[Tuple[str, Tuple[int, ...]]]:
    """Critic.parameters() order (sac_model.py:75-89,142-151) under ``prefix``."""
    out = []
    for q in ("q1", "q2"):
        out += [(f"{prefix}.{q}.body.0.weight", (HIDDEN, D + K)), (f"{prefix}.{q}.body.0.bias", (HIDDEN,)),
                (f"{prefix}.{q}.body.2.weight", (HIDDEN, HIDDEN)), (f"{prefix}.{q}.body.2.bias", (HIDDEN,)),
                (f"{prefix}.{q}.body.4.weight", (1, HIDDEN)), (f"{prefix}.{q}.body.4.bias", (1,))]
    return out


def _count(specs) -> int:
    return sum(int(np.prod(s)) for _, s in specs)


class _Node(nn.Module):
    pass


def _attach(root: nn.Module, specs, flat: torch.Tensor, grad: Optional[torch.Tensor],
            requires_grad: bool = True) -> None:
    off = 0
    for name, shape in specs:
        cnt = int(np.prod(shape))
        parts = name.split(".")
        mod = root
        for p in parts[:-1]:
            if not hasattr(mod, p) or not isinstance(getattr(mod, p), nn.Module):
                mod.add_module(p, _Node())
            mod = getattr(mod, p)
        param = nn.Parameter(flat[off:off + cnt].view(shape), requires_grad=requires_grad)
        if grad is not None:
            param.grad = grad[off:off + cnt].view(shape)
        mod.register_parameter(parts[-1], param)
        off += cnt
    assert off == flat.numel()


def _uniform_linear(fan_in: int, fan_out: int, scale: float = 0.33) -> nn.Linear:
    """nn.Linear then models/common.py:161-167 layer_init_uniform (consumes the global torch RNG
    exactly as the reference's construction does)."""
    layer = nn.Linear(fan_in, fan_out)
    with torch.no_grad():
        s = np.sqrt(3 / max(1, layer.weight.shape[1])) * scale
        torch.nn.init.uniform_(layer.weight, -s, s)
        torch.nn.init.constant_(layer.bias, 0.)
    return layer


def _flat_of(layers) -> torch.Tensor:
    return torch.cat([t.detach().reshape(-1) for l in layers for t in (l.weight, l.bias)])


def init_critic_flat(D: int, K: int) -> torch.Tensor:
    """SoftCritic(D, K) construction order (sac_model.py:154-165): critic.q1, critic.q2, then
    target_critic's own draws (overwritten by load_state_dict)."""
    q = [_uniform_linear(D + K, HIDDEN), _uniform_linear(HIDDEN, HIDDEN), _uniform_linear(HIDDEN, 1)]
    q += [_uniform_linear(D + K, HIDDEN), _uniform_linear(HIDDEN, HIDDEN), _uniform_linear(HIDDEN, 1)]
    flat = _flat_of(q)
    for _ in range(2):  # target_critic = Critic(...) consumes the RNG too
        _uniform_linear(D + K, HIDDEN), _uniform_linear(HIDDEN, HIDDEN), _uniform_linear(HIDDEN, 1)
    return flat


def init_actor_flat(D: int, K: int) -> torch.Tensor:
    """SoftActor(D, K) construction order (sac_model.py:92-139,181-188)."""
    return _flat_of([_uniform_linear(D, HIDDEN), _uniform_linear(HIDDEN, HIDDEN),
                     _uniform_linear(HIDDEN, K), _uniform_linear(HIDDEN, K)])


def _dev_f32(x, device) -> torch.Tensor:
    t = torch.as_tensor(x)
    if t.device != device:
        t = t.to(device, non_blocking=True)
    return t.float().contiguous()


class SoftCritic(nn.Module):
    """models/sac_model.py:154-178.  ``critic`` / ``target_critic`` / ``log_alpha`` /
    ``target_entropy`` as the reference's state_dict; target parameters do not require grad."""

    def __init__(self, observation_space, action_space, alpha: float = 1., device="cuda",
                 init: bool = True):
        super().__init__()
        self.obs_dim, self.act_dim = _prod(observation_space), _prod(action_space)
        D, K = self.obs_dim, self.act_dim
        device = torch.device(device)
        n = _count(critic_specs("critic", D, K))
        self.flat = torch.zeros(n, dtype=torch.float32, device=device)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=device)
        self.target_flat = torch.zeros(n, dtype=torch.float32, device=device)
        self.la_buf = torch.zeros(4, dtype=torch.float32, device=device)  # value, grad, m, v
        _attach(self, critic_specs("critic", D, K), self.flat, self.flat_grad)
        _attach(self, critic_specs("target_critic", D, K), self.target_flat, None, requires_grad=False)
        self.log_alpha = nn.Parameter(self.la_buf[0:1].view(()))
        self.log_alpha.grad = self.la_buf[1:2].view(())
        self.register_buffer("target_entropy", torch.tensor(-float(K), dtype=torch.float32, device=device))
        self._version = 0
        self._engine = None
        with torch.no_grad():
            self.la_buf[0] = math.log(alpha)
            if init:
                self.flat.copy_(init_critic_flat(D, K).to(device))
                self.target_flat.copy_(self.flat)

    def params_changed(self) -> None:
        self._version += 1

    def __getstate__(self):  # whole-model torch.save: drop the native engine handle
        return picklable_state(self)

    def __setstate__(self, state):
        super().__setstate__(state)
        D, K = self.obs_dim, self.act_dim
        rebind_views(self, critic_specs("critic", D, K), self.flat, self.flat_grad)
        rebind_views(self, critic_specs("target_critic", D, K), self.target_flat, None)
        self.log_alpha.data = self.la_buf[0:1].view(())
        self.log_alpha.grad = self.la_buf[1:2].view(())
        self.params_changed()

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict, assign=False)
        self.params_changed()
        return res

    @property
    def alpha(self) -> torch.Tensor:
        return self.log_alpha.exp()

    def _q(self, s, a, target: int):
        eng = self._engine
        if eng is None:
            raise RuntimeError("SoftCritic.forward needs a SACEngine (SACLearner) on the HIP path")
        return eng.q_forward(s, a, target)

    def forward(self, s, a):  # sac_model.py:170-171
        return self._q(s, a, 0)

    @torch.no_grad()
    def target(self, s, a):  # sac_model.py:173-175
        return self._q(s, a, 1)


class SoftActor(nn.Module):
    """models/sac_model.py:181-203 (with Actor / ActorBody / ContionusHead).  ``forward`` ->
    (mean, log_std); ``act(obs, eps)`` -> tanh-squashed noisy action on the CPU; ``policy(s)``
    -> (action, log_prob, std) with rsample noise drawn on the device."""

    def __init__(self, observation_space, action_space, action_scale: float = 1.,
                 action_bias: float = 0., device="cuda", dtype: str = "fp32", init: bool = True):
        super().__init__()
        self.obs_dim, self.act_dim = _prod(observation_space), _prod(action_space)
        self.observation_space, self.action_space = observation_space, action_space
        self.compute_dtype = dtype
        device = torch.device(device)
        specs = actor_specs(self.obs_dim, self.act_dim)
        n = _count(specs)
        self.flat = torch.zeros(n, dtype=torch.float32, device=device)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=device)
        _attach(self, specs, self.flat, self.flat_grad)
        self.actor.head.register_buffer("action_scale", torch.tensor(action_scale, dtype=torch.float32))
        self.actor.head.register_buffer("action_bias", torch.tensor(action_bias, dtype=torch.float32))
        self._version = 0
        self._train_engine = None
        self._infer_engine = None
        self.downstream = None
        if init:
            with torch.no_grad():
                self.flat.copy_(init_actor_flat(self.obs_dim, self.act_dim).to(device))

    # ------------------------------------------------------------- parameters
    def params_changed(self) -> None:
        self._version += 1

    def __getstate__(self):  # whole-model torch.save: drop the native engine handles
        return picklable_state(self)

    def __setstate__(self, state):
        super().__setstate__(state)
        rebind_views(self, actor_specs(self.obs_dim, self.act_dim), self.flat, self.flat_grad)
        self.params_changed()

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict, assign=False)
        self.params_changed()
        return res

    def load_flat_from(self, other: "SoftActor") -> None:
        with torch.no_grad():
            self.flat.copy_(other.flat.to(self.flat.device, non_blocking=True))
        self.params_changed()

    def clone_to(self, device) -> "SoftActor":
        m = SoftActor(self.observation_space, self.action_space,
                      float(self.actor.head.action_scale), float(self.actor.head.action_bias),
                      device=device, dtype=self.compute_dtype, init=False)
        m.load_flat_from(self)
        for p in m.parameters():
            p.requires_grad_(False)
        return m

    def __deepcopy__(self, memo):  # learning.py:134 copy.deepcopy(target_actor)
        m = self.clone_to(self.flat.device)
        for p in m.parameters():
            p.requires_grad_(True)
        return m

    def push(self) -> None:
        """rlmeta DownstreamModel.push: publish the learner weights to the inference copy."""
        if self.downstream is not None:
            self.downstream.load_flat_from(self)

    # ------------------------------------------------------------- compute
    def _engine(self, n: int) -> "SACEngine":
        if self._train_engine is not None and n <= self._train_engine.batch_size:
            return self._train_engine
        if self._infer_engine is None or n > self._infer_engine.batch_size:
            # the reference serves act() in batches of <= 128 (sac_model.py:190)
            self._infer_engine = SACEngine.inference(self, max(128, n))
        return self._infer_engine

    def _obs(self, x) -> torch.Tensor:
        if self.flat.device.type != "cuda":
            raise RuntimeError("SoftActor runs on the HIP path only (cuda device)")
        x = _dev_f32(x, self.flat.device)
        return x.reshape(-1, self.obs_dim)

    def forward(self, x):  # sac_model.py:115-122 -> (mean, log_std)
        x = self._obs(x)
        eng = self._engine(x.shape[0])
        mean, log_std, *_ = eng.policy(x, None)
        return mean, log_std

    @torch.no_grad()
    def act(self, obs, eps=0.):  # sac_model.py:190-200
        x = self._obs(obs)
        eng = self._engine(x.shape[0])
        e = float(torch.as_tensor(eps).reshape(-1)[0]) if not isinstance(eps, (int, float)) else float(eps)
        noise = torch.randn(x.shape[0], self.act_dim, device=x.device) if e != 0. else None
        a = eng.act(x, noise, e, float(self.actor.head.action_scale), float(self.actor.head.action_bias))
        return a.cpu()

    def policy(self, s, noise: Optional[torch.Tensor] = None):  # sac_model.py:202-203
        x = self._obs(s)
        eng = self._engine(x.shape[0])
        if noise is None:  # Normal.rsample draws eps ~ N(0, 1)
            noise = torch.randn(x.shape[0], self.act_dim, device=x.device)
        _, _, action, logp, std = eng.policy(x, noise)
        return action, logp, std


class SACEngine:
    """One ``sac_learner`` handle bound to the modules' flat buffers (see module doc)."""

    def __init__(self, actor: SoftActor, critic: Optional[SoftCritic], target_actor: Optional[SoftActor],
                 batch_size: int = 256, dtype: Optional[str] = None, critic_lr: float = 3e-3,
                 actor_lr: float = 3e-4, eps: float = 1e-5, betas=(0.9, 0.999),
                 max_grad_norm: Optional[float] = 40., tau: float = 0.005, gamma: float = 0.99,
                 tune_alpha: bool = True, seed: int = 0):
        L = _lib.lib()
        dev = actor.flat.device
        if dev.type != "cuda":
            raise RuntimeError("SACEngine needs a cuda (HIP) device")
        self.device = dev
        self.batch_size = int(batch_size)
        D, K = actor.obs_dim, actor.act_dim
        self.D, self.K = D, K
        dtype = dtype or actor.compute_dtype
        if dtype not in ("fp32", "bf16"):
            raise ValueError("dtype must be 'fp32' or 'bf16'")
        self.dtype = dtype
        if critic is None:  # inference-only handle: placeholder critic state
            critic = SoftCritic((D,), (K,), device=dev, init=False)
        if target_actor is None:
            target_actor = actor
        self.actor, self.critic, self.target_actor = actor, critic, target_actor
        f32 = dict(dtype=torch.float32, device=dev)
        self.actor_m = torch.zeros(actor.flat.numel(), **f32)
        self.actor_v = torch.zeros(actor.flat.numel(), **f32)
        self.critic_m = torch.zeros(critic.flat.numel(), **f32)
        self.critic_v = torch.zeros(critic.flat.numel(), **f32)
        self.metrics = torch.zeros(_lib.SAC_NUM_METRICS, **f32)
        cfg = _lib.SacConfig()
        _lib.check(L.sac_config_default(C.byref(cfg)), "sac_config_default")
        cfg.obs_dim, cfg.act_dim, cfg.batch_size = D, K, self.batch_size
        cfg.dtype = _lib.IMPALA_DTYPE_BF16 if dtype == "bf16" else _lib.IMPALA_DTYPE_F32
        cfg.critic_lr, cfg.actor_lr, cfg.adam_eps = critic_lr, actor_lr, eps
        cfg.adam_beta1, cfg.adam_beta2 = betas
        cfg.max_grad_norm = -1.0 if max_grad_norm is None else float(max_grad_norm)
        cfg.tau, cfg.gamma, cfg.tune_alpha = tau, gamma, int(bool(tune_alpha))
        cfg.target_entropy = float(critic.target_entropy)
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.tune_alpha = bool(tune_alpha)
        self.cfg = cfg
        h = C.c_void_p()
        _lib.check(L.sac_create(C.byref(cfg), dev.index or 0, C.byref(h)), "sac_create")
        self._h = h
        self._versions = None
        self._bind()

    @classmethod
    def inference(cls, actor: SoftActor, n: int) -> "SACEngine":
        return cls(actor, None, None, batch_size=n)

    def _bind(self):
        a, c, t = self.actor, self.critic, self.target_actor
        st = _lib.SacState(a.flat.data_ptr(), a.flat_grad.data_ptr(), self.actor_m.data_ptr(),
                           self.actor_v.data_ptr(), t.flat.data_ptr(), c.flat.data_ptr(),
                           c.flat_grad.data_ptr(), self.critic_m.data_ptr(), self.critic_v.data_ptr(),
                           c.target_flat.data_ptr(), c.la_buf.data_ptr(), self.metrics.data_ptr())
        self._state = st
        _lib.check(_lib.lib().sac_bind_state(self._h, C.byref(st), _lib.stream_ptr(None)),
                   "sac_bind_state")
        self._versions = (a._version, c._version, t._version)

    def _sync_weights(self):
        v = (self.actor._version, self.critic._version, self.target_actor._version)
        if v != self._versions:
            _lib.check(_lib.lib().sac_refresh_weights(self._h, _lib.stream_ptr(None)),
                       "sac_refresh_weights")
            self._versions = v

    def set_steps(self, critic_step: int, actor_step: int, alpha_step: int) -> None:
        _lib.check(_lib.lib().sac_set_steps(self._h, critic_step, actor_step, alpha_step,
                                            _lib.stream_ptr(None)), "sac_set_steps")

    def train_step(self, s, a, r, s1, done, probabilities=None, noise=None, priorities=None,
                   stream=None) -> None:
        """agents/sac/learning.py:146-193 (after sampling) on device tensors."""
        N, D, K = self.batch_size, self.D, self.K
        dev = self.device
        s, a, r, s1 = (_dev_f32(x, dev) for x in (s, a, r, s1))
        if s.numel() != N * D or s1.numel() != N * D or a.numel() != N * K or r.numel() != N:
            raise ValueError(f"SAC batch must be N={N} transitions of obs {D} / action {K}")
        d = torch.as_tensor(done).to(dev).reshape(-1).to(torch.uint8).contiguous()
        p = None if probabilities is None else _dev_f32(probabilities, dev).reshape(-1)
        if noise is not None:
            noise = _dev_f32(noise, dev)
            if noise.numel() != 3 * N * K:
                raise ValueError("noise must hold [3][N][K] standard-normal draws")
        if priorities is not None and (priorities.numel() != N or priorities.dtype != torch.float32):
            raise ValueError("priorities must be a float32 [N] device tensor")
        self._keep = (s, a, r, s1, d, p, noise, priorities)  # alive until the next call
        self._sync_weights()
        b = _lib.SacBatch(s.data_ptr(), a.data_ptr(), r.data_ptr(), s1.data_ptr(), d.data_ptr(),
                          _lib.ptr(p), _lib.ptr(noise), _lib.ptr(priorities))
        _lib.check(_lib.lib().sac_train_step(self._h, C.byref(b), _lib.stream_ptr(stream)),
                   "sac_train_step")

    def act(self, x, noise, noise_scale: float, scale: float, bias: float) -> torch.Tensor:
        self._sync_weights()
        n = x.shape[0]
        out = torch.empty(n, self.K, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().sac_act(self._h, x.data_ptr(), n, _lib.ptr(noise), noise_scale,
                                      scale, bias, out.data_ptr(), _lib.stream_ptr(None)), "sac_act")
        return out

    def policy(self, x, noise):
        self._sync_weights()
        n = x.shape[0]
        f = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)  # noqa: E731
        mean, ls, act, std = f(n, self.K), f(n, self.K), f(n, self.K), f(n, self.K)
        logp = f(n)
        if noise is not None:
            noise = _dev_f32(noise, self.device)
        _lib.check(_lib.lib().sac_policy(self._h, x.data_ptr(), n, _lib.ptr(noise), mean.data_ptr(),
                                         ls.data_ptr(), act.data_ptr(), logp.data_ptr(),
                                         std.data_ptr(), _lib.stream_ptr(None)), "sac_policy")
        return mean, ls, act, logp, std

    def q_forward(self, s, a, target: int):
        self._sync_weights()
        s = _dev_f32(s, self.device).reshape(-1, self.D)
        a = _dev_f32(a, self.device).reshape(-1, self.K)
        n = s.shape[0]
        q1 = torch.empty(n, dtype=torch.float32, device=self.device)
        q2 = torch.empty(n, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().sac_q_forward(self._h, s.data_ptr(), a.data_ptr(), n, int(target),
                                            q1.data_ptr(), q2.data_ptr(), _lib.stream_ptr(None)),
                   "sac_q_forward")
        return q1, q2

    # live per-phase timer (bench roofline)
    @staticmethod
    def phase_names() -> List[str]:
        L = _lib.lib()
        return [L.sac_phase_name(i).decode() for i in range(L.sac_phase_count())]

    def timer_start(self, phase: int, max_launches: int) -> None:
        _lib.check(_lib.lib().sac_timer_start(self._h, phase, max_launches), "sac_timer_start")

    def timer_read(self) -> Tuple[float, int]:
        ms, n = C.c_float(), C.c_int()
        _lib.check(_lib.lib().sac_timer_read(self._h, C.byref(ms), C.byref(n)), "sac_timer_read")
        return float(ms.value), int(n.value)

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.lib().sac_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _adam_hparams(opt, default_lr: float):
    if opt is None:
        return default_lr, 1e-5, (0.9, 0.999)
    if not isinstance(opt, torch.optim.Adam):
        raise TypeError("the HIP SAC learner implements torch.optim.Adam only")
    g = opt.param_groups[0]
    if g.get("weight_decay", 0) or g.get("amsgrad", False) or g.get("maximize", False):
        raise ValueError("weight_decay / amsgrad / maximize are not used by the reference")
    return float(g["lr"]), float(g["eps"]), tuple(g["betas"])


class SACLearner(Learner):
    """agents/sac/learning.py:93-193 on one MI355X."""

    def __init__(self, model: SoftActor, critic: SoftCritic, target_actor: SoftActor,
                 replay_buffer, critic_optimizer=None, actor_optimizer=None, batch_size: int = 256,
                 tune_alpha: bool = True, max_grad_norm: Optional[float] = 40., epochs: int = 2,
                 policy_update_period: int = 2, tau: float = 0.005,
                 learning_starts: Optional[int] = 1000, model_push_period: int = 10,
                 dtype: Optional[str] = None, gamma: float = 0.99, seed: int = 0):
        self._model = model
        self._critic = critic
        self._replay_buffer = replay_buffer
        self._critic_optimizer = critic_optimizer
        self._actor_optimizer = actor_optimizer
        self._batch_size = batch_size
        self._max_grad_norm = max_grad_norm
        self._tune_alpha = tune_alpha
        self._tau = tau
        self._epochs = epochs  # stored, unused -- as the reference
        self._policy_update_period = policy_update_period  # stored, unused -- as the reference
        self._learning_starts = learning_starts
        self._model_push_period = model_push_period
        self._step_counter = 0
        self._device = None
        self.can_train = False
        self._target_actor = copy.deepcopy(target_actor)  # learning.py:134
        c_lr, c_eps, c_betas = _adam_hparams(critic_optimizer, 3e-3)
        a_lr, a_eps, a_betas = _adam_hparams(actor_optimizer, 3e-4)
        if c_eps != a_eps or c_betas != a_betas:
            raise ValueError("the two optimizers must share eps and betas (builder.py:42-47)")
        self._engine = SACEngine(model, critic, self._target_actor, batch_size=batch_size,
                                 dtype=dtype, critic_lr=c_lr, actor_lr=a_lr, eps=c_eps,
                                 betas=c_betas, max_grad_norm=max_grad_norm, tau=tau, gamma=gamma,
                                 tune_alpha=tune_alpha, seed=seed)
        model._train_engine = self._engine
        critic._engine = self._engine
        self._prio = torch.zeros(batch_size, dtype=torch.float32, device=model.flat.device)

    @property
    def engine(self) -> SACEngine:
        return self._engine

    @property
    def target_actor(self) -> SoftActor:
        return self._target_actor

    def device(self) -> torch.device:
        if self._device is None:
            self._device = self._model.flat.device
        return self._device

    @property
    def samples_per_step(self) -> int:
        """Environment frames one train_step consumes (DistributedAgent.train's total without
        a controller)."""
        return self._batch_size

    def prepare(self):  # learning.py:141-144
        if self.can_train is False:
            self._replay_buffer.warm_up(self._learning_starts)
        self.can_train = True

    def train_step(self) -> Dict[str, object]:  # learning.py:146-193
        t0 = time.perf_counter()
        rb = self._replay_buffer
        if isinstance(rb, DeviceTransitionReplay):  # consumed by this step before the next sample
            keys, batch, values = rb.sample(self._batch_size, copy=False)
        else:
            keys, batch, values = rb.sample(self._batch_size)
        dev = self.device()
        s, a, r, s1, d = (torch.as_tensor(x).to(dev, non_blocking=True) for x in batch)
        s, a, r, s1, d = (x.squeeze(dim=-1) if x.dim() > 1 and x.shape[-1] == 1 else x
                          for x in (s, a, r, s1, d))
        t1 = time.perf_counter()
        self._engine.train_step(s, a, r, s1, d, probabilities=values, priorities=self._prio)
        m = self._engine.metrics.clone()  # device scalars; float(v) synchronises lazily
        metrics = {k: m[i] for k, i in _lib.SAC_CRITIC_METRICS if self._max_grad_norm is not None or i != 5}
        metrics.update({k: m[i] for k, i in _lib.SAC_ACTOR_METRICS if self._max_grad_norm is not None or i != 8})
        if self._tune_alpha:
            metrics.update({k: m[i] for k, i in _lib.SAC_ALPHA_METRICS})
        t2 = time.perf_counter()
        update_time = 0
        if self._step_counter % self._model_push_period == 0:
            start = time.perf_counter()
            self._model.push()
            update_time = time.perf_counter() - start
        capacity, size = self._replay_buffer.info()
        metrics["debug/rb_capacity"] = capacity
        self._step_counter += 1
        metrics["debug/replay_sample_per_second"] = (self._batch_size / ((t1 - t0) * 1000))
        metrics["debug/gradient_per_second"] = (self._batch_size / ((t2 - t1) * 1000))
        metrics["debug/total_time"] = (time.perf_counter() - t0) * 1000
        metrics["debug/sample_dt"] = (t1 - t0) * 1000
        metrics["debug/forward_dt"] = (t2 - t1) * 1000
        metrics["debug/update_dt"] = update_time * 1000
        return metrics

    @property
    def next_priorities(self) -> torch.Tensor:
        """critic_loss next_priorities of the last step (learning.py:240-241)."""
        return self._prio


class DeviceTransitionReplay:
    """ReplayBuffer(CircularBuffer(capacity), UniformSampler()) (agents/sac/builder.py:30-36)
    with the circular store in HBM: transitions (s [D], a [K], r, s1 [D], done) are appended
    from the host (one H2D per append call) and ``sample`` draws keys, probabilities and the
    batch on the device (``sac_sample``).  Storage is allocated on the first append."""

    def __init__(self, capacity: int = 1_000_000, device="cuda", seed: Optional[int] = None):
        self.capacity = int(capacity)
        self.device = torch.device(device)
        self.seed = 0 if seed is None else int(seed)
        self._size = 0
        self._cursor = 0
        self._next_key = 0
        self._draws = 0
        self._cv = threading.Condition()
        self._fields: Optional[List[torch.Tensor]] = None
        self._out = None

    def reset(self, seed: Optional[int] = None):  # UniformSampler.reset(seed)
        self.seed = 0 if seed is None else int(seed)
        self._draws = 0

    def __len__(self):
        return self._size

    def info(self) -> Tuple[int, int]:
        return self.capacity, self._size

    def _alloc(self, D: int, K: int):
        C_, d = self.capacity, self.device
        self._fields = [torch.zeros(C_, D, dtype=torch.float32, device=d),
                        torch.zeros(C_, K, dtype=torch.float32, device=d),
                        torch.zeros(C_, dtype=torch.float32, device=d),
                        torch.zeros(C_, D, dtype=torch.float32, device=d),
                        torch.zeros(C_, dtype=torch.uint8, device=d)]
        self._keys = torch.zeros(C_, dtype=torch.int64, device=d)

    def extend(self, items: Sequence) -> None:
        """Append transitions: a list of [s, a, r, s1, done] items (each field with or without a
        leading unit dim, as SACActor._make_replay unbatches them), or one collated 5-tuple."""
        if len(items) == 5 and isinstance(items[0], torch.Tensor) and items[0].dim() == 2 \
                and items[2].dim() <= 2 and items[2].reshape(-1).numel() == items[0].shape[0]:
            cols = list(items)
        else:
            cols = [torch.stack([torch.as_tensor(it[j]).reshape(-1) for it in items]) for j in range(5)]
        s, a, r, s1, d = cols
        n = s.shape[0]
        s = s.reshape(n, -1).float()
        a = a.reshape(n, -1).float()
        r = r.reshape(n).float()
        s1 = s1.reshape(n, -1).float()
        d = d.reshape(n).to(torch.uint8)
        with self._cv:
            if self._fields is None:
                self._alloc(s.shape[1], a.shape[1])
            src = [s, a, r, s1, d]
            pos = 0
            while pos < n:
                take = min(n - pos, self.capacity - self._cursor)
                for f, x in zip(self._fields, src):
                    f[self._cursor:self._cursor + take].copy_(x[pos:pos + take], non_blocking=True)
                self._keys[self._cursor:self._cursor + take] = torch.arange(
                    self._next_key, self._next_key + take, device=self.device)
                self._next_key += take
                self._cursor = (self._cursor + take) % self.capacity
                pos += take
            self._size = min(self._size + n, self.capacity)
            self._cv.notify_all()

    def append(self, item) -> None:
        self.extend([item])

    async def async_extend(self, items) -> None:
        self.extend(items)

    def warm_up(self, learning_starts: Optional[int] = None, timeout: float = 240.0) -> None:
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

    def sample(self, batch_size: int, copy: bool = True):
        """-> (keys [n] i64, [s, a, r, s1, done] device tensors, probabilities [n] f32).
        copy=False returns the buffer's persistent output tensors (overwritten by the next
        sample; the learner consumes them first), so a step's sampling is two launches."""
        with self._cv:
            if self._size == 0:
                raise RuntimeError("sample from an empty replay buffer")
            n = int(batch_size)
            if self._out is None or self._out[0].shape[0] != n:
                d = self.device
                self._out = [torch.empty(n, *f.shape[1:], dtype=f.dtype, device=d) for f in self._fields]
                self._idx = torch.empty(n, dtype=torch.int64, device=d)
                self._probs = torch.empty(n, dtype=torch.float32, device=d)
                self._keys_out = torch.empty(n, dtype=torch.int64, device=d)
            out, idx, probs, keys_out = self._out, self._idx, self._probs, self._keys_out
            fields = self._fields + [self._keys]
            dsts = out + [keys_out]
            src = (C.c_void_p * 6)(*[f.data_ptr() for f in fields])
            dst = (C.c_void_p * 6)(*[t.data_ptr() for t in dsts])
            rb = (C.c_size_t * 6)(*[f[0].numel() * f.element_size() if f.dim() > 1 else f.element_size()
                                     for f in fields])
            self._draws += 1
            _lib.check(_lib.lib().sac_sample(self.seed, self._draws, self._size, n, idx.data_ptr(),
                                             probs.data_ptr(), src, dst, rb, 6,
                                             _lib.stream_ptr(None)), "sac_sample")
        if not copy:
            return keys_out, list(out), probs
        return keys_out.clone(), [t.clone() for t in out], probs.clone()


class SACActor(Actor):
    """SACActorRemote (agents/sac/learning.py:15-57): act with exploration noise, collect
    (obs, act, reward, next_obs, done) with truncations not counted as terminal, send
    ``rollout_length`` transitions to the replay per update."""

    def __init__(self, model, replay_buffer=None, exploration_noise: float = 0.3, gamma: float = 0.99,
                 rollout_length: int = 100):
        self._model = model
        self._exploration_noise = torch.tensor([exploration_noise], dtype=torch.float32)
        self._gamma = gamma
        self._replay_buffer = replay_buffer
        self._rollout_length = rollout_length
        self._trajectory: List[tuple] = []
        self._last_transition = None

    async def async_act(self, timestep):
        obs = timestep.observation if hasattr(timestep, "observation") else timestep[0]
        return self._model.act(obs, self._exploration_noise)

    async def async_observe_init(self, timestep) -> None:
        if self._replay_buffer is None:
            return
        self._last_transition = timestep.observation if hasattr(timestep, "observation") else timestep[0]

    def observe(self, action, next_timestep) -> None:
        if self._replay_buffer is None:
            return
        obs = self._last_transition
        act = action[0] if isinstance(action, (tuple, list)) else action
        next_obs, reward, done, info = next_timestep
        done = torch.as_tensor(done, dtype=torch.bool).clone().reshape(-1)
        trunc = torch.as_tensor(info.get("terminated", False), dtype=torch.bool).reshape(-1)
        done[trunc.expand_as(done)] = False  # learning.py:46-48: truncation is not terminal
        self._trajectory.append((torch.as_tensor(obs, dtype=torch.float32),
                                 torch.as_tensor(act, dtype=torch.float32),
                                 torch.as_tensor(reward, dtype=torch.float32),
                                 torch.as_tensor(next_obs, dtype=torch.float32), done))
        self._last_transition = torch.as_tensor(next_obs).clone()

    async def async_observe(self, action, next_timestep) -> None:
        self.observe(action, next_timestep)

    def update(self) -> None:
        if self._replay_buffer is None or not self._trajectory:
            return
        self._replay_buffer.extend(self._make_replay())

    async def async_update(self) -> None:
        self.update()

    def _make_replay(self):  # learning.py:59-61: one item per transition
        items, self._trajectory = self._trajectory, []
        return [list(t) for t in items]


class SACBuilder(Builder):
    """agents/sac/builder.py:22-74 on the HIP learner."""

    def __init__(self, cfg):
        self.cfg = cfg
        self._learner_model = None
        self._actor_model = None

    def _learner_cfg(self, key, default):
        lc = self.cfg.get("learner", {}) if isinstance(self.cfg, dict) else getattr(self.cfg, "learner", {})
        return lc.get(key, default) if lc else default

    def make_replay(self):  # builder.py:30-36
        return DeviceTransitionReplay(int(self.cfg.agent.replay_buffer_size),
                                      device=self.cfg.distributed.train_device,
                                      seed=self.cfg.training.seed)

    def make_actor(self, model, rb=None, deterministic: bool = False):  # builder.py:38-40
        noise = 0. if deterministic else float(self.cfg.agent.exploration_noise)
        rl = int(self.cfg.agent.rollout_length)
        return lambda index: SACActor(model, rb, exploration_noise=noise, rollout_length=rl)

    def make_learner(self, model, rb):  # builder.py:42-58
        actor, critic = self._learner_model
        a = self.cfg.agent
        c_opt = torch.optim.Adam([{"params": list(critic.critic.parameters())}, {"params": [critic.log_alpha]}],
                                 lr=float(a.optimizer.critic_lr), eps=float(a.optimizer.eps))
        a_opt = torch.optim.Adam(actor.parameters(), lr=float(a.optimizer.actor_lr), eps=float(a.optimizer.eps))
        return SACLearner(model, critic=critic, target_actor=actor, replay_buffer=rb,
                          batch_size=int(a.batch_size), critic_optimizer=c_opt, actor_optimizer=a_opt,
                          model_push_period=int(a.push_period), learning_starts=int(a.learning_starts),
                          tune_alpha=bool(a.tune_alpha), dtype=self._learner_cfg("dtype", None),
                          seed=int(self.cfg.training.seed))

    def make_network(self, env_spec):  # builder.py:60-74
        obs_shape = tuple(env_spec.observation_space.shape)
        act_shape = tuple(env_spec.action_space.shape)
        dev = self.cfg.distributed.train_device
        critic = SoftCritic(obs_shape, act_shape, alpha=float(self.cfg.agent.alpha), device=dev)
        actor = SoftActor(obs_shape, act_shape, device=dev, dtype=self._learner_cfg("dtype", "fp32"))
        self._learner_model = (actor, critic)
        inference = actor.clone_to(self.cfg.distributed.infer_device)
        self._actor_model = inference
        actor.downstream = inference
        return actor
