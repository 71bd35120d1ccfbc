"""ORACLE — test infrastructure only (never shipped, never on the product path).

Torch-CPU fp32 restatement of the reference SAC learner step (SURVEY.md §8(f) row 4,
BASELINE config 5), op for op.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg use it.

Follows:

* models : ``models/sac_model.py:19-31`` (``to_action``), ``:75-122`` (``SoftQNetwork``,
  ``ActorBody``, ``Actor``), ``:125-139`` (``ContionusHead``), ``:142-178`` (``Critic``,
  ``SoftCritic``), ``:181-203`` (``SoftActor.policy``); init ``models/common.py:161-167``
  (``layer_init_uniform``, scale 0.33, bias 0)
* step   : ``agents/sac/learning.py:145-265`` (``SACLearner.train_step``, ``_train_critic``,
  ``_train_actor``, ``_train_alpha``, ``critic_loss``, ``actor_loss``, ``alpha_loss``)
* optim  : ``agents/sac/builder.py:42-47`` (critic Adam over critic.critic + log_alpha at
  critic_lr, actor Adam at actor_lr, eps from conf/agent/sac.yaml)

The reparameterised samples ``Normal(mean, std).rsample()`` are ``mean + eps * std`` with
``eps`` standard normal; here ``eps`` is an explicit input (one [N, K] draw per ``policy``
call: target actor on s1, actor on s, actor on s again for alpha), so the GPU path and this
oracle see the same noise.  Pinned against the reference by ``tests/golden/make_sac_golden.py``.
"""
from __future__ import annotations

import copy
import math
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

LOG_STD_MAX = 2
LOG_STD_MIN = -5


def layer_init_uniform(layer: nn.Linear, scale: float = 0.33) -> nn.Linear:
    """models/common.py:161-167."""
    with torch.no_grad():
        fan_in = max(1, layer.weight.shape[1])
        s = np.sqrt(3 / fan_in) * scale
        torch.nn.init.uniform_(layer.weight, -s, s)
        torch.nn.init.constant_(layer.bias, 0.)
    return layer


class SoftQNetwork(nn.Module):  # sac_model.py:75-89
    def __init__(self, obs_dim: int, act_dim: int):
        super().__init__()
        self.body = nn.Sequential(layer_init_uniform(nn.Linear(obs_dim + act_dim, 256)), nn.ReLU(),
                                  layer_init_uniform(nn.Linear(256, 256)), nn.ReLU(),
                                  layer_init_uniform(nn.Linear(256, 1)))

    def forward(self, x, a):
        return self.body(torch.cat([x, a], dim=-1)).squeeze(-1)


class ActorBody(nn.Module):  # sac_model.py:92-109
    def __init__(self, obs_dim: int):
        super().__init__()
        self.body = nn.Sequential(layer_init_uniform(nn.Linear(obs_dim, 256)), nn.ReLU(),
                                  layer_init_uniform(nn.Linear(256, 256)), nn.ReLU())

    def forward(self, x):
        return self.body(x)


class ContionusHead(nn.Module):  # sac_model.py:125-139 (reference spelling kept for keys)
    def __init__(self, act_dim: int):
        super().__init__()
        self.fc_mean = layer_init_uniform(nn.Linear(256, act_dim))
        self.fc_logstd = layer_init_uniform(nn.Linear(256, act_dim))
        self.register_buffer("action_scale", torch.tensor(1.0, dtype=torch.float32))
        self.register_buffer("action_bias", torch.tensor(0.0, dtype=torch.float32))

    def forward(self, h):
        mean = self.fc_mean(h)
        log_std = torch.tanh(self.fc_logstd(h))
        log_std = LOG_STD_MIN + 0.5 * (LOG_STD_MAX - LOG_STD_MIN) * (log_std + 1)
        return mean, log_std


class Actor(nn.Module):  # sac_model.py:112-122
    def __init__(self, obs_dim: int, act_dim: int):
        super().__init__()
        self.body = ActorBody(obs_dim)
        self.head = ContionusHead(act_dim)

    def forward(self, x):
        return self.head(self.body(x))


class SoftActor(nn.Module):  # sac_model.py:181-203 (the actor key prefix is `actor.`)
    def __init__(self, obs_dim: int, act_dim: int):
        super().__init__()
        self.actor = Actor(obs_dim, act_dim)

    def forward(self, x):
        return self.actor(x)

    def policy(self, s, eps):
        mu, log_std = self.actor(s)
        return to_action(mu, log_std, eps)


class Critic(nn.Module):  # sac_model.py:142-151
    def __init__(self, obs_dim: int, act_dim: int):
        super().__init__()
        self.q1 = SoftQNetwork(obs_dim, act_dim)
        self.q2 = SoftQNetwork(obs_dim, act_dim)

    def forward(self, s, a):
        return self.q1(s, a), self.q2(s, a)


class SoftCritic(nn.Module):  # sac_model.py:154-178
    def __init__(self, obs_dim: int, act_dim: int, alpha: float = 1.0):
        super().__init__()
        self.critic = Critic(obs_dim, act_dim)
        self.target_critic = Critic(obs_dim, act_dim)
        self.target_critic.load_state_dict(self.critic.state_dict())
        self.log_alpha = nn.Parameter(torch.tensor(math.log(alpha), dtype=torch.float32))
        self.register_buffer("target_entropy", torch.tensor(-float(act_dim), dtype=torch.float32))
        for p in self.target_critic.parameters():
            p.requires_grad = False

    def forward(self, s, a):
        return self.critic.q1(s, a), self.critic.q2(s, a)

    @property
    def alpha(self):
        return self.log_alpha.exp()


def to_action(mean, log_std, eps, action_scale=1.0, action_bias=0.):
    """sac_model.py:19-29 with rsample() = mean + eps * std (torch's Normal.rsample)."""
    std = log_std.exp()
    normal = torch.distributions.Normal(mean, std)
    x_t = mean + eps * std
    y_t = torch.tanh(x_t)
    action = y_t * action_scale + action_bias
    log_prob = normal.log_prob(x_t)
    log_prob = log_prob - torch.log(action_scale * (1 - y_t.pow(2)) + 1e-6)
    return action, log_prob.sum(-1), std


def make_models(obs_dim: int, act_dim: int, seed: int = 0, alpha: float = 1.0):
    """SACBuilder.make_network order (builder.py:60-66): critic first, then actor."""
    torch.manual_seed(seed)
    critic = SoftCritic(obs_dim, act_dim, alpha=alpha)
    actor = SoftActor(obs_dim, act_dim)
    return actor, critic


def critic_loss(actor, critic, batch, weight, eps, gamma=0.99):  # learning.py:233-248
    s, a, r, s1, d = batch
    with torch.no_grad():
        a1, logp1, _ = actor.policy(s1, eps)
        t1, t2 = critic.target_critic(s1, a1)
        min_next = torch.min(t1, t2) - critic.alpha * logp1
        y = r + d.logical_not() * gamma * min_next
    q1, q2 = critic(s, a)
    with torch.no_grad():
        prio = (y - torch.min(q1, q2)).abs()
    l1 = (y - q1).pow(2).mul(weight).mean()
    l2 = (y - q2).pow(2).mul(weight).mean()
    loss = l1 + l2
    return loss, prio, {"train/qf1_loss": l1, "train/qf2_loss": l2, "train/qf1": q1.mean(),
                        "train/qf2": q2.mean(), "train/qf_loss": loss / 2.}


def actor_loss(actor, critic, batch, eps):  # learning.py:251-257
    s = batch[0]
    pi, logp, std = actor.policy(s, eps)
    q1, q2 = critic(s, pi)
    loss = ((critic.alpha * logp) - torch.min(q1, q2)).mean()
    return loss, {"train/actor_loss": loss, "train/actor_std": std.mean(dim=-1).mean()}


def alpha_loss(actor, critic, batch, eps):  # learning.py:260-265
    s = batch[0]
    with torch.no_grad():
        _, logp, _ = actor.policy(s, eps)
    loss = -(critic.log_alpha * (logp + critic.target_entropy)).mean()
    return loss, {"train/alpha_loss": loss, "train/alpha": critic.alpha}


class SACState:
    """The learner's mutable state: actor, critic (+ target critic, log_alpha), the target
    actor (a deep copy of the actor, learning.py:134), both optimizers (builder.py:42-47)."""

    def __init__(self, actor, critic, critic_lr=3e-3, actor_lr=3e-4, eps=1e-5, tau=0.005,
                 max_grad_norm=40.0, tune_alpha=True):
        self.actor, self.critic = actor, critic
        self.target_actor = copy.deepcopy(actor)
        self.critic_opt = torch.optim.Adam([{"params": critic.critic.parameters()},
                                            {"params": critic.log_alpha}], lr=critic_lr, eps=eps)
        self.actor_opt = torch.optim.Adam(actor.parameters(), lr=actor_lr, eps=eps)
        self.tau, self.max_grad_norm, self.tune_alpha = tau, max_grad_norm, tune_alpha


def train_step(st: SACState, batch, probabilities, eps3) -> Dict[str, torch.Tensor]:
    """learning.py:146-193 without the replay / timing / push plumbing.  ``eps3`` = the three
    [N, K] noise draws in call order (target actor on s1, actor on s, actor on s for alpha)."""
    w = probabilities.to(torch.float32).pow(-0.4)
    w.div_(w.max())
    # _train_critic (learning.py:195-211)
    loss, prio, metrics = critic_loss(st.target_actor, st.critic, batch, w, eps3[0])
    st.critic_opt.zero_grad(set_to_none=True)
    loss.backward()
    metrics["train/critic_grad_norm"] = torch.nn.utils.clip_grad_norm_(st.critic.parameters(),
                                                                       st.max_grad_norm)
    st.critic_opt.step()
    # _train_actor (learning.py:213-223)
    loss, am = actor_loss(st.actor, st.critic, batch, eps3[1])
    st.actor_opt.zero_grad(set_to_none=True)
    loss.backward()
    am["train/actor_grad_norm"] = torch.nn.utils.clip_grad_norm_(st.actor.parameters(),
                                                                 st.max_grad_norm)
    st.actor_opt.step()
    metrics.update(am)
    if st.tune_alpha:  # _train_alpha (learning.py:225-230)
        loss, alm = alpha_loss(st.actor, st.critic, batch, eps3[2])
        st.critic_opt.zero_grad(set_to_none=True)
        loss.backward()
        st.critic_opt.step()
        metrics.update(alm)
    with torch.no_grad():  # Polyak (learning.py:174-180)
        for p, tp in zip(st.critic.critic.parameters(), st.critic.target_critic.parameters()):
            tp.data.copy_(st.tau * p.data + (1 - st.tau) * tp.data)
        for p, tp in zip(st.actor.parameters(), st.target_actor.parameters()):
            tp.data.copy_(st.tau * p.data + (1 - st.tau) * tp.data)
    metrics["prio"] = prio
    return metrics


def flat(params) -> np.ndarray:
    return torch.cat([p.detach().reshape(-1) for p in params]).numpy().copy()


def load_flat(params, v: np.ndarray) -> None:
    off = 0
    with torch.no_grad():
        for p in params:
            n = p.numel()
            p.copy_(torch.from_numpy(np.ascontiguousarray(v[off:off + n])).reshape(p.shape))
            off += n
    assert off == v.size


def synthetic_batch(N: int, obs_dim: int, act_dim: int, seed: int = 0):
    """Continuous-control transitions: s, s1 ~ N(0,1); a ~ U(-1,1); r ~ N(0,1); done ~ 5%."""
    rng = np.random.default_rng(seed)
    s = rng.standard_normal((N, obs_dim)).astype(np.float32)
    a = rng.uniform(-1, 1, (N, act_dim)).astype(np.float32)
    r = rng.standard_normal(N).astype(np.float32)
    s1 = rng.standard_normal((N, obs_dim)).astype(np.float32)
    d = rng.random(N) < 0.05
    return s, a, r, s1, d
