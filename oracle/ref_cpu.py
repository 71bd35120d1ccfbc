"""ORACLE — test infrastructure only (never shipped, never on the product path).

Torch-CPU fp32 restatement of the reference IMPALA learner step, op for op.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it,
and only as the checker / the timed CPU baseline ("kind": "port").

Follows, line by line:

* model  : ``models/models.py:61-76`` (``AtariActorCritic``), ``models/common.py:108-126``
  (``AtariBody``), ``models/common.py:151-158`` (``layer_init_truncated``),
  ``models/distributed_models.py:12-19`` (``AtariPPOModel`` wrapper -> ``model.`` key prefix)
* step   : ``agents/impala/learning.py:140-177`` (``ImpalaLearner._train_step``)
* V-trace: ``oracle/vtrace.py`` (restated rlego/rlax; see its header)
* optim  : ``agents/impala/builder.py:43-44`` (``torch.optim.Adam(lr, eps)``),
  ``agents/impala/learning.py:172-176`` (``clip_grad_norm_`` then ``step``)

Pinned against the reference itself by ``tests/golden/make_golden.py`` (imports
``/root/reference`` in the survey container with rlmeta/moolib/envs stubbed at their import
boundary) -> ``tests/golden/*.npz`` -> ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

try:  # functorch.vmap as at agents/impala/learning.py:15-18
    from torch.func import vmap as _vmap
except Exception:  # pragma: no cover
    _vmap = None

from oracle.vtrace import DEFAULT_GRAD_MODE, mode_kwargs, vtrace_td_error_and_advantage

# state_dict key order == flat parameter order
PARAM_SPECS: List[Tuple[str, Tuple[int, ...]]] = [
    ("model.body.body.0.weight", (32, 3, 8, 8)),
    ("model.body.body.0.bias", (32,)),
    ("model.body.body.2.weight", (64, 32, 4, 4)),
    ("model.body.body.2.bias", (64,)),
    ("model.body.body.4.weight", (64, 64, 3, 3)),
    ("model.body.body.4.bias", (64,)),
    ("model.projection.0.weight", (1024,)),
    ("model.projection.0.bias", (1024,)),
    ("model.projection.1.weight", (256, 1024)),
    ("model.projection.1.bias", (256,)),
    ("model.actor.weight", (15, 256)),
    ("model.actor.bias", (15,)),
    ("model.critic.weight", (1, 256)),
    ("model.critic.bias", (1,)),
]


def _layer_init_truncated(layer: nn.Module, scale: float = 1.0) -> nn.Module:
    """models/common.py:151-158: trunc_normal(std=sqrt(scale/fan_in)/0.8796...), bias 0."""
    with torch.no_grad():
        if isinstance(layer, nn.Conv2d):
            fan_in = layer.weight.shape[1] * layer.weight.shape[2] * layer.weight.shape[3]
        else:
            fan_in = layer.weight.shape[1]
        fan_in = max(1, fan_in)
        std = np.sqrt(scale / fan_in) / np.asarray(.87962566103423978, dtype=np.float32)
        torch.nn.init.trunc_normal_(layer.weight, std=float(std))
        torch.nn.init.constant_(layer.bias, 0.)
    return layer


class _Body(nn.Module):
    """models/common.py:108-126 (NatureCNN; output_dim hard-coded 1024 => 64x64 input)."""

    def __init__(self, c: int = 3):
        super().__init__()
        self.body = nn.Sequential(
            _layer_init_truncated(nn.Conv2d(c, 32, 8, stride=4)), nn.ReLU(),
            _layer_init_truncated(nn.Conv2d(32, 64, 4, stride=2)), nn.ReLU(),
            _layer_init_truncated(nn.Conv2d(64, 64, 3, stride=1)), nn.ReLU(),
            nn.Flatten())

    def forward(self, x):
        return self.body(x)


class _ActorCritic(nn.Module):
    """models/models.py:61-76."""

    def __init__(self, action_dim: int = 15, h_dim: int = 256):
        super().__init__()
        self.body = _Body()
        self.projection = nn.Sequential(nn.LayerNorm(1024),
                                        _layer_init_truncated(nn.Linear(1024, h_dim)),
                                        nn.GELU())
        self.actor = _layer_init_truncated(nn.Linear(h_dim, action_dim))
        self.critic = _layer_init_truncated(nn.Linear(h_dim, 1))

    def forward(self, x):
        x = x / 255.
        h = self.body(x)
        h = self.projection(h)
        return self.actor(h), self.critic(h)


class RefModel(nn.Module):
    """models/distributed_models.py:12-19 (``AtariPPOModel``: ``self.model`` prefix)."""

    def __init__(self, action_dim: int = 15):
        super().__init__()
        self.model = _ActorCritic(action_dim)

    def forward(self, obs):
        return self.model(obs)


def make_model(seed: int = 0, action_dim: int = 15) -> RefModel:
    torch.manual_seed(seed)
    return RefModel(action_dim)


def flat_params(model: nn.Module) -> np.ndarray:
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()]).numpy().copy()


def flat_grads(model: nn.Module) -> np.ndarray:
    return torch.cat([p.grad.detach().reshape(-1) for p in model.parameters()]).numpy().copy()


def load_flat(model: nn.Module, flat: np.ndarray) -> None:
    off = 0
    with torch.no_grad():
        for p in model.parameters():
            n = p.numel()
            p.copy_(torch.from_numpy(np.ascontiguousarray(flat[off:off + n])).reshape(p.shape))
            off += n
    assert off == flat.size


def batched_vtrace(*args, **kw):
    """agents/impala/learning.py:15-26: vmap over the batch dim (loop fallback)."""
    if _vmap is not None:
        try:
            return _vmap(lambda *a: vtrace_td_error_and_advantage(*a, **kw))(*args)
        except Exception:  # pragma: no cover - same fallback as the reference
            pass
    outs = [vtrace_td_error_and_advantage(*[a[i] for a in args], **kw)
            for i in range(args[0].shape[0])]
    return tuple(torch.stack(x) for x in zip(*outs))


def collate(batch: Sequence[Sequence[torch.Tensor]]):
    """learning.py:142: ``collate_nested(lambda x: torch.stack(x).squeeze(dim=-1), batch)``."""
    return [torch.stack([item[j] for item in batch]).squeeze(dim=-1) for j in range(len(batch[0]))]


def train_step(model: nn.Module, optimizer: torch.optim.Optimizer, batch,
               max_grad_norm: float = 0.5, entropy_coeff: float = 0.01,
               collated: bool = False, capture: Optional[dict] = None,
               grad_mode: str = DEFAULT_GRAD_MODE) -> Dict[str, torch.Tensor]:
    """agents/impala/learning.py:140-177 restated. ``batch`` = list of B trajectories
    ``[s u8 (T,3,64,64), a i64 (T,1), r f32 (T,1), g f32 (T,1), mu f32 (T,A)]``
    (format of ``ImpalaActor._make_replay``, learning.py:77-80), or already-collated
    ``(s, a, r, g, mu)`` tensors when ``collated``.  ``capture`` (a dict) receives the step's
    intermediate values: logits, values, rho, and the V-trace adv / err / q.  ``grad_mode``:
    the V-trace gradient semantics (oracle/vtrace.py GRAD_MODES)."""
    optimizer.zero_grad(set_to_none=True)
    s, a, r, discount_t, pi_ref = batch if collated else collate(batch)
    pi, values = model.forward(s.flatten(0, 1))
    pi = pi.reshape(s.shape[0], s.shape[1], -1)
    values = values.reshape(s.shape[0], s.shape[1])
    pi = torch.distributions.Categorical(logits=pi)
    pi_ref = torch.distributions.Categorical(logits=pi_ref)
    rho_tm1 = torch.exp(pi.log_prob(a) - pi_ref.log_prob(a))
    adv, err, q = batched_vtrace(values[:, :-1], values[:, 1:], r[:, :-1],
                                 discount_t[:, :-1], rho_tm1[:, :-1], **mode_kwargs(grad_mode))
    if capture is not None:
        capture.update(logits=pi.logits.detach().clone(), values=values.detach().clone(),
                       rho=rho_tm1.detach().clone(), adv=adv.detach().clone(),
                       err=err.detach().clone(), q=q.detach().clone())
    pg_loss = (pi.log_prob(a)[:, :-1] * adv).mean()
    value_loss = err.pow(2).mean()
    entropy_loss = pi.entropy().mean()
    loss = - pg_loss + value_loss - entropy_coeff * entropy_loss
    loss.backward()
    metrics = {
        "train/loss": loss.detach(),
        "train/entropy": entropy_loss.detach(),
        "train/td": value_loss.detach(),
        "train/pg": pg_loss.detach(),
        "train/kl": torch.distributions.kl_divergence(pi, pi_ref).mean().detach(),
        "train/ratio": rho_tm1.mean().detach(),
    }
    grad_norm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_grad_norm)
    metrics["train/grad_norm"] = grad_norm
    optimizer.step()
    return metrics


def train_step_fp64(flat: np.ndarray, batch_np, A: int = 15, steps: int = 1,
                    capture: Optional[dict] = None, grad_mode: str = DEFAULT_GRAD_MODE,
                    metrics_each: Optional[list] = None):
    """The same step in float64 (model, batch floats, autograd, Adam): the exact-arithmetic
    yardstick against which both the fp32 oracle and the HIP fp32 path are measured.
    -> (final flat params, flat post-clip grads (p.grad after clip_grad_norm_) of the last step, metrics of the last step).
    ``metrics_each`` (a list) receives every step's metrics as floats."""
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        ref = RefModel(A).double()
        with torch.no_grad():
            off = 0
            for p in ref.parameters():
                n = p.numel()
                p.copy_(torch.from_numpy(np.asarray(flat[off:off + n], np.float64)).reshape(p.shape))
                off += n
        opt = make_optimizer(ref)
        obs, act, rew, disc, mu = batch_np
        b = [torch.from_numpy(obs), torch.from_numpy(act),
             torch.from_numpy(rew.astype(np.float64)), torch.from_numpy(disc.astype(np.float64)),
             torch.from_numpy(mu.astype(np.float64))]
        for _ in range(steps):
            met = train_step(ref, opt, b, collated=True, capture=capture, grad_mode=grad_mode)
            if metrics_each is not None:
                metrics_each.append({k: float(v) for k, v in met.items()})
        grads = torch.cat([p.grad.detach().reshape(-1) for p in ref.parameters()]).numpy().copy()
        params = torch.cat([p.detach().reshape(-1) for p in ref.parameters()]).numpy().copy()
        return params, grads, {k: float(v) for k, v in met.items()}
    finally:
        torch.set_default_dtype(prev)


def local_grads(model: nn.Module, batch_collated, entropy_coeff: float = 0.01,
                grad_mode: str = DEFAULT_GRAD_MODE) -> np.ndarray:
    """Loss + backward only (learning.py:141-160), no clip / Adam: the per-replica gradient of
    the data-parallel learner (mean over the LOCAL batch)."""
    model.zero_grad(set_to_none=True)
    s, a, r, discount_t, pi_ref = batch_collated
    pi, values = model.forward(s.flatten(0, 1))
    pi = torch.distributions.Categorical(logits=pi.reshape(s.shape[0], s.shape[1], -1))
    values = values.reshape(s.shape[0], s.shape[1])
    pim = torch.distributions.Categorical(logits=pi_ref)
    rho = torch.exp(pi.log_prob(a) - pim.log_prob(a))
    adv, err, _ = batched_vtrace(values[:, :-1], values[:, 1:], r[:, :-1], discount_t[:, :-1],
                                 rho[:, :-1], **mode_kwargs(grad_mode))
    loss = -(pi.log_prob(a)[:, :-1] * adv).mean() + err.pow(2).mean() \
        - entropy_coeff * pi.entropy().mean()
    loss.backward()
    return flat_grads(model)


def make_optimizer(model: nn.Module, lr: float = 1e-4, eps: float = 1e-5):
    """agents/impala/builder.py:43-44."""
    return torch.optim.Adam(model.parameters(), lr=lr, eps=eps)


def synthetic_batch(B: int, T: int = 20, A: int = 15, seed: int = 1234):
    """BASELINE.md §3 synthetic rollout: obs u8 uniform; a ~ U[0,A); r ~ N(0,1) clipped
    +-10; g = 0.99*(u>0.05); mu-logits ~ N(0,1).  Returns collated numpy arrays in the
    reference layout (B,T,...) (learning.py:142)."""
    rng = np.random.default_rng(seed)
    obs = rng.integers(0, 256, size=(B, T, 3, 64, 64), dtype=np.uint8)
    act = rng.integers(0, A, size=(B, T), dtype=np.int64)
    rew = np.clip(rng.standard_normal((B, T)), -10, 10).astype(np.float32)
    disc = (0.99 * (rng.random((B, T)) > 0.05)).astype(np.float32)
    mu = rng.standard_normal((B, T, A)).astype(np.float32)
    return obs, act, rew, disc, mu


def to_trajectories(obs, act, rew, disc, mu):
    """Collated arrays -> list of B replay items as stored by learning.py:77-80."""
    return [[torch.from_numpy(obs[b]), torch.from_numpy(act[b]).unsqueeze(-1),
             torch.from_numpy(rew[b]).unsqueeze(-1), torch.from_numpy(disc[b]).unsqueeze(-1),
             torch.from_numpy(mu[b])] for b in range(obs.shape[0])]


def forward_numpy(model: nn.Module, obs_u8: np.ndarray):
    with torch.no_grad():
        lg, v = model(torch.from_numpy(obs_u8))
    return lg.numpy(), v.numpy()


def loss_from_outputs(logits, values, act, rew, disc, mu, entropy_coeff=0.01,
                      lambda_=1.0, clip_rho=1.0, clip_pg_rho=1.0, grad_mode=DEFAULT_GRAD_MODE,
                      dtype=torch.float32):
    """Head-only restatement (learning.py:144-159) given the network outputs, returning
    every intermediate plus the analytic gradient w.r.t. (logits, values) via autograd.
    Used to check the fused V-trace/loss kernel in isolation."""
    npd = np.float64 if dtype == torch.float64 else np.float32
    lg = torch.tensor(np.asarray(logits, npd), dtype=dtype, requires_grad=True)
    v = torch.tensor(np.asarray(values, npd), dtype=dtype, requires_grad=True)
    a = torch.from_numpy(np.asarray(act, dtype=np.int64))
    r = torch.from_numpy(np.asarray(rew, dtype=npd))
    g = torch.from_numpy(np.asarray(disc, dtype=npd))
    pr = torch.from_numpy(np.asarray(mu, dtype=npd))
    pi = torch.distributions.Categorical(logits=lg)
    pim = torch.distributions.Categorical(logits=pr)
    rho = torch.exp(pi.log_prob(a) - pim.log_prob(a))
    adv, err, q = batched_vtrace(v[:, :-1], v[:, 1:], r[:, :-1], g[:, :-1], rho[:, :-1],
                                 lambda_=lambda_, clip_rho_threshold=clip_rho,
                                 clip_pg_rho_threshold=clip_pg_rho, **mode_kwargs(grad_mode))
    pg = (pi.log_prob(a)[:, :-1] * adv).mean()
    vl = err.pow(2).mean()
    ent = pi.entropy().mean()
    loss = -pg + vl - entropy_coeff * ent
    loss.backward()
    kl = torch.distributions.kl_divergence(pi, pim).mean()
    out = dict(adv=adv.detach().numpy(), err=err.detach().numpy(), q=q.detach().numpy(),
               rho=rho.detach().numpy(), loss=float(loss.detach()), pg=float(pg.detach()), td=float(vl.detach()),
               entropy=float(ent.detach()), kl=float(kl.detach()), ratio=float(rho.detach().mean()),
               dlogits=lg.grad.numpy().copy(), dvalues=v.grad.numpy().copy())
    return out


# ------------------------------------------------------------------------------------- PPO
# SURVEY.md §8(f) row 3.  PPOLearner._train_step (agents/ppo/learning.py:131-143) calls
# losses.ppo_loss (losses.py:131-155) with entropy_cost = the learner's entropy_coeff (0.01:
# PPOBuilder.make_learner passes no cfg, agents/ppo/builder.py:44-47), clip_coeff 0.1, then
# backward, clip_grad_norm_(0.5), Adam.step, zero_grad.  Batch = flat transitions:
# s u8 (N,3,64,64), a i64 (N,), v_target f32 (N,), pi_ref logits f32 (N,A).

def ppo_loss(model: nn.Module, batch, entropy_cost: float = 0.01, clip_coeff: float = 0.1):
    """losses.py:131-155 restated."""
    s, a, v_target, pi_ref = batch
    pi_tm1, v_tm1 = model(s)
    pi_tm1 = torch.distributions.Categorical(logits=pi_tm1)
    pi_ref = torch.distributions.Categorical(logits=pi_ref)
    ratio = torch.exp(pi_tm1.log_prob(a) - pi_ref.log_prob(a))
    adv = v_target - v_tm1.squeeze(-1)
    td_loss = 0.5 * adv.pow(2).mean()
    adv = adv.detach()
    pg_loss_1 = -(adv * ratio)
    pg_loss_2 = -torch.clamp(ratio, 1 - clip_coeff, 1 + clip_coeff) * adv
    pg_loss = torch.max(pg_loss_1, pg_loss_2).mean()
    kl = torch.distributions.kl_divergence(pi_tm1, pi_ref).mean().clamp_min(0.)
    entropy = pi_tm1.entropy().mean()
    loss = pg_loss + td_loss - entropy_cost * entropy
    return loss, {
        "train/loss": loss.detach(), "train/entropy": entropy.detach(),
        "train/td": td_loss.detach(), "train/pg": pg_loss.detach(),
        "train/target": v_target.mean().detach(), "train/kl": kl.detach(),
        "train/ratio": ratio.mean().detach(),
    }


def ppo_train_step(model: nn.Module, optimizer: torch.optim.Optimizer, batch,
                   max_grad_norm: float = 0.5, entropy_coeff: float = 0.01,
                   clip_coeff: float = 0.1) -> Dict[str, torch.Tensor]:
    """agents/ppo/learning.py:131-143 restated (the reference zeroes grads after the step)."""
    loss, metrics = ppo_loss(model, batch, entropy_cost=entropy_coeff, clip_coeff=clip_coeff)
    loss.backward()
    metrics["train_step/grad_norm"] = torch.nn.utils.clip_grad_norm_(model.parameters(),
                                                                     max_grad_norm)
    optimizer.step()
    optimizer.zero_grad()
    return metrics


class _Outputs(nn.Module):
    """A 'model' returning fixed (logits, values) leaves, to run ppo_loss on given outputs."""

    def __init__(self, logits, values):
        super().__init__()
        self.lg, self.v = logits, values

    def forward(self, s):
        return self.lg, self.v


def ppo_loss_from_outputs(logits, values, act, target, pi_ref, entropy_coeff=0.01,
                          clip_coeff=0.1):
    """ppo_loss given the network outputs: metrics and d loss / d (logits, values)."""
    lg = torch.tensor(logits, dtype=torch.float32, requires_grad=True)
    v = torch.tensor(values, dtype=torch.float32, requires_grad=True)
    batch = (None, torch.from_numpy(np.asarray(act, dtype=np.int64)),
             torch.from_numpy(np.asarray(target, dtype=np.float32)),
             torch.from_numpy(np.asarray(pi_ref, dtype=np.float32)))
    loss, met = ppo_loss(_Outputs(lg, v), batch, entropy_cost=entropy_coeff,
                         clip_coeff=clip_coeff)
    loss.backward()
    return {k.split("/")[1]: float(x) for k, x in met.items()}, lg.grad.numpy(), v.grad.numpy()


def synthetic_ppo_batch(N: int, A: int = 15, seed: int = 4321, ratio_spread: float = 0.3):
    """Flat PPO transitions: obs u8 uniform, a ~ U[0,A), v_target ~ N(0,1), pi_ref logits
    ~ N(0,1).  (The reference actor's target computation, agents/ppo/learning.py:64-69,
    cannot run: it references an undefined ``values``)"""
    rng = np.random.default_rng(seed)
    obs = rng.integers(0, 256, size=(N, 3, 64, 64), dtype=np.uint8)
    act = rng.integers(0, A, size=(N,), dtype=np.int64)
    tgt = rng.standard_normal(N).astype(np.float32)
    mu = (ratio_spread * rng.standard_normal((N, A))).astype(np.float32)
    return obs, act, tgt, mu
