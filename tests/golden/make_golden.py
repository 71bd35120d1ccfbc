"""Generate the golden fixtures in tests/golden/ FROM THE REFERENCE ITSELF.

Run in the survey container only (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

How the reference is run: ``/root/reference`` is put on ``sys.path`` read-only (no bytecode is
written) and the absent third-party modules are stubbed at their import boundary with
semantics-only shims: ``rlmeta.core.remote.remote_method`` (identity decorator),
``rlmeta.core.model.RemotableModel`` (= ``nn.Module``), ``rlmeta.utils.nested_utils``
(``collate_nested``/``map_nested``/``unbatch_nested``), ``moolib`` and ``envs`` (names only;
unused on the learner path).  ``rlego`` is absent and unpinned; it is
provided by the oracle's restatement ``oracle/vtrace.py`` — so the V-trace arithmetic itself is
"parity unpinned", while the model, collate, loss, autograd, clip and Adam that surround it are
the reference's own code (``agents/impala/learning.py:140-177``,
``models/models.py:61-76``, ``models/common.py:108-158``).

The rlego stub runs under one of the V-trace gradient modes (``oracle/vtrace.py``
``GRAD_MODES``: what rlego's function holds constant -- the forward values are the same in all
three), and the gradient-carrying fixtures are written once per mode, each from the reference
learner running with the matching stub.

Fixtures written (all float32 unless stated):

* ``vtrace_random.npz``  G1: B=64, L=19 random V-trace inputs (rho in [0.1,3], ~5% zero
  discounts) for lambda 1.0 and 0.95, outputs from the float64 numpy restatement.
* ``model_forward.npz``  G2: reference ``AtariPPOModel`` (seed-0 init) flat params, obs
  (2*20 frames), logits, values.
* ``train_step_<mode>.npz``  G3/G4: reference ``ImpalaLearner`` with Adam(1e-4, 1e-5), B=2,
  T=20: three consecutive ``_train_step`` calls on three batches; metrics per step, flat
  post-clip grads and flat params after step 1, flat params after step 3.
* ``head_loss_<mode>.npz``   the loss head alone (learning.py:144-159) at B=64,T=20 on random
  logits/values, with d(loss)/d(logits), d(loss)/d(values) from the reference's autograd.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

from oracle import vtrace as ovt  # noqa: E402


def _install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class Remote:  # rlmeta.core.remote.Remote
        def connect(self):
            pass

    def remote_method(*a, **k):
        def deco(f):
            return f
        return deco

    def collate_nested(fn, batch):
        return [fn([item[j] for item in batch]) for j in range(len(batch[0]))]

    def map_nested(fn, x):
        if isinstance(x, (list, tuple)):
            return type(x)(map_nested(fn, y) for y in x)
        return fn(x)

    def unbatch_nested(fn, batch, n):
        return [[fn(x[i]) for x in batch] for i in range(n)]

    rl = mod("rlmeta")
    core = mod("rlmeta.core")
    rl.core = core
    core.remote = mod("rlmeta.core.remote", Remote=Remote, remote_method=remote_method)
    core.model = mod("rlmeta.core.model", RemotableModel=torch.nn.Module, ModelLike=object)
    core.replay_buffer = mod("rlmeta.core.replay_buffer", ReplayBufferLike=object)
    core.types = mod("rlmeta.core.types", Action=tuple, TimeStep=tuple, NestedTensor=object)
    utils = mod("rlmeta.utils")
    rl.utils = utils
    utils.nested_utils = mod("rlmeta.utils.nested_utils", collate_nested=collate_nested,
                             map_nested=map_nested, unbatch_nested=unbatch_nested)
    mod("moolib", Batcher=object)
    mod("envs", EnvSpec=object)
    def rlego_vtrace(*args, **kw):  # rlego.vtrace_td_error_and_advantage under _MODE
        return ovt.vtrace_td_error_and_advantage(*args, **{**ovt.mode_kwargs(_MODE[0]), **kw})

    mod("rlego", vtrace_td_error_and_advantage=rlego_vtrace)


_MODE = [ovt.DEFAULT_GRAD_MODE]  # the stub's gradient mode (read at every call)


def _import_reference():
    _install_stubs()
    sys.path.insert(0, REF)
    import models.distributed_models as dm  # noqa: E402  (reference)
    import agents.impala.learning as il  # noqa: E402  (reference)
    return dm, il


def _flat(params):
    return torch.cat([p.detach().reshape(-1) for p in params]).numpy().copy()


def _flat_grad(params):
    return torch.cat([p.grad.detach().reshape(-1) for p in params]).numpy().copy()


class _FakeReplay:
    def __init__(self, batches):
        self.batches = list(batches)

    def warm_up(self, n):
        pass

    def sample(self, b):
        return None, self.batches.pop(0), None


class _FakeModel:
    """Wraps the reference AtariPPOModel: forward/parameters from it, push() no-op
    (rlmeta DownstreamModel, utils.py:87-88)."""

    def __init__(self, m):
        self.m = m

    def forward(self, x):
        return self.m.forward(x)

    def parameters(self):
        return self.m.parameters()

    def push(self):
        pass


def gen_vtrace(out):
    rng = np.random.default_rng(7)
    B, L = 64, 19
    v_tm1 = rng.standard_normal((B, L))
    v_t = np.concatenate([v_tm1[:, 1:], rng.standard_normal((B, 1))], axis=1)
    r = np.clip(rng.standard_normal((B, L)), -10, 10)
    g = 0.99 * (rng.random((B, L)) > 0.05)
    rho = rng.uniform(0.1, 3.0, (B, L))
    res = {}
    for tag, lam in (("l100", 1.0), ("l095", 0.95)):
        adv, err, q = ovt.vtrace_numpy(v_tm1, v_t, r, g, rho, lambda_=lam)
        res[f"adv_{tag}"], res[f"err_{tag}"], res[f"q_{tag}"] = adv, err, q
        # torch fp32 form must agree with the float64 numpy form
        tv = [torch.tensor(x, dtype=torch.float32) for x in (v_tm1, v_t, r, g, rho)]
        ta, te, tq = zip(*[ovt.vtrace_td_error_and_advantage(*[x[i] for x in tv], lambda_=lam)
                           for i in range(B)])
        assert np.allclose(torch.stack(ta).numpy(), adv, rtol=1e-4, atol=1e-5)
        assert np.allclose(torch.stack(te).numpy(), err, rtol=1e-4, atol=1e-5)
    np.savez_compressed(os.path.join(out, "vtrace_random.npz"),
                        v_tm1=v_tm1.astype(np.float32), v_t=v_t.astype(np.float32),
                        r=r.astype(np.float32), g=g.astype(np.float32),
                        rho=rho.astype(np.float32),
                        **{k: v.astype(np.float32) for k, v in res.items()})


def _synthetic(B, T, A, seed):
    rng = np.random.default_rng(seed)
    obs = rng.integers(0, 256, size=(B, T, 3, 64, 64), dtype=np.uint8)
    act = rng.integers(0, A, size=(B, T), dtype=np.int64)
    rew = np.clip(rng.standard_normal((B, T)), -10, 10).astype(np.float32)
    disc = (0.99 * (rng.random((B, T)) > 0.05)).astype(np.float32)
    mu = rng.standard_normal((B, T, A)).astype(np.float32)
    return obs, act, rew, disc, mu


def _traj(obs, act, rew, disc, mu):
    return [[torch.from_numpy(obs[b]), torch.from_numpy(act[b]).unsqueeze(-1),
             torch.from_numpy(rew[b]).unsqueeze(-1), torch.from_numpy(disc[b]).unsqueeze(-1),
             torch.from_numpy(mu[b])] for b in range(obs.shape[0])]


def gen_model_and_step(out, dm, il, mode):
    A = 15
    torch.manual_seed(0)
    model = dm.AtariPPOModel((3, 64, 64), A)
    keys = list(model.state_dict().keys())
    params0 = _flat(model.parameters())
    obs, *_ = _synthetic(2, 20, A, 99)
    with torch.no_grad():
        lg, v = model(torch.from_numpy(obs.reshape(-1, 3, 64, 64)))
    if mode == ovt.DEFAULT_GRAD_MODE:
        np.savez_compressed(os.path.join(out, "model_forward.npz"), params=params0,
                            obs=obs.reshape(-1, 3, 64, 64), logits=lg.numpy(),
                            values=v.numpy(), keys=np.array(keys))

    B, T = 2, 20
    batches = [_synthetic(B, T, A, 1234 + i) for i in range(3)]
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, eps=1e-5)  # builder.py:43-44
    learner = il.ImpalaLearner(_FakeModel(model), _FakeReplay([_traj(*b) for b in batches]),
                               opt, batch_size=B)  # builder.py:48-49 (defaults otherwise)
    res = {}
    for i in range(3):
        m = learner.train_step()  # learning.py:119-138 -> _train_step :140-177
        for k in ("train/loss", "train/entropy", "train/td", "train/pg", "train/kl",
                  "train/ratio", "train/grad_norm"):
            res.setdefault(k.split("/")[1], []).append(float(m[k]))
        if i == 0:
            res["grads1"] = _flat_grad(model.parameters())
            res["params1"] = _flat(model.parameters())
    res["params3"] = _flat(model.parameters())
    arrays = {f"obs{i}": b[0] for i, b in enumerate(batches)}
    for i, b in enumerate(batches):
        arrays[f"act{i}"], arrays[f"rew{i}"], arrays[f"disc{i}"], arrays[f"mu{i}"] = b[1:]
    np.savez_compressed(os.path.join(out, f"train_step_{mode}.npz"), params0=params0,
                        **arrays, **{k: np.asarray(v, dtype=np.float32) if isinstance(v, list)
                                     else v for k, v in res.items()})


def gen_head_loss(out, il, mode):
    """learning.py:144-159 given network outputs; autograd grads of the loss."""
    rng = np.random.default_rng(11)
    B, T, A = 64, 20, 15
    logits = (2.0 * rng.standard_normal((B, T, A))).astype(np.float32)
    values = rng.standard_normal((B, T)).astype(np.float32)
    act = rng.integers(0, A, size=(B, T), dtype=np.int64)
    rew = np.clip(rng.standard_normal((B, T)), -10, 10).astype(np.float32)
    disc = (0.99 * (rng.random((B, T)) > 0.05)).astype(np.float32)
    mu = rng.standard_normal((B, T, A)).astype(np.float32)
    lg = torch.tensor(logits, requires_grad=True)
    v = torch.tensor(values, requires_grad=True)
    a = torch.from_numpy(act)
    pi = torch.distributions.Categorical(logits=lg)
    pi_ref = torch.distributions.Categorical(logits=torch.from_numpy(mu))
    rho_tm1 = torch.exp(pi.log_prob(a) - pi_ref.log_prob(a))
    adv, err, q = il.batched_vtrace(v[:, :-1], v[:, 1:], torch.from_numpy(rew)[:, :-1],
                                    torch.from_numpy(disc)[:, :-1], rho_tm1[:, :-1])
    pg = (pi.log_prob(a)[:, :-1] * adv).mean()
    vl = err.pow(2).mean()
    ent = pi.entropy().mean()
    loss = -pg + vl - 0.01 * ent
    loss.backward()
    kl = torch.distributions.kl_divergence(pi, pi_ref).mean()
    np.savez_compressed(os.path.join(out, f"head_loss_{mode}.npz"), logits=logits, values=values,
                        act=act, rew=rew, disc=disc, mu=mu, adv=adv.detach().numpy(),
                        err=err.detach().numpy(), q=q.detach().numpy(),
                        rho=rho_tm1.detach().numpy(),
                        scalars=np.array([float(loss), float(ent), float(vl), float(pg),
                                          float(kl), float(rho_tm1.mean())], np.float32),
                        dlogits=lg.grad.numpy(), dvalues=v.grad.numpy())


def main():
    torch.set_num_threads(max(1, min(8, os.cpu_count() or 1)))
    dm, il = _import_reference()
    gen_vtrace(HERE)
    for mode in ovt.GRAD_MODES:
        _MODE[0] = mode
        gen_head_loss(HERE, il, mode)
        gen_model_and_step(HERE, dm, il, mode)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
