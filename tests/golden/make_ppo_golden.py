"""Generate the PPO golden fixtures in tests/golden/ FROM THE REFERENCE ITSELF (SURVEY.md §8(f)
row 3).  Survey container only (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_ppo_golden.py

The reference is imported read-only with the same import-boundary stubs as make_golden.py;
``losses.ppo_loss`` (losses.py:131-155) and ``PPOLearner`` (agents/ppo/learning.py:78-143) are
the reference's own code and need no rlego.  Fixtures (float32 unless stated):

* ``ppo_head.npz``        ppo_loss on given outputs: N=256 random logits / values, targets and
  behaviour logits spread so both clip branches and in-range ratios occur; the 7 metrics
  (loss, entropy, td, pg, target, kl, ratio) and d loss / d logits, d loss / d values.
* ``ppo_train_step.npz``  PPOLearner with Adam(1e-4, eps 1e-5) (agents/ppo/builder.py:44-47,
  conf/agent/ppo.yaml optimizer), three ``train_step`` calls on three N=16 batches from the
  seed-0 model: the 8 metrics per step, the post-clip grads of step 1 (captured before the
  learner's zero_grad), flat params after steps 1 and 3.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (stubs, fake replay/model, flat helpers)

METRICS = ("train/loss", "train/entropy", "train/td", "train/pg", "train/target", "train/kl",
           "train/ratio", "train_step/grad_norm")


def _import_reference():
    mg._install_stubs()
    sys.path.insert(0, mg.REF)
    import models.distributed_models as dm  # noqa: E402  (reference)
    import losses  # noqa: E402  (reference)
    import agents.ppo.learning as pl  # noqa: E402  (reference)
    return dm, losses, pl


class _Outputs(torch.nn.Module):
    def __init__(self, lg, v):
        super().__init__()
        self.lg, self.v = lg, v

    def forward(self, s):
        return self.lg, self.v


def gen_head(out, losses):
    rng = np.random.default_rng(17)
    N, A = 256, 15
    logits = (1.5 * rng.standard_normal((N, A))).astype(np.float32)
    values = rng.standard_normal((N, 1)).astype(np.float32)
    act = rng.integers(0, A, size=(N,), dtype=np.int64)
    tgt = rng.standard_normal(N).astype(np.float32)
    # behaviour logits = current logits + noise: ratios spread around 1 (both clips + inside)
    mu = (logits + 0.25 * rng.standard_normal((N, A))).astype(np.float32)
    lg = torch.tensor(logits, requires_grad=True)
    v = torch.tensor(values, requires_grad=True)
    loss, met = losses.ppo_loss(_Outputs(lg, v), (None, torch.from_numpy(act),
                                                 torch.from_numpy(tgt), torch.from_numpy(mu)),
                                entropy_cost=0.01)
    loss.backward()
    keys = METRICS[:-1]
    with torch.no_grad():
        ratio = torch.exp(torch.distributions.Categorical(logits=lg).log_prob(torch.from_numpy(act))
                          - torch.distributions.Categorical(logits=torch.from_numpy(mu)).log_prob(
                              torch.from_numpy(act)))
    np.savez_compressed(os.path.join(out, "ppo_head.npz"), logits=logits, values=values,
                        act=act, target=tgt, mu=mu, ratio=ratio.numpy(),
                        scalars=np.array([float(met[k]) for k in keys], np.float32),
                        dlogits=lg.grad.numpy(), dvalues=v.grad.numpy())


class _GradSnapAdam(torch.optim.Adam):
    """Adam that records the (post-clip) grads it is stepped with: PPOLearner zeroes them
    right after optimizer.step() (agents/ppo/learning.py:139-141)."""

    snaps: list

    def step(self, closure=None):
        self.snaps.append(torch.cat([p.grad.detach().reshape(-1) for g in self.param_groups
                                     for p in g["params"]]).numpy().copy())
        return super().step(closure)


class _CallableModel(mg._FakeModel):
    """ppo_loss calls the model (losses.py:133): rlmeta's DownstreamModel is callable."""

    def __call__(self, x):
        return self.forward(x)


def _batch(N, A, seed):
    rng = np.random.default_rng(seed)
    obs = rng.integers(0, 256, size=(N, 3, 64, 64), dtype=np.uint8)
    act = rng.integers(0, A, size=(N,), dtype=np.int64)
    tgt = rng.standard_normal(N).astype(np.float32)
    mu = (0.3 * rng.standard_normal((N, A))).astype(np.float32)
    return obs, act, tgt, mu


def gen_train_step(out, dm, pl):
    A, N = 15, 16
    torch.manual_seed(0)
    model = dm.AtariPPOModel((3, 64, 64), A)
    params0 = mg._flat(model.parameters())
    batches = [_batch(N, A, 2024 + i) for i in range(3)]
    opt = _GradSnapAdam(model.parameters(), lr=1e-4, eps=1e-5)
    opt.snaps = []
    learner = pl.PPOLearner(_CallableModel(model),
                            mg._FakeReplay([[torch.from_numpy(x) for x in b] for b in batches]),
                            opt)  # builder.py:44-47: defaults otherwise
    res = {}
    for i in range(3):
        m = learner.train_step()
        for k in METRICS:
            res.setdefault(k.split("/")[1], []).append(float(m[k]))
        if i == 0:
            res["params1"] = mg._flat(model.parameters())
    res["grads1"] = opt.snaps[0]
    res["params3"] = mg._flat(model.parameters())
    arrays = {}
    for i, b in enumerate(batches):
        arrays[f"obs{i}"], arrays[f"act{i}"], arrays[f"tgt{i}"], arrays[f"mu{i}"] = b
    np.savez_compressed(os.path.join(out, "ppo_train_step.npz"), params0=params0, **arrays,
                        **{k: np.asarray(v, dtype=np.float32) if isinstance(v, list) else v
                           for k, v in res.items()})


def main():
    torch.set_num_threads(max(1, min(8, os.cpu_count() or 1)))
    dm, losses, pl = _import_reference()
    gen_head(HERE, losses)
    gen_train_step(HERE, dm, pl)
    print("PPO golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
