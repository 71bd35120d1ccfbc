"""Generate the SAC golden fixture in tests/golden/ FROM THE REFERENCE ITSELF (SURVEY.md §8(f)
row 4, BASELINE config 5).  Survey container only (``/root/reference`` does not exist on the
GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_sac_golden.py

Runs the reference's ``SACBuilder``-equivalent construction (``models/sac_model.py``
``SoftCritic`` then ``SoftActor``, seed 0; Adam groups as ``agents/sac/builder.py:42-47``
with conf/agent/sac.yaml lrs) and three ``SACLearner.train_step`` calls
(``agents/sac/learning.py:146-193``) on three N=64 batches of a D=17 / K=6 task, with the same
import-boundary stubs as make_golden.py.  ``Normal.rsample`` is the one thing intercepted: it
returns ``loc + eps * scale`` (torch's own formula) with ``eps`` taken from a pre-drawn
standard-normal list, so the fixture records the noise and the GPU path can replay it.

``sac_train_step.npz``: the initial flat actor / critic / target-critic params and
log_alpha, per step the batch, sampler probabilities, the three eps draws and the 11 metrics,
and after step 1 and step 3 the flat actor, critic, target critic, target actor and log_alpha.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402

METRICS = ("train/qf1_loss", "train/qf2_loss", "train/qf1", "train/qf2", "train/qf_loss",
           "train/critic_grad_norm", "train/actor_loss", "train/actor_std",
           "train/actor_grad_norm", "train/alpha_loss", "train/alpha")
D, K, N = 17, 6, 64


def _import_reference():
    mg._install_stubs()
    sys.path.insert(0, mg.REF)
    import models.sac_model as sm  # noqa: E402  (reference)
    import agents.sac.learning as sl  # noqa: E402  (reference)
    return sm, sl


class _Replay:
    def __init__(self, batches):
        self.batches = list(batches)

    def warm_up(self, n):
        pass

    def sample(self, b):
        s, a, r, s1, d, probs = self.batches.pop(0)
        batch = [torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(r).unsqueeze(-1),
                 torch.from_numpy(s1), torch.from_numpy(d).unsqueeze(-1)]
        return None, batch, torch.from_numpy(probs)

    def info(self):
        return 1000, 1000


def main():
    torch.set_num_threads(max(1, min(8, os.cpu_count() or 1)))
    sm, sl = _import_reference()
    torch.manual_seed(0)
    critic = sm.SoftCritic((D,), (K,), alpha=1.0)  # builder.py:60-66 order
    actor = sm.SoftActor((D,), (K,))
    actor.push = lambda: None  # rlmeta DownstreamModel.push (utils.py:87-88)
    c_opt = torch.optim.Adam([{"params": critic.critic.parameters()}, {"params": critic.log_alpha}],
                             lr=0.003, eps=1e-5)
    a_opt = torch.optim.Adam(actor.parameters(), lr=0.0003, eps=1e-5)
    rng = np.random.default_rng(5)
    batches, eps = [], []
    for i in range(3):
        s = rng.standard_normal((N, D)).astype(np.float32)
        a = rng.uniform(-1, 1, (N, K)).astype(np.float32)
        r = rng.standard_normal(N).astype(np.float32)
        s1 = rng.standard_normal((N, D)).astype(np.float32)
        d = rng.random(N) < 0.1
        probs = rng.uniform(0.5, 2.0, N).astype(np.float32) / 1000.0  # prioritised-style weights
        batches.append((s, a, r, s1, d, probs))
        eps.append(rng.standard_normal((3, N, K)).astype(np.float32))
    learner = sl.SACLearner(actor, critic=critic, target_actor=actor, replay_buffer=_Replay(batches),
                            critic_optimizer=c_opt, actor_optimizer=a_opt, batch_size=N,
                            model_push_period=5, learning_starts=0, tune_alpha=True)
    res = {"actor0": mg._flat(actor.parameters()), "critic0": mg._flat(critic.critic.parameters()),
           "target0": mg._flat(critic.target_critic.parameters()),
           "log_alpha0": np.float32(critic.log_alpha.item())}
    queue = []
    orig = torch.distributions.Normal.rsample

    def rsample(self, sample_shape=torch.Size()):
        e = torch.from_numpy(queue.pop(0))
        assert e.shape == self.loc.shape
        return self.loc + e * self.scale

    torch.distributions.Normal.rsample = rsample
    try:
        for i in range(3):
            queue[:] = [eps[i][j] for j in range(3)]
            m = learner.train_step()
            assert not queue
            for k in METRICS:
                res.setdefault(k.split("/")[1], []).append(float(m[k]))
            if i in (0, 2):
                t = i + 1
                res[f"actor{t}"] = mg._flat(actor.parameters())
                res[f"critic{t}"] = mg._flat(critic.critic.parameters())
                res[f"target{t}"] = mg._flat(critic.target_critic.parameters())
                res[f"tactor{t}"] = mg._flat(learner._target_actor.parameters())
                res[f"log_alpha{t}"] = np.float32(critic.log_alpha.item())
    finally:
        torch.distributions.Normal.rsample = orig
    arrays = {}
    for i, (s, a, r, s1, d, probs) in enumerate(batches):
        arrays.update({f"s{i}": s, f"a{i}": a, f"r{i}": r, f"s1{i}": s1, f"d{i}": d,
                       f"probs{i}": probs, f"eps{i}": eps[i]})
    np.savez_compressed(os.path.join(HERE, "sac_train_step.npz"), **arrays,
                        **{k: np.asarray(v, dtype=np.float32) for k, v in res.items()})
    print("SAC golden fixture written to", HERE)


if __name__ == "__main__":
    main()
