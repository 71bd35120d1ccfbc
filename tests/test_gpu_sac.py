"""SAC learner on the HIP path (BASELINE config 5) against the
reference's own SACLearner (tests/golden/make_sac_golden.py) and the oracle
(oracle/sac_cpu.py), through the C-ABI (include/sac_hip.h).

Tolerances (fp32 parity mode): metrics 1e-4 rel; parameters after Adam / Polyak 2e-6 abs
(critic lr 3e-3, actor lr 3e-4: one Adam step moves a weight by up to ~lr, so 2e-6 is 1e-3 of
an update); log_alpha 1e-6 abs.  Forward heads (policy, act, Q) 1e-5 rel.  bf16 mode tracks
fp32 loosely (metrics 5e-2 rel).  Launch modes (hipGraph replay vs direct) are bitwise equal,
and so are repeated runs.
"""
import os

import numpy as np
import pytest
import torch

from oracle import sac_cpu

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
KEYS = ("qf1_loss", "qf2_loss", "qf1", "qf2", "qf_loss", "critic_grad_norm", "actor_loss",
        "actor_std", "actor_grad_norm", "alpha_loss", "alpha")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _setup(dev, D, K, N, dtype="fp32", actor0=None, critic0=None, la0=0.0, **kw):
    from impala_amd.sac import SACEngine, SoftActor, SoftCritic
    torch.manual_seed(0)
    critic = SoftCritic((D,), (K,), device=dev)
    actor = SoftActor((D,), (K,), device=dev, dtype=dtype)
    if actor0 is not None:
        actor.flat.copy_(torch.from_numpy(actor0).to(dev))
    if critic0 is not None:
        critic.flat.copy_(torch.from_numpy(critic0).to(dev))
        critic.target_flat.copy_(critic.flat)
    critic.la_buf[0] = la0
    tactor = actor.clone_to(dev)
    eng = SACEngine(actor, critic, tactor, batch_size=N, dtype=dtype, **kw)
    actor._train_engine = eng
    critic._engine = eng
    return actor, critic, tactor, eng


def _metrics(eng):
    m = eng.metrics.cpu().numpy()
    return {k: float(m[i]) for i, k in enumerate(KEYS)}


def _oracle(D, K, actor0, critic0, la0=0.0, **kw):
    actor, critic = sac_cpu.make_models(D, K, seed=0)
    sac_cpu.load_flat(list(actor.parameters()), actor0)
    sac_cpu.load_flat(list(critic.critic.parameters()), critic0)
    sac_cpu.load_flat(list(critic.target_critic.parameters()), critic0)
    with torch.no_grad():
        critic.log_alpha.fill_(la0)
    return sac_cpu.SACState(actor, critic, **kw)


def _batch(N, D, K, seed, probs=True):
    rng = np.random.default_rng(seed)
    s, a, r, s1, d = sac_cpu.synthetic_batch(N, D, K, seed)
    p = (rng.uniform(0.5, 2.0, N) / 1000).astype(np.float32) if probs else None
    eps = rng.standard_normal((3, N, K)).astype(np.float32)
    return (s, a, r, s1, d), p, eps


def _run(eng, batch, probs, eps, dev):
    s, a, r, s1, d = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in batch)
    p = None if probs is None else torch.from_numpy(probs).to(dev)
    prio = torch.zeros(s.shape[0], dtype=torch.float32, device=dev)
    eng.train_step(s, a, r, s1, d, probabilities=p, noise=torch.from_numpy(eps).to(dev), priorities=prio)
    torch.cuda.synchronize()
    return prio.cpu().numpy()


def test_sac_train_steps_match_reference():
    """Three SACLearner.train_step calls of the reference (learning.py:146-193), with its
    recorded rsample noise: metrics each step, every parameter set after steps 1 and 3."""
    dev = _dev()
    d = np.load(os.path.join(G, "sac_train_step.npz"), allow_pickle=False)
    actor, critic, tactor, eng = _setup(dev, 17, 6, 64, actor0=d["actor0"], critic0=d["critic0"])
    for i in range(3):
        batch = (d[f"s{i}"], d[f"a{i}"], d[f"r{i}"], d[f"s1{i}"], d[f"d{i}"])
        _run(eng, batch, d[f"probs{i}"], d[f"eps{i}"], dev)
        got = _metrics(eng)
        for k in KEYS:
            np.testing.assert_allclose(got[k], float(d[k][i]), rtol=1e-4, atol=1e-6, err_msg=f"{k} step {i}")
        if i in (0, 2):
            t = i + 1
            np.testing.assert_allclose(actor.flat.cpu().numpy(), d[f"actor{t}"], rtol=0, atol=2e-6)
            np.testing.assert_allclose(critic.flat.cpu().numpy(), d[f"critic{t}"], rtol=0, atol=2e-6)
            np.testing.assert_allclose(critic.target_flat.cpu().numpy(), d[f"target{t}"], rtol=0, atol=2e-6)
            np.testing.assert_allclose(tactor.flat.cpu().numpy(), d[f"tactor{t}"], rtol=0, atol=2e-6)
            np.testing.assert_allclose(float(critic.la_buf[0]), float(d[f"log_alpha{t}"]), atol=1e-6)
    assert int(eng.metrics[11]) == 3


@pytest.mark.parametrize("N,D,K,probs,tune", [(256, 17, 6, True, True), (100, 3, 1, False, True),
                                              (37, 11, 16, True, False), (512, 40, 8, False, True)])
def test_sac_matches_oracle(N, D, K, probs, tune):
    """Ragged batch sizes, 1 and 16 action dims, uniform weights, fixed alpha: 2 steps vs the
    oracle restatement of learning.py:146-265."""
    dev = _dev()
    torch.manual_seed(0)
    a0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=3)[0].parameters())
    c0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=4)[1].critic.parameters())
    actor, critic, tactor, eng = _setup(dev, D, K, N, actor0=a0, critic0=c0, la0=-0.3, tune_alpha=tune)
    st = _oracle(D, K, a0, c0, la0=-0.3, tune_alpha=tune)
    for step in range(2):
        batch, p, eps = _batch(N, D, K, 10 + step, probs)
        prio = _run(eng, batch, p, eps, dev)
        pt = torch.from_numpy(p) if p is not None else torch.ones(N)
        met = sac_cpu.train_step(st, [torch.from_numpy(np.ascontiguousarray(x)) for x in batch], pt,
                                 [torch.from_numpy(eps[j]) for j in range(3)])
        got = _metrics(eng)
        keys = KEYS if tune else KEYS[:9]
        for k in keys:
            np.testing.assert_allclose(got[k], float(met[f"train/{k}"]), rtol=1e-4, atol=1e-5,
                                       err_msg=f"{k} step {step}")
        np.testing.assert_allclose(prio, met["prio"].numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(actor.flat.cpu().numpy(), sac_cpu.flat(st.actor.parameters()), atol=2e-6)
    np.testing.assert_allclose(critic.flat.cpu().numpy(), sac_cpu.flat(st.critic.critic.parameters()), atol=2e-6)
    np.testing.assert_allclose(critic.target_flat.cpu().numpy(),
                               sac_cpu.flat(st.critic.target_critic.parameters()), atol=2e-6)
    np.testing.assert_allclose(tactor.flat.cpu().numpy(), sac_cpu.flat(st.target_actor.parameters()), atol=2e-6)
    np.testing.assert_allclose(float(critic.la_buf[0]), float(st.critic.log_alpha), atol=1e-6)


def test_sac_grads_match_oracle_one_step():
    """Post-clip gradients of the critic and actor steps (the grad buffers) vs autograd."""
    dev = _dev()
    D, K, N = 17, 6, 256
    a0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=5)[0].parameters())
    c0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=6)[1].critic.parameters())
    actor, critic, tactor, eng = _setup(dev, D, K, N, actor0=a0, critic0=c0)
    st = _oracle(D, K, a0, c0)
    batch, p, eps = _batch(N, D, K, 77)
    _run(eng, batch, p, eps, dev)
    # oracle: keep the critic-step grads before the actor step touches them
    w = torch.from_numpy(p).pow(-0.4)
    w.div_(w.max())
    tb = [torch.from_numpy(np.ascontiguousarray(x)) for x in batch]
    loss, _, _ = sac_cpu.critic_loss(st.target_actor, st.critic, tb, w, torch.from_numpy(eps[0]))
    loss.backward()
    torch.nn.utils.clip_grad_norm_(st.critic.parameters(), 40.0)
    gc = torch.cat([q.grad.reshape(-1) for q in st.critic.critic.parameters()]).numpy()
    got = critic.flat_grad.cpu().numpy()
    assert np.linalg.norm(got - gc) / np.linalg.norm(gc) < 1e-4
    st.critic_opt.step()
    loss, _ = sac_cpu.actor_loss(st.actor, st.critic, tb, torch.from_numpy(eps[1]))
    st.actor_opt.zero_grad(set_to_none=True)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(st.actor.parameters(), 40.0)
    ga = torch.cat([q.grad.reshape(-1) for q in st.actor.parameters()]).numpy()
    got = actor.flat_grad.cpu().numpy()
    assert np.linalg.norm(got - ga) / np.linalg.norm(ga) < 1e-4


def test_sac_policy_act_q_forward():
    """SoftActor.forward / policy / act and SoftCritic.forward / target vs the oracle modules."""
    dev = _dev()
    D, K, n = 17, 6, 50
    actor, critic, tactor, eng = _setup(dev, D, K, 64)
    ra, rc = sac_cpu.make_models(D, K, seed=0)
    rng = np.random.default_rng(1)
    s = rng.standard_normal((n, D)).astype(np.float32)
    e = rng.standard_normal((n, K)).astype(np.float32)
    mean, ls = actor(torch.from_numpy(s).to(dev))
    rm, rls = ra(torch.from_numpy(s))
    np.testing.assert_allclose(mean.cpu().numpy(), rm.detach().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ls.cpu().numpy(), rls.detach().numpy(), rtol=1e-5, atol=1e-6)
    act, logp, std = actor.policy(torch.from_numpy(s).to(dev), noise=torch.from_numpy(e).to(dev))
    ract, rlogp, rstd = ra.policy(torch.from_numpy(s), torch.from_numpy(e))
    np.testing.assert_allclose(act.cpu().numpy(), ract.detach().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(logp.cpu().numpy(), rlogp.detach().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(std.cpu().numpy(), rstd.detach().numpy(), rtol=1e-5, atol=1e-6)
    a_det = actor.act(torch.from_numpy(s), 0.)  # eps 0: tanh(mu)
    np.testing.assert_allclose(a_det.numpy(), torch.tanh(rm).detach().numpy(), rtol=1e-5, atol=1e-6)
    a = rng.uniform(-1, 1, (n, K)).astype(np.float32)
    q1, q2 = critic(torch.from_numpy(s).to(dev), torch.from_numpy(a).to(dev))
    r1, r2 = rc(torch.from_numpy(s), torch.from_numpy(a))
    np.testing.assert_allclose(q1.cpu().numpy(), r1.detach().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(q2.cpu().numpy(), r2.detach().numpy(), rtol=1e-5, atol=1e-6)
    t1, _ = critic.target(torch.from_numpy(s).to(dev), torch.from_numpy(a).to(dev))
    np.testing.assert_allclose(t1.cpu().numpy(), r1.detach().numpy(), rtol=1e-5, atol=1e-6)


def test_sac_graph_replay_and_determinism_bitwise():
    dev = _dev()
    D, K, N = 17, 6, 256
    a0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=3)[0].parameters())
    c0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=4)[1].critic.parameters())
    outs = []
    for graph in ("1", "0", "1"):
        os.environ["SAC_GRAPH"] = graph
        try:
            actor, critic, tactor, eng = _setup(dev, D, K, N, actor0=a0, critic0=c0)
        finally:
            os.environ.pop("SAC_GRAPH", None)
        for step in range(3):
            batch, p, eps = _batch(N, D, K, 20 + step)
            _run(eng, batch, p, eps, dev)
        outs.append((actor.flat.cpu().numpy(), critic.flat.cpu().numpy(), eng.metrics.cpu().numpy()))
        eng.close()
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("dtype,N,K", [("fp32", 256, 6), ("bf16", 256, 6), ("fp32", 37, 16),
                                         ("bf16", 100, 1)])
def test_sac_fused_chains_match_per_layer_bitwise(dtype, N, K):
    """The per-row-block chain kernels (sac_fused.h, default) and the one-launch-per-layer
    path (SAC_FUSED=0) give bitwise-identical parameters, gradients, metrics, priorities."""
    dev = _dev()
    D = 17
    a0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=3)[0].parameters())
    c0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=4)[1].critic.parameters())
    outs = []
    for fused in ("1", "0"):
        os.environ["SAC_FUSED"] = fused
        try:
            actor, critic, tactor, eng = _setup(dev, D, K, N, dtype=dtype, actor0=a0, critic0=c0)
        finally:
            os.environ.pop("SAC_FUSED", None)
        prios = []
        for step in range(3):
            batch, p, eps = _batch(N, D, K, 40 + step)
            prios.append(_run(eng, batch, p, eps, dev))
        q1, q2 = critic(torch.from_numpy(batch[0]).to(dev), torch.from_numpy(batch[1]).to(dev))
        pol = actor.policy(torch.from_numpy(batch[0]).to(dev), noise=torch.from_numpy(eps[0]).to(dev))
        outs.append([actor.flat, actor.flat_grad, critic.flat, critic.flat_grad, critic.target_flat,
                     tactor.flat, critic.la_buf, eng.metrics, q1, q2, *pol])
        outs[-1] = [t.cpu().numpy() for t in outs[-1]] + prios
        eng.close()
    for x, y in zip(*outs):
        np.testing.assert_array_equal(x, y)


def test_sac_device_noise_seeded():
    """noise=None: the three rsample blocks come from the device generator keyed by (seed,
    learner step): same seed -> bitwise-equal runs, another seed -> different updates."""
    dev = _dev()
    D, K, N = 17, 6, 256
    batch, p, _ = _batch(N, D, K, 3)
    res = []
    for seed in (11, 11, 12):
        actor, critic, tactor, eng = _setup(dev, D, K, N, seed=seed)
        s, a, r, s1, d = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in batch)
        for _ in range(2):
            eng.train_step(s, a, r, s1, d, probabilities=torch.from_numpy(p).to(dev))
        torch.cuda.synchronize()
        m = _metrics(eng)
        assert all(np.isfinite(v) for v in m.values())
        res.append(actor.flat.cpu().numpy())
        eng.close()
    np.testing.assert_array_equal(res[0], res[1])
    assert not np.array_equal(res[0], res[2])


def test_sac_bf16_tracks_fp32():
    dev = _dev()
    D, K, N = 17, 6, 256
    a0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=3)[0].parameters())
    c0 = sac_cpu.flat(sac_cpu.make_models(D, K, seed=4)[1].critic.parameters())
    res = {}
    for dt in ("fp32", "bf16"):
        actor, critic, tactor, eng = _setup(dev, D, K, N, dtype=dt, actor0=a0, critic0=c0)
        batch, p, eps = _batch(N, D, K, 5)
        _run(eng, batch, p, eps, dev)
        res[dt] = _metrics(eng)
    for k in ("qf1_loss", "qf2_loss", "qf1", "qf2", "actor_loss", "actor_std", "alpha_loss"):
        np.testing.assert_allclose(res["bf16"][k], res["fp32"][k], rtol=5e-2, atol=2e-2, err_msg=k)


def test_sac_sample_uniform_without_replacement():
    dev = _dev()
    from impala_amd.sac import DeviceTransitionReplay
    rb = DeviceTransitionReplay(5000, device=dev, seed=7)
    n = 3000
    rng = np.random.default_rng(0)
    s = torch.from_numpy(rng.standard_normal((n, 5)).astype(np.float32))
    a = torch.from_numpy(rng.standard_normal((n, 2)).astype(np.float32))
    r = torch.arange(n, dtype=torch.float32)
    s1 = s + 1
    d = torch.from_numpy(rng.random(n) < 0.3)
    rb.extend([s, a, r, s1, d])
    assert rb.info() == (5000, n)
    keys, (bs, ba, br, bs1, bd), probs = rb.sample(1024)
    keys = keys.cpu().numpy()
    assert len(np.unique(keys)) == 1024 and keys.min() >= 0 and keys.max() < n
    idx = br.cpu().numpy().astype(np.int64)  # r = the row index
    np.testing.assert_array_equal(idx, keys)
    np.testing.assert_array_equal(bs.cpu().numpy(), s.numpy()[idx])
    np.testing.assert_array_equal(ba.cpu().numpy(), a.numpy()[idx])
    np.testing.assert_array_equal(bs1.cpu().numpy(), s1.numpy()[idx])
    np.testing.assert_array_equal(bd.cpu().numpy(), d.numpy()[idx].astype(np.uint8))
    np.testing.assert_allclose(probs.cpu().numpy(), 1.0 / n)
    # wrap-around: capacity 5000, 3000 more -> keys 3000..5999 stored in slots
    rb.extend([s, a, r + n, s1, d])
    assert rb.info() == (5000, 5000)
    keys2, batch2, _ = rb.sample(256)
    k2 = keys2.cpu().numpy()
    assert len(np.unique(k2)) == 256 and k2.min() >= 1000 and k2.max() < 6000


def test_sac_learner_end_to_end():
    """SACBuilder -> DeviceTransitionReplay -> SACLearner.train_step with the reference's keys."""
    dev = _dev()
    from impala_amd.config import Cfg
    from impala_amd.sac import SACBuilder

    class Space:
        def __init__(self, shape):
            self.shape = shape

    class Spec:
        observation_space = Space((17,))
        action_space = Space((6,))

    cfg = Cfg.wrap({"agent": {"replay_buffer_size": 10000, "batch_size": 256, "push_period": 5,
                              "learning_starts": 1000, "tune_alpha": True, "alpha": 1.0,
                              "exploration_noise": 1.0, "rollout_length": 100,
                              "optimizer": {"eps": 1e-5, "actor_lr": 3e-4, "critic_lr": 3e-3}},
                    "distributed": {"train_device": "cuda:0", "infer_device": "cuda:0"},
                    "training": {"seed": 123}, "learner": {"dtype": "fp32"}})
    b = SACBuilder(cfg)
    actor = b.make_network(Spec())
    rb = b.make_replay()
    learner = b.make_learner(actor, rb)
    rng = np.random.default_rng(0)
    n = 2000
    rb.extend([torch.from_numpy(rng.standard_normal((n, 17)).astype(np.float32)),
               torch.from_numpy(rng.uniform(-1, 1, (n, 6)).astype(np.float32)),
               torch.from_numpy(rng.standard_normal(n).astype(np.float32)),
               torch.from_numpy(rng.standard_normal((n, 17)).astype(np.float32)),
               torch.from_numpy(rng.random(n) < 0.05)])
    learner.prepare()
    for _ in range(3):
        m = learner.train_step()
    keys = {"train/qf1_loss", "train/qf2_loss", "train/qf1", "train/qf2", "train/qf_loss",
            "train/critic_grad_norm", "train/actor_loss", "train/actor_std",
            "train/actor_grad_norm", "train/alpha_loss", "train/alpha", "debug/rb_capacity",
            "debug/replay_sample_per_second", "debug/gradient_per_second", "debug/total_time",
            "debug/sample_dt", "debug/forward_dt", "debug/update_dt"}
    assert set(m) == keys
    assert all(np.isfinite(float(v)) for v in m.values())
    # push() published the actor to the inference copy at step 0 (push period 5)
    act = b.actor_model.act(torch.zeros(4, 17), torch.tensor([0.]))
    assert act.shape == (4, 6) and bool(torch.all(act.abs() <= 1))
