"""Pin the oracle (oracle/ref_cpu.py, oracle/vtrace.py) against fixtures produced by the
reference's own code (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu, vtrace as ovt

G = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def test_param_layout_matches_reference_state_dict():
    d = _load("model_forward.npz")
    keys = [str(k) for k in d["keys"]]
    assert keys == [k for k, _ in ref_cpu.PARAM_SPECS]
    m = ref_cpu.RefModel()
    assert [k for k in m.state_dict().keys()] == keys
    assert sum(int(np.prod(s)) for _, s in ref_cpu.PARAM_SPECS) == 344496 == d["params"].size


def test_forward_matches_reference():
    d = _load("model_forward.npz")
    m = ref_cpu.RefModel()
    ref_cpu.load_flat(m, d["params"])
    lg, v = ref_cpu.forward_numpy(m, d["obs"])
    np.testing.assert_allclose(lg, d["logits"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(v, d["values"], rtol=1e-6, atol=1e-6)


def test_seed0_init_matches_reference():
    d = _load("model_forward.npz")
    m = ref_cpu.make_model(0)
    # bit-exact on the fixture's host; torch's CPU erfinv uses the host libm's log (CPU-dependent
    # ifunc variant), so other hosts differ by 1-2 ulp in ~0.6 % of the weights
    np.testing.assert_allclose(ref_cpu.flat_params(m), d["params"], rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("mode", ovt.GRAD_MODES)
def test_train_steps_match_reference(mode):
    d = _load(f"train_step_{mode}.npz")
    m = ref_cpu.RefModel()
    ref_cpu.load_flat(m, d["params0"])
    opt = ref_cpu.make_optimizer(m)
    names = ("loss", "entropy", "td", "pg", "kl", "ratio", "grad_norm")
    for i in range(3):
        batch = ref_cpu.to_trajectories(d[f"obs{i}"], d[f"act{i}"], d[f"rew{i}"],
                                        d[f"disc{i}"], d[f"mu{i}"])
        met = ref_cpu.train_step(m, opt, batch, grad_mode=mode)
        got = np.array([float(met["train/" + k]) for k in names])
        exp = np.array([d[k][i] for k in names])
        np.testing.assert_allclose(got, exp, rtol=1e-5, atol=1e-6)
        if i == 0:
            np.testing.assert_allclose(ref_cpu.flat_grads(m), d["grads1"], rtol=1e-5, atol=1e-8)
            np.testing.assert_allclose(ref_cpu.flat_params(m), d["params1"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(ref_cpu.flat_params(m), d["params3"], rtol=0, atol=1e-7)


@pytest.mark.parametrize("mode", ovt.GRAD_MODES)
def test_head_loss_matches_reference(mode):
    d = _load(f"head_loss_{mode}.npz")
    out = ref_cpu.loss_from_outputs(d["logits"], d["values"], d["act"], d["rew"], d["disc"],
                                    d["mu"], grad_mode=mode)
    for k in ("adv", "err", "q", "rho", "dlogits", "dvalues"):
        np.testing.assert_allclose(out[k], d[k], rtol=1e-5, atol=1e-7, err_msg=k)
    got = [out[k] for k in ("loss", "entropy", "td", "pg", "kl", "ratio")]
    # 1e-5 (the north-star bar): pg is a mean of mixed-sign terms (0.0071), so the host libm's
    # exp/log (CPU-dependent ifunc variants) moves it by ~2e-6 relative on other hosts
    np.testing.assert_allclose(got, d["scalars"], rtol=1e-5)


@pytest.mark.parametrize("tag,lam", [("l100", 1.0), ("l095", 0.95)])
def test_vtrace_golden(tag, lam):
    d = _load("vtrace_random.npz")
    adv, err, q = ovt.vtrace_numpy(d["v_tm1"].astype(np.float64), d["v_t"], d["r"], d["g"],
                                   d["rho"], lambda_=lam)
    np.testing.assert_allclose(adv, d[f"adv_{tag}"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(err, d[f"err_{tag}"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(q, d[f"q_{tag}"], rtol=1e-5, atol=1e-6)


def test_grad_modes_forward_identical_gradients_differ():
    """The gradient mode changes only what the backward holds constant: the fixtures of the
    three modes share every forward value and differ in the gradients."""
    ds = {m: _load(f"head_loss_{m}.npz") for m in ovt.GRAD_MODES}
    a = ds[ovt.GRAD_MODES[0]]
    for m, d in ds.items():
        for k in ("adv", "err", "q", "rho", "scalars"):
            np.testing.assert_array_equal(d[k], a[k], err_msg=(m, k))
    for k in ("dlogits", "dvalues"):
        assert not np.array_equal(ds["sg_targets"][k], ds["sg_advantage"][k]), k
        assert not np.array_equal(ds["sg_none"][k], ds["sg_targets"][k]), k


def test_vtrace_known_answers():
    rng = np.random.default_rng(3)
    B, L = 5, 12
    v_tm1 = rng.standard_normal((B, L))
    v_t = rng.standard_normal((B, L))
    r = rng.standard_normal((B, L))
    g = np.full((B, L), 0.9)
    # rho == 1, lambda == 1  =>  err_t = n-step return to the end minus v_tm1
    # (telescoping needs v_t[k] == v_tm1[k+1], as in the learner: values[:, 1:])
    v_t2 = np.concatenate([v_tm1[:, 1:], rng.standard_normal((B, 1))], axis=1)
    adv, err, q = ovt.vtrace_numpy(v_tm1, v_t2, r, g, np.ones((B, L)))
    for t in range(L):
        ret = sum((0.9 ** (k - t)) * r[:, k] for k in range(t, L)) + 0.9 ** (L - t) * v_t2[:, L - 1]
        np.testing.assert_allclose(err[:, t], ret - v_tm1[:, t], rtol=1e-10, atol=1e-10)
    # discount == 0  =>  err = r - v_tm1 (rho<=1), adv == err
    rho = rng.uniform(0.2, 1.0, (B, L))
    adv, err, q = ovt.vtrace_numpy(v_tm1, v_t, r, np.zeros((B, L)), rho)
    np.testing.assert_allclose(err, rho * (r - v_tm1), atol=1e-12)
    np.testing.assert_allclose(adv, rho * (r - v_tm1), atol=1e-12)
    # rho == 0  =>  err == 0 and adv == 0
    adv, err, q = ovt.vtrace_numpy(v_tm1, v_t, r, g, np.zeros((B, L)))
    assert np.all(err == 0) and np.all(adv == 0)


# ------------------------------------------------------------------------------------- PPO
PPO_KEYS = ("loss", "entropy", "td", "pg", "target", "kl", "ratio")


def test_ppo_head_matches_reference():
    """ppo_loss (losses.py:131-155) restated vs the reference on given outputs."""
    d = _load("ppo_head.npz")
    met, dl, dv = ref_cpu.ppo_loss_from_outputs(d["logits"], d["values"], d["act"],
                                                d["target"], d["mu"])
    np.testing.assert_allclose([met[k] for k in PPO_KEYS], d["scalars"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(dl, d["dlogits"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(dv, d["dvalues"], rtol=1e-5, atol=1e-9)
    r = d["ratio"]
    assert (r < 0.9).any() and (r > 1.1).any() and ((r >= 0.9) & (r <= 1.1)).any()


def test_ppo_train_steps_match_reference():
    """PPOLearner._train_step (agents/ppo/learning.py:131-143) restated, 3 steps."""
    d = _load("ppo_train_step.npz")
    m = ref_cpu.RefModel()
    ref_cpu.load_flat(m, d["params0"])
    opt = ref_cpu.make_optimizer(m)
    snaps = []
    orig = opt.step

    def step(*a, **k):
        snaps.append(ref_cpu.flat_grads(m))
        return orig(*a, **k)

    opt.step = step
    for i in range(3):
        b = [torch.from_numpy(d[f"{k}{i}"]) for k in ("obs", "act", "tgt", "mu")]
        met = ref_cpu.ppo_train_step(m, opt, b)
        got = [float(met[f"train/{k}"]) for k in PPO_KEYS] + [float(met["train_step/grad_norm"])]
        exp = [float(d[k][i]) for k in PPO_KEYS + ("grad_norm",)]
        np.testing.assert_allclose(got, exp, rtol=1e-5, atol=1e-7, err_msg=f"step {i}")
        if i == 0:
            np.testing.assert_allclose(snaps[0], d["grads1"], rtol=1e-4, atol=1e-8)
            np.testing.assert_allclose(ref_cpu.flat_params(m), d["params1"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(ref_cpu.flat_params(m), d["params3"], rtol=0, atol=1e-7)


# ------------------------------------------------------------------------------------- SAC
SAC_METRICS = ("qf1_loss", "qf2_loss", "qf1", "qf2", "qf_loss", "critic_grad_norm",
               "actor_loss", "actor_std", "actor_grad_norm", "alpha_loss", "alpha")


def _sac_batch(d, i):
    return (torch.from_numpy(d[f"s{i}"]), torch.from_numpy(d[f"a{i}"]), torch.from_numpy(d[f"r{i}"]),
            torch.from_numpy(d[f"s1{i}"]), torch.from_numpy(d[f"d{i}"]))


def test_sac_train_steps_match_reference():
    """SACLearner.train_step (agents/sac/learning.py:146-193) restated, 3 steps, with the
    reference's recorded rsample noise."""
    from oracle import sac_cpu
    d = _load("sac_train_step.npz")
    actor, critic = sac_cpu.make_models(17, 6, seed=0)
    # seed-0 init is the reference's (critic then actor, layer_init_uniform)
    np.testing.assert_array_equal(sac_cpu.flat(actor.parameters()), d["actor0"])
    np.testing.assert_array_equal(sac_cpu.flat(critic.critic.parameters()), d["critic0"])
    np.testing.assert_array_equal(sac_cpu.flat(critic.target_critic.parameters()), d["target0"])
    st = sac_cpu.SACState(actor, critic)
    for i in range(3):
        eps = [torch.from_numpy(d[f"eps{i}"][j]) for j in range(3)]
        met = sac_cpu.train_step(st, _sac_batch(d, i), torch.from_numpy(d[f"probs{i}"]), eps)
        got = [float(met[f"train/{k}"].detach()) for k in SAC_METRICS]
        np.testing.assert_allclose(got, [float(d[k][i]) for k in SAC_METRICS], rtol=1e-5,
                                   atol=1e-6, err_msg=f"step {i}")
        if i in (0, 2):
            t = i + 1
            np.testing.assert_allclose(sac_cpu.flat(actor.parameters()), d[f"actor{t}"], atol=1e-6)
            np.testing.assert_allclose(sac_cpu.flat(critic.critic.parameters()), d[f"critic{t}"],
                                       atol=1e-6)
            np.testing.assert_allclose(sac_cpu.flat(critic.target_critic.parameters()),
                                       d[f"target{t}"], atol=1e-6)
            np.testing.assert_allclose(sac_cpu.flat(st.target_actor.parameters()), d[f"tactor{t}"],
                                       atol=1e-6)
            np.testing.assert_allclose(float(critic.log_alpha), float(d[f"log_alpha{t}"]), atol=1e-7)
