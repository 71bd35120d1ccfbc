"""PPO learner on the shared CNN kernels (BASELINE config 4) against
the reference's own outputs (tests/golden/make_ppo_golden.py) and the oracle.

Tolerances as the IMPALA parity tests: loss head on identical inputs 1e-5 rel; fp32 train
step metrics 1e-4 rel, post-clip grads 1e-3 rel-L2, post-Adam params 1e-6 / 2e-6 abs.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
KEYS = ("loss", "entropy", "td", "pg", "kl", "ratio", "target")


# impala_stage copy paths: the default (obs over 2 SDMA streams, the small fields in one pull
# launch), all SDMA copies, 3 obs streams, and the pull kernel for everything
H2D_MODES = {"default": {},
             "sdma_only": {"IMPALA_H2D_SMALL_PULL": "0"},
             "sdma_3streams": {"IMPALA_H2D_STREAMS": "3"},
             "pull8": {"IMPALA_H2D_KERNEL": "8"}}


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _setup(dev, N, dtype="fp32", A=15, flat=None, **kw):
    from impala_amd.engine import Engine
    from impala_amd.model import AtariPPOModel
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype=dtype, seed=0)
    if flat is not None:
        m.load_flat(flat)
    e = Engine(m, batch_size=N, algo="ppo", **kw)
    m._train_engine = e
    return m, e


def _metrics(e):
    met = e.metrics.cpu().numpy()
    # slots: loss, entropy, td, pg, kl, ratio, grad_norm, step, target
    return dict(loss=met[0], entropy=met[1], td=met[2], pg=met[3], kl=met[4], ratio=met[5],
                grad_norm=met[6], step=met[7], target=met[8])


def test_ppo_loss_head_matches_reference():
    from impala_amd.engine import ppo_loss_head
    dev = _dev()
    d = _load("ppo_head.npz")
    out = ppo_loss_head(_t(d["logits"], dev), _t(d["values"], dev), _t(d["act"], dev),
                        _t(d["target"], dev), _t(d["mu"], dev))
    met = out["metrics"].cpu().numpy()
    # fixture order: loss, entropy, td, pg, target, kl, ratio
    exp = dict(zip(("loss", "entropy", "td", "pg", "target", "kl", "ratio"), d["scalars"]))
    np.testing.assert_allclose(met, [exp[k] for k in KEYS], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(out["dlogits"].cpu().numpy(), d["dlogits"], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(out["dvalues"].cpu().numpy(), d["dvalues"].reshape(-1),
                               rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("N,A,seed", [(1, 15, 1), (37, 6, 2), (300, 15, 3)])
def test_ppo_loss_head_ragged_vs_oracle(N, A, seed):
    from impala_amd.engine import ppo_loss_head
    dev = _dev()
    rng = np.random.default_rng(seed)
    lg = (1.5 * rng.standard_normal((N, A))).astype(np.float32)
    v = rng.standard_normal(N).astype(np.float32)
    a = rng.integers(0, A, N).astype(np.int64)
    t = rng.standard_normal(N).astype(np.float32)
    mu = (lg + 0.3 * rng.standard_normal((N, A))).astype(np.float32)
    met, dl, dv = ref_cpu.ppo_loss_from_outputs(lg, v.reshape(N, 1), a, t, mu)
    out = ppo_loss_head(_t(lg, dev), _t(v, dev), _t(a, dev), _t(t, dev), _t(mu, dev))
    np.testing.assert_allclose(out["metrics"].cpu().numpy(), [met[k] for k in KEYS],
                               rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(out["dlogits"].cpu().numpy(), dl, rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(out["dvalues"].cpu().numpy(), dv.reshape(-1), rtol=1e-5, atol=1e-8)


def test_ppo_train_steps_fp32_match_reference():
    """Three PPOLearner steps (agents/ppo/learning.py:131-143) against the reference."""
    dev = _dev()
    d = _load("ppo_train_step.npz")
    m, e = _setup(dev, 16, flat=d["params0"])
    for i in range(3):
        e.train_step(*[_t(d[f"{k}{i}"], dev) for k in ("obs", "act", "tgt", "mu")])
        met = _metrics(e)
        for k in KEYS + ("grad_norm",):
            np.testing.assert_allclose(met[k], d[k][i], rtol=1e-4, atol=1e-6,
                                       err_msg=f"{k} step {i}")
        assert met["step"] == i + 1
        if i == 0:
            assert _rel_l2(m.flat_grad.cpu().numpy(), d["grads1"]) < 1e-3
            np.testing.assert_allclose(m.flat.cpu().numpy(), d["params1"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(m.flat.cpu().numpy(), d["params3"], rtol=0, atol=2e-6)


@pytest.mark.parametrize("N,A", [(1, 15), (100, 6), (256, 15)])
def test_ppo_train_step_shapes_fp32_vs_oracle(N, A):
    dev = _dev()
    obs, act, tgt, mu = ref_cpu.synthetic_ppo_batch(N, A, seed=N + A)
    m, e = _setup(dev, N, A=A)
    ref = ref_cpu.RefModel(A)
    ref_cpu.load_flat(ref, m.flat.cpu().numpy())
    opt = ref_cpu.make_optimizer(ref)
    exp = ref_cpu.ppo_train_step(ref, opt, [torch.from_numpy(x) for x in (obs, act, tgt, mu)])
    e.train_step(*[_t(x, dev) for x in (obs, act, tgt, mu)])
    met = _metrics(e)
    for k in KEYS:
        np.testing.assert_allclose(met[k], float(exp[f"train/{k}"]), rtol=2e-4, atol=1e-6,
                                   err_msg=k)
    np.testing.assert_allclose(met["grad_norm"], float(exp["train_step/grad_norm"]), rtol=2e-4)
    np.testing.assert_allclose(m.flat.cpu().numpy(), ref_cpu.flat_params(ref), rtol=0, atol=1e-6)


def test_ppo_bf16_tracks_fp32():
    dev = _dev()
    batch = [_t(x, dev) for x in ref_cpu.synthetic_ppo_batch(256, 15, seed=9)]
    mf, ef = _setup(dev, 256, dtype="fp32")
    mb, eb = _setup(dev, 256, dtype="bf16")
    ef.compute_grads(*batch)
    eb.compute_grads(*batch)
    torch.cuda.synchronize()
    gf, gb = mf.flat_grad.cpu().numpy(), mb.flat_grad.cpu().numpy()
    cos = float(np.dot(gf, gb) / (np.linalg.norm(gf) * np.linalg.norm(gb)))
    assert cos > 0.99, cos
    a, b = _metrics(ef), _metrics(eb)
    for k in ("loss", "entropy", "td", "kl", "ratio", "target"):
        np.testing.assert_allclose(b[k], a[k], rtol=5e-2, atol=5e-3, err_msg=k)


def test_ppo_grad_parts_match_whole():
    """The data-parallel two-bucket split works for PPO handles too."""
    dev = _dev()
    batch = [_t(x, dev) for x in ref_cpu.synthetic_ppo_batch(64, 15, seed=5)]
    m, e = _setup(dev, 64)
    e.compute_grads(*batch)
    torch.cuda.synchronize()
    g, met = m.flat_grad.cpu().numpy().copy(), e.metrics.cpu().numpy().copy()
    m2, e2 = _setup(dev, 64)
    e2.compute_grads_part(0, *batch)
    e2.compute_grads_part(1, *batch)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m2.flat_grad.cpu().numpy(), g)
    np.testing.assert_array_equal(e2.metrics.cpu().numpy(), met)
    m3, e3 = _setup(dev, 64)  # three buckets
    for part in (2, 3, 4):
        e3.compute_grads_part(part, *batch)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m3.flat_grad.cpu().numpy(), g)
    np.testing.assert_array_equal(e3.metrics.cpu().numpy(), met)


@pytest.mark.parametrize("h2d", sorted(H2D_MODES))
def test_ppo_host_staging_ring_matches_device_batch(h2d, monkeypatch):
    """impala_stage on a PPO handle (no discounts field): bitwise the same step as the batch
    handed over in HBM, with hipMemcpyAsync or the pull kernel."""
    dev = _dev()
    for k, v in H2D_MODES[h2d].items():
        monkeypatch.setenv(k, v)
    host = [torch.from_numpy(np.ascontiguousarray(x)) for x in ref_cpu.synthetic_ppo_batch(64, 6, seed=8)]
    m1, e1 = _setup(dev, 64, A=6)
    e1.train_step(*[t.to(dev) for t in host])
    m2, e2 = _setup(dev, 64, A=6)
    e2.stage_init(1)
    e2.stage(0, *[t.pin_memory() for t in host])
    e2.train_step(e2.slot_batch(0))
    e2.slot_release(0)
    torch.cuda.synchronize()
    assert torch.equal(m1.flat, m2.flat) and torch.equal(e1.metrics, e2.metrics)


def test_ppo_learner_interface_matches_reference():
    """PPOLearner.train_step (agents/ppo/learning.py:110-143) through the host replay: same
    metric keys, and the step equals the oracle's on the sampled transitions."""
    from impala_amd.model import AtariPPOModel
    from impala_amd.ppo import PPOLearner
    from impala_amd.replay import ReplayBuffer
    dev = _dev()
    N = 32
    obs, act, tgt, mu = ref_cpu.synthetic_ppo_batch(N, 15, seed=12)
    rb = ReplayBuffer(100, seed=0)
    for i in range(N):  # transition items as the reference actor stores them (leading dim 1)
        rb.append([torch.from_numpy(obs[i:i + 1]), torch.from_numpy(act[i:i + 1]),
                   torch.from_numpy(tgt[i:i + 1]), torch.from_numpy(mu[i:i + 1])])
    m = AtariPPOModel((3, 64, 64), 15, device=dev, dtype="fp32", seed=0)
    ref = ref_cpu.RefModel(15)
    ref_cpu.load_flat(ref, m.flat.cpu().numpy())
    learner = PPOLearner(m, rb, torch.optim.Adam(ref.parameters(), lr=1e-4, eps=1e-5),
                         batch_size=N, learning_starts=N)
    learner.prepare()
    assert learner.can_train
    out = learner.train_step()
    keys = {"train/loss", "train/entropy", "train/td", "train/pg", "train/target", "train/kl",
            "train/ratio", "train_step/grad_norm", "debug/replay_sample_per_second",
            "debug/gradient_per_second", "debug/total_time", "debug/forward_dt",
            "debug/update_time"}
    assert set(out) == keys
    # the oracle on the same (uniformly sampled, permuted) transitions: metrics are means, so
    # any permutation of all N transitions gives the same values
    opt = ref_cpu.make_optimizer(ref)
    exp = ref_cpu.ppo_train_step(ref, opt, [torch.from_numpy(x) for x in (obs, act, tgt, mu)])
    for k in keys - {k for k in keys if k.startswith("debug/")}:
        np.testing.assert_allclose(float(out[k]), float(exp[k]), rtol=2e-4, atol=1e-6, err_msg=k)
