"""GPU parity: the HIP path (through the C-ABI) against the oracle and the golden fixtures.

Tolerances (fp32 parity mode): V-trace / loss head on identical inputs 1e-5 rel (north_star);
network forward 1e-4 rel (f32 MFMA fma-chain vs MKLDNN summation order); full train step
metrics 1e-5 rel, post-clip gradients 1e-5 relative L2, post-Adam params 1e-6 abs (the
Adam update itself is ~1e-4).  The BASELINE-size (C1, C2) full-step parity, against fp32 and
float64 oracles, is tests/test_gpu_parity_full.py.  bf16 perf mode: bounds stated per test.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu, vtrace as ovt

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


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


# ----------------------------------------------------------------------------- V-trace
@pytest.mark.parametrize("tag,lam", [("l100", 1.0), ("l095", 0.95)])
def test_vtrace_matches_golden(tag, lam):
    from impala_amd.engine import vtrace
    dev = _dev()
    d = _load("vtrace_random.npz")
    adv, err, q = vtrace(*[_t(d[k], dev) for k in ("v_tm1", "v_t", "r", "g", "rho")], lambda_=lam)
    np.testing.assert_allclose(adv.cpu().numpy(), d[f"adv_{tag}"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(err.cpu().numpy(), d[f"err_{tag}"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(q.cpu().numpy(), d[f"q_{tag}"], rtol=1e-5, atol=1e-6)
    # the kernel keeps the fp32 restatement's operation order: bit-identical on these inputs
    seq32 = ovt.vtrace_numpy(*[d[k] for k in ("v_tm1", "v_t", "r", "g", "rho")], lambda_=lam)
    for got, want in zip((adv, err, q), seq32):
        np.testing.assert_array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("B,L", [(1, 1), (3, 7), (5, 19), (2, 33), (4, 64)])
def test_vtrace_ragged_shapes(B, L):
    from impala_amd.engine import vtrace
    dev = _dev()
    rng = np.random.default_rng(B * 100 + L)
    v_tm1 = rng.standard_normal((B, L)).astype(np.float32)
    v_t = rng.standard_normal((B, L)).astype(np.float32)
    r = rng.standard_normal((B, L)).astype(np.float32)
    g = (0.99 * (rng.random((B, L)) > 0.1)).astype(np.float32)
    rho = rng.uniform(0.0, 3.0, (B, L)).astype(np.float32)
    exp = ovt.vtrace_numpy(v_tm1.astype(np.float64), v_t, r, g, rho, lambda_=0.9,
                           clip_rho_threshold=1.2, clip_pg_rho_threshold=0.8)
    got = vtrace(*[_t(x, dev) for x in (v_tm1, v_t, r, g, rho)], lambda_=0.9,
                 clip_rho_threshold=1.2, clip_pg_rho_threshold=0.8)
    for gt, ex in zip(got, exp):
        np.testing.assert_allclose(gt.cpu().numpy(), ex, rtol=1e-5, atol=1e-5)
    seq32 = ovt.vtrace_numpy(v_tm1, v_t, r, g, rho, lambda_=0.9, clip_rho_threshold=1.2,
                             clip_pg_rho_threshold=0.8)
    for gt, ex in zip(got, seq32):  # bit-identical to the fp32 sequential loop
        np.testing.assert_array_equal(gt.cpu().numpy(), ex)


# ----------------------------------------------------------------------------- loss head
@pytest.mark.parametrize("mode", ovt.GRAD_MODES)
def test_loss_head_matches_golden(mode):
    """The loss head against the reference's own autograd (make_golden.py, rlego stubbed in
    each V-trace gradient mode)."""
    from impala_amd.engine import loss_head
    dev = _dev()
    d = _load(f"head_loss_{mode}.npz")
    out = loss_head(*[_t(d[k], dev) for k in ("logits", "values", "act", "rew", "disc", "mu")],
                    grad_mode=mode)
    # O(1) quantities: 1e-5 rel + 1e-6 abs (a few fp32 ulps near zero)
    for k, atol in (("adv", 1e-6), ("err", 1e-6), ("q", 1e-6), ("rho", 1e-6)):
        np.testing.assert_allclose(out[k].cpu().numpy(), d[k], rtol=1e-5, atol=atol, err_msg=k)
    np.testing.assert_allclose(out["metrics"].cpu().numpy(), d["scalars"], rtol=1e-5)
    # gradients, O(1e-4): 1e-5 rel + 1e-9 abs of the reference's fp32 autograd, plus that
    # reference's own distance from float64 (the same loss in float64 on the fixture's inputs:
    # sg_none sums the scan's adjoint in another order); and against float64 no further than
    # 1e-5 rel + 1e-9 or twice the reference's own distance
    x64 = ref_cpu.loss_from_outputs(*[d[k] for k in ("logits", "values", "act", "rew", "disc",
                                                     "mu")], grad_mode=mode, dtype=torch.float64)
    for k in ("dlogits", "dvalues"):
        got, ref, exact = out[k].cpu().numpy().astype(np.float64), d[k].astype(np.float64), x64[k]
        tol = 1e-5 * np.abs(ref) + 1e-9 + np.abs(ref - exact)
        assert np.all(np.abs(got - ref) <= tol), (k, float(np.max(np.abs(got - ref) - tol)))
        t64 = 1e-5 * np.abs(exact) + 1e-9
        own = float(np.max(np.abs(ref - exact) / t64))
        r = float(np.max(np.abs(got - exact) / t64))
        print(f"head {mode} {k}: vs float64 {r:.2f} of 1e-5 rel + 1e-9 (reference fp32: {own:.2f})")
        assert r <= max(1.0, 2 * own), (k, r, own)


@pytest.mark.parametrize("mode", ovt.GRAD_MODES)
@pytest.mark.parametrize("B,T,A", [(1, 2, 1), (3, 5, 6), (2, 33, 15), (1, 64, 4)])
def test_loss_head_edge_shapes(B, T, A, mode):
    """Edge shapes in every V-trace gradient mode: V-trace outputs and metrics against the
    fp32 oracle; the gradients against the fp64 oracle at 1e-5 rel + 1e-8, or twice the fp32
    oracle's own distance from fp64 where that is larger."""
    from impala_amd.engine import loss_head
    dev = _dev()
    rng = np.random.default_rng(B + 10 * T + 100 * A)
    logits = (3 * rng.standard_normal((B, T, A))).astype(np.float32)
    values = rng.standard_normal((B, T)).astype(np.float32)
    act = rng.integers(0, A, (B, T)).astype(np.int64)
    rew = rng.standard_normal((B, T)).astype(np.float32)
    disc = (0.99 * (rng.random((B, T)) > 0.2)).astype(np.float32)
    mu = rng.standard_normal((B, T, A)).astype(np.float32)
    exp = ref_cpu.loss_from_outputs(logits, values, act, rew, disc, mu, grad_mode=mode)
    exp64 = ref_cpu.loss_from_outputs(logits, values, act, rew, disc, mu, grad_mode=mode,
                                      dtype=torch.float64)
    out = loss_head(*[_t(x, dev) for x in (logits, values, act, rew, disc, mu)], grad_mode=mode)
    for k, atol in (("adv", 1e-5), ("err", 1e-5), ("q", 1e-5), ("rho", 1e-6)):
        np.testing.assert_allclose(out[k].cpu().numpy(), exp[k], rtol=1e-5, atol=atol, err_msg=k)
    for k in ("dlogits", "dvalues"):
        x64 = exp64[k]
        tol = 1e-5 * np.abs(x64) + 1e-8
        own = float(np.max(np.abs(exp[k] - x64) / tol))
        got = float(np.max(np.abs(out[k].cpu().numpy() - x64) / tol))
        assert got <= max(1.0, 2 * own), (k, mode, got, own)
    got = out["metrics"].cpu().numpy()
    want = [exp[k] for k in ("loss", "entropy", "td", "pg", "kl", "ratio")]
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-7)


# ----------------------------------------------------------------------------- forward
def _model(dev, dtype="fp32", A=15, flat=None, seed=0):
    from impala_amd.model import AtariPPOModel
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype=dtype, seed=seed)
    if flat is not None:
        m.load_flat(flat)
    return m


def test_seed_init_matches_reference():
    dev = _dev()
    d = _load("model_forward.npz")
    m = _model(dev, seed=0)
    # same RNG stream; torch-CPU trunc_normal_ may differ by 1 ulp across host ISAs
    np.testing.assert_allclose(m.flat.cpu().numpy(), d["params"], rtol=1e-6, atol=1e-9)
    assert list(m.state_dict().keys()) == [str(k) for k in d["keys"]]


def test_forward_fp32_matches_reference():
    dev = _dev()
    d = _load("model_forward.npz")
    m = _model(dev, flat=d["params"])
    lg, v = m(_t(d["obs"], dev))
    np.testing.assert_allclose(lg.cpu().numpy(), d["logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(v.cpu().numpy(), d["values"], rtol=1e-4, atol=1e-5)


def test_forward_bf16_close_to_reference():
    dev = _dev()
    d = _load("model_forward.npz")
    m = _model(dev, "bf16", flat=d["params"])
    lg, v = m(_t(d["obs"], dev))
    assert _rel_l2(lg.cpu().numpy(), d["logits"]) < 3e-2
    assert _rel_l2(v.cpu().numpy(), d["values"]) < 5e-2


@pytest.mark.parametrize("n", [1, 7, 129, 300])
def test_forward_ragged_frames(n):
    dev = _dev()
    rng = np.random.default_rng(n)
    obs = rng.integers(0, 256, (n, 3, 64, 64), dtype=np.uint8)
    ref = ref_cpu.make_model(3)
    m = _model(dev, flat=ref_cpu.flat_params(ref))
    lg, v = m(_t(obs, dev))
    elg, ev = ref_cpu.forward_numpy(ref, obs)
    np.testing.assert_allclose(lg.cpu().numpy(), elg, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(v.cpu().numpy(), ev, rtol=1e-4, atol=1e-5)


# ----------------------------------------------------------------------------- train step
def _engine(m, B, T, **kw):
    from impala_amd.engine import Engine
    e = Engine(m, batch_size=B, rollout_length=T, **kw)
    m._train_engine = e
    return e


@pytest.mark.parametrize("env,mode", [({}, m) for m in ovt.GRAD_MODES] +
                         [({"IMPALA_LNC3_FUSED": "0"}, ovt.DEFAULT_GRAD_MODE),
                          ({"IMPALA_FWD_FUSED": "0"}, ovt.DEFAULT_GRAD_MODE)])
def test_train_steps_fp32_match_reference(env, mode, monkeypatch):
    """Three fp32 steps against the reference's own ImpalaLearner (make_golden.py, rlego
    stubbed in the same V-trace gradient mode), for the default kernels in every mode and each
    unfused variant in the default mode."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    dev = _dev()
    d = _load(f"train_step_{mode}.npz")
    m = _model(dev, flat=d["params0"])
    e = _engine(m, 2, 20, vtrace_grad_mode=mode)
    names = ("loss", "entropy", "td", "pg", "kl", "ratio", "grad_norm")
    for i in range(3):
        batch = [_t(d[f"{k}{i}"], dev) for k in ("obs", "act", "rew", "disc", "mu")]
        e.train_step(*batch)
        met = e.metrics.cpu().numpy()
        np.testing.assert_allclose(met[:7], [d[k][i] for k in names], rtol=1e-5, atol=1e-7,
                                   err_msg=f"metrics step {i}")
        assert met[7] == i + 1
        if i == 0:
            assert _rel_l2(m.flat_grad.cpu().numpy(), d["grads1"]) < 1e-5
            np.testing.assert_allclose(m.flat.cpu().numpy(), d["params1"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(m.flat.cpu().numpy(), d["params3"], rtol=0, atol=2e-6)


def _oracle_step(flat, batch_np, A=15):
    ref = ref_cpu.RefModel(A)
    ref_cpu.load_flat(ref, flat)
    opt = ref_cpu.make_optimizer(ref)
    obs, act, rew, disc, mu = batch_np
    met = ref_cpu.train_step(ref, opt, [torch.from_numpy(x) for x in batch_np], collated=True)
    return ref, {k: float(v) for k, v in met.items()}


@pytest.mark.parametrize("B,T,A", [(1, 2, 15), (3, 7, 6), (5, 20, 15)])
def test_train_step_edge_shapes_fp32(B, T, A):
    dev = _dev()
    batch = ref_cpu.synthetic_batch(B, T, A, seed=B * T + A)
    ref0 = ref_cpu.make_model(1, A)
    flat0 = ref_cpu.flat_params(ref0)
    ref, met = _oracle_step(flat0, batch, A)
    m = _model(dev, A=A, flat=flat0)
    e = _engine(m, B, T)
    e.train_step(*[_t(x, dev) for x in batch])
    got = e.metrics.cpu().numpy()
    names = ("loss", "entropy", "td", "pg", "kl", "ratio", "grad_norm")
    # against float64 at 1e-5; against the fp32 oracle at 1e-5 or twice the fp32 oracle's own
    # error vs float64 where that is larger (grad_norm at B=1, T=2: ~5e-6)
    p64, g64, met64 = ref_cpu.train_step_fp64(flat0, batch, A)
    for i, k in enumerate(names):
        x32, x64 = met["train/" + k], met64["train/" + k]
        assert abs(got[i] - x64) <= 1e-5 * abs(x64) + 1e-7, (k, got[i], x64)
        bound = max(1e-5, 2 * abs(x32 - x64) / abs(x64))
        assert abs(got[i] - x32) <= bound * abs(x32) + 1e-7, (k, got[i], x32)
    assert _rel_l2(m.flat_grad.cpu().numpy(), g64) < 1e-5
    np.testing.assert_allclose(m.flat.cpu().numpy(), ref_cpu.flat_params(ref), atol=1e-6)


def test_train_step_bf16_tracks_reference():
    dev = _dev()
    d = _load(f"train_step_{ovt.DEFAULT_GRAD_MODE}.npz")
    m = _model(dev, "bf16", flat=d["params0"])
    e = _engine(m, 2, 20)
    batch = [_t(d[f"{k}0"], dev) for k in ("obs", "act", "rew", "disc", "mu")]
    e.train_step(*batch)
    met = e.metrics.cpu().numpy()
    names = ("loss", "entropy", "td", "pg", "kl", "ratio", "grad_norm")
    exp = np.array([d[k][0] for k in names])
    assert np.all(np.abs(met[:7] - exp) <= 5e-2 * np.abs(exp) + 5e-3), (met, exp)
    g, gr = m.flat_grad.cpu().numpy(), d["grads1"]
    cos = float(np.dot(g, gr) / (np.linalg.norm(g) * np.linalg.norm(gr)))
    assert cos > 0.99, cos


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_train_step_deterministic(dtype):
    dev = _dev()
    batch = [_t(x, dev) for x in ref_cpu.synthetic_batch(8, 20, 15, seed=5)]
    flats = []
    for _ in range(2):
        m = _model(dev, dtype, seed=0)
        e = _engine(m, 8, 20)
        for _ in range(2):
            e.train_step(*batch)
        torch.cuda.synchronize()
        flats.append((m.flat.cpu().numpy().copy(), e.metrics.cpu().numpy().copy()))
    np.testing.assert_array_equal(flats[0][0], flats[1][0])
    np.testing.assert_array_equal(flats[0][1], flats[1][1])


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_step_clock(dtype):
    """The device step clock (impala_step_clock): clocked steps are bitwise the unclocked ones,
    every step gets a positive interval, the intervals tile the region (their sum is within the
    wall time of the synced region), and a full clock ignores extra steps."""
    import time
    dev = _dev()
    batch = [_t(x, dev) for x in ref_cpu.synthetic_batch(8, 20, 15, seed=5)]
    flats = []
    for clocked in (False, True):
        m = _model(dev, dtype, seed=0)
        e = _engine(m, 8, 20)
        e.train_step(*batch)
        torch.cuda.synchronize()
        if clocked:
            e.step_clock_start(3)
        t0 = time.perf_counter()
        for _ in range(4):  # one step past the clock's capacity
            e.train_step(*batch)
        if clocked:
            e.step_clock_end()
        torch.cuda.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3
        if clocked:
            ms = e.step_clock_read()
            assert len(ms) == 3 and all(0 < x < wall_ms for x in ms), (ms, wall_ms)
            assert sum(ms) < wall_ms
        flats.append((m.flat.cpu().numpy().copy(), e.metrics.cpu().numpy().copy()))
    np.testing.assert_array_equal(flats[0][0], flats[1][0])
    np.testing.assert_array_equal(flats[0][1], flats[1][1])


@pytest.mark.parametrize("var", ["IMPALA_FC_SPLITK", "IMPALA_FWD_CHAIN", "IMPALA_FUSED_UPDATE",
                                 "IMPALA_EARLY_RED"])
def test_product_library_refuses_ab_variants(var, monkeypatch):
    """The measured-slower alternatives are compiled into the A/B library only
    (tests/test_gpu_ab_variants.py runs them against it): the product library refuses the switch
    at create, loudly, instead of silently running the default path."""
    from impala_amd import _lib
    if _lib.LIB_PATH.endswith("_ab.so"):
        pytest.skip("the A/B library is loaded")
    dev = _dev()
    monkeypatch.setenv(var, "1")
    with pytest.raises(RuntimeError, match="A/B variant"):
        _engine(_model(dev, "fp32", seed=0), 8, 20)
    if var == "IMPALA_FC_SPLITK":  # an fp32-only variant: bf16 handles ignore the switch
        _engine(_model(dev, "bf16", seed=0), 8, 20).close()
    else:
        with pytest.raises(RuntimeError, match="A/B variant"):
            _engine(_model(dev, "bf16", seed=0), 8, 20)


@pytest.mark.parametrize("env,exact", [({"IMPALA_GRAPH": "1"}, True),
                                       ({"IMPALA_FC_DIRECT": "1"}, False),
                                       ({"IMPALA_FC_MERGED": "0"}, True),
                                       ({"IMPALA_WG23_MERGED": "0"}, True),
                                       ({"IMPALA_C3_TAIL": "0"}, True),
                                       ({"IMPALA_LC12": "0"}, True),
                                       ({"IMPALA_SIDE_STREAM": "1"}, True),
                                       ({"IMPALA_FWD_FUSED": "0"}, True),
                                       ({"IMPALA_LNC3_FUSED": "0"}, False)])
def test_launch_modes_agree(env, exact, monkeypatch):
    """hipGraph replay (opt-in), the single-stream schedule and the unfused conv1/conv2 forward
    give bit-identical steps to the default; the unfused LayerNorm backward sums its per-frame
    reductions in another order, so it agrees to fp32 rounding (params after 3 Adam steps)."""
    dev = _dev()
    batch = [_t(x, dev) for x in ref_cpu.synthetic_batch(8, 20, 15, seed=6)]

    def run():
        m = _model(dev, "bf16", seed=0)
        e = _engine(m, 8, 20)
        for _ in range(3):
            e.train_step(*batch)
        torch.cuda.synchronize()
        return m.flat.cpu().numpy().copy(), e.metrics.cpu().numpy().copy()

    base = run()
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    alt = run()
    if exact:
        np.testing.assert_array_equal(base[0], alt[0])
        np.testing.assert_array_equal(base[1], alt[1])
    else:
        # Adam's normalised update (lr 1e-4) turns rounding in a near-zero gradient into an
        # O(lr) parameter difference: bound every param by one lr step, and require all but
        # 0.1% of them to agree to 1e-5.
        np.testing.assert_allclose(base[0], alt[0], rtol=0, atol=1e-4)
        assert np.mean(np.abs(base[0] - alt[0]) > 1e-5) < 1e-3
        # step-3 metrics come from those diverged bf16 params: pg (near 0) and grad_norm move
        # by ~1e-3; the fp32 oracle test above checks the unfused path exactly
        np.testing.assert_allclose(base[1], alt[1], rtol=1e-2, atol=3e-3)


@pytest.mark.parametrize("env", [{"IMPALA_GRAPH": "1"}, {"IMPALA_FC_MERGED": "0"},
                                 {"IMPALA_WG23_MERGED": "0"}, {"IMPALA_C3_TAIL": "0"},
                                 {"IMPALA_LC12": "0"}, {"IMPALA_SIDE_STREAM": "1"},
                                 {"IMPALA_FWD_FUSED": "0"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_launch_modes_agree_fp32(env, monkeypatch):
    """The fp32 headline path (the reference's arithmetic): every fused / merged launch --
    the conv3 + LayerNorm tail of the forward, the fused per-frame backward, the merged FC and
    conv weight-gradient launches -- is bit-identical to the separate kernels it replaces, at
    C2's frame run (B=64, T=20: 5 frames per workgroup, the fp32 tail's limit).
    One exception: the fused forward computes conv2's last 4 output pixels on 4x4x1 MFMA blocks
    whose four k-phases are summed at the end, the unfused gemm_tile conv2 in one k-ordered
    chain, so IMPALA_FWD_FUSED=0 agrees to fp32 rounding: after two Adam steps every parameter
    within one lr step (1e-4; Adam's normalised update turns rounding in a near-zero gradient
    into an O(lr) move) and all but 0.1 % within 1e-7; metrics within 1e-5 relative."""
    dev = _dev()
    batch = [_t(x, dev) for x in ref_cpu.synthetic_batch(64, 20, 15, seed=16)]

    def run():
        m = _model(dev, "fp32", seed=0)
        e = _engine(m, 64, 20)
        for _ in range(2):
            e.train_step(*batch)
        torch.cuda.synchronize()
        return m.flat.cpu().numpy().copy(), e.metrics.cpu().numpy().copy()

    base = run()
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    alt = run()
    assert np.isfinite(base[1]).all()
    if env.get("IMPALA_FWD_FUSED") == "0":
        d = np.abs(base[0] - alt[0])
        print(f"fp32 fused vs unfused forward after 2 steps: max |dp| {d.max():.2e}, "
              f"frac > 1e-7 {np.mean(d > 1e-7):.2e}")
        assert d.max() <= 1e-4
        assert np.mean(d > 1e-7) < 1e-3
        np.testing.assert_allclose(base[1], alt[1], rtol=1e-5, atol=1e-7)
        return
    np.testing.assert_array_equal(base[0], alt[0])
    np.testing.assert_array_equal(base[1], alt[1])


@pytest.mark.parametrize("B,T", [(24, 64), (160, 20)])
def test_merged_launches_at_other_frame_runs(B, T, monkeypatch):
    """The merged / fused launches against the separate ones, bitwise, where the per-workgroup
    frame run differs from C2's 5: N = 1536 (6 frames per workgroup, the conv3 tail's limit)
    and N = 3200 (13: the tail is off, the fused backward and merged GEMMs stay on)."""
    dev = _dev()
    batch = [_t(x, dev) for x in ref_cpu.synthetic_batch(B, T, 15, seed=77)]

    def run():
        m = _model(dev, "bf16", seed=0)
        e = _engine(m, B, T)
        for _ in range(2):
            e.train_step(*batch)
        torch.cuda.synchronize()
        return m.flat.cpu().numpy().copy(), e.metrics.cpu().numpy().copy()

    base = run()
    for k in ("IMPALA_C3_TAIL", "IMPALA_LC12", "IMPALA_WG23_MERGED", "IMPALA_FC_MERGED"):
        monkeypatch.setenv(k, "0")
    alt = run()
    np.testing.assert_array_equal(base[0], alt[0])
    np.testing.assert_array_equal(base[1], alt[1])
    assert np.isfinite(base[1]).all()


def test_full_size_bf16_step_properties():
    """B=64, T=20 (BASELINE config 2): finite, loss decreases on a repeated batch,
    grad norm positive, params move by <= ~lr per step (Adam bound)."""
    dev = _dev()
    batch = [_t(x, dev) for x in ref_cpu.synthetic_batch(64, 20, 15, seed=1234)]
    m = _model(dev, "bf16", seed=0)
    e = _engine(m, 64, 20)
    p0 = m.flat.clone()
    losses = []
    for _ in range(20):
        e.train_step(*batch)
        losses.append(float(e.metrics[0]))
    torch.cuda.synchronize()
    assert np.all(np.isfinite(losses))
    assert losses[-1] < losses[0]
    delta = (m.flat - p0).abs().max().item()
    assert 0 < delta <= 20 * 1e-4 * 3  # Adam: |step| ~ lr (bias-corrected ratio can exceed 1)


def test_bf16_tracks_fp32_over_100_steps_c2():
    """bf16 perf mode (bf16 operands, fp32 accumulation / master weights / Adam) against the
    fp32 parity mode for 100 learner steps at C2 (B=64, T=20) on 4 rotating synthetic batches
    from the same init.  Stated bounds (measured drift in DESIGN.md §2): per-step loss within
    2 % (+0.02 abs) of fp32's, the final parameters within 2 % relative L2 of fp32's, the
    update (final - initial parameters) within 15 % relative L2 of fp32's update, and both
    runs reduce the loss on their batches by the same amount to within 10 %."""
    dev = _dev()
    batches = [[_t(x, dev) for x in ref_cpu.synthetic_batch(64, 20, 15, seed=3000 + i)]
               for i in range(4)]
    runs = {}
    for dtype in ("fp32", "bf16"):
        m = _model(dev, dtype, seed=0)
        e = _engine(m, 64, 20)
        p0 = m.flat.clone()
        losses = []
        for s in range(100):
            e.train_step(*batches[s % 4])
            losses.append(e.metrics[0].clone())
        torch.cuda.synchronize()
        runs[dtype] = (np.array([float(x) for x in losses]), m.flat.cpu().numpy().copy(),
                       (m.flat - p0).cpu().numpy())
    l32, p32, d32 = runs["fp32"]
    l16, p16, d16 = runs["bf16"]
    dl = np.abs(l16 - l32)
    prl2 = _rel_l2(p16, p32)
    upd = _rel_l2(d16, d32)  # drift relative to how far training moved the weights
    print(f"bf16 vs fp32 over 100 C2 steps: max |dloss| {dl.max():.3e} "
          f"(max rel {np.max(dl / np.abs(l32)):.3e}), params rel-L2 {prl2:.3e}, "
          f"update rel-L2 {upd:.3e}, loss fp32 {l32[0]:.4f}->{l32[-4:].mean():.4f} "
          f"bf16 {l16[0]:.4f}->{l16[-4:].mean():.4f}")
    assert np.all(np.isfinite(l16))
    assert np.all(dl <= 2e-2 * np.abs(l32) + 2e-2), dl.max()
    assert prl2 < 2e-2, prl2
    # the update itself (params - init): 7.7e-2 measured (profiles/r03d/parity.log), bound 2x
    assert upd < 0.15, upd
    drop32, drop16 = l32[:4].mean() - l32[-4:].mean(), l16[:4].mean() - l16[-4:].mean()
    assert drop32 > 0 and abs(drop16 - drop32) <= 0.1 * abs(drop32), (drop32, drop16)
