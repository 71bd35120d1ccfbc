"""GPU parity at the BASELINE sizes: the whole fp32 learner step on the HIP path against the
oracle (agents/impala/learning.py:140-177 op for op, torch CPU) at C1 (B=8, T=20) and C2 (B=64,
T=20), on the synthetic rollouts of SURVEY.md §8(d).

Three CPU yardsticks, all the same oracle step:
* ``fp64``   -- the step in float64 (oracle ``train_step_fp64``): exact arithmetic for our
  purposes, the truth every fp32 path is measured against;
* ``native`` -- fp32 with torch's native CPU convolutions (oneDNN off);
* ``fp32``   -- fp32 with torch's defaults, i.e. exactly what the reference learner computes.
  At C2 its oneDNN convolution weight gradients are ~1.6e-3 rel-L2 away from float64 (its
  gradient and grad_norm inherit that; C1 is ~1.5e-6), so against it the bound is its own
  measured error.

North_star: "V-trace returns and losses match the reference CPU path within 1e-5 rel fp32".
* V-trace outputs of the step itself -- pg_advantage, td_error, q_estimate [B,T-1] and rho
  [B,T], exported from inside the fused head kernel (impala_set_debug_vtrace) -- within a
  NORMWISE 1e-5: |hip - x| <= 1e-5 * (|x| + rms(x)) per element, rms over the whole output.
  A pure element-wise relative bound cannot hold at the step level: the values the scan runs on
  come out of the fp32 trunk forward (~1e-7..1e-6 relative rounding from its convolutions), and
  advantages / TD errors are differences of such values that cross zero.  The element-wise
  relative error (with a floor of 1e-3 * rms) is printed beside the bound.
* The scan itself, fed its own exported inputs (the values and rho the fused head used), is
  BIT-IDENTICAL to the fp32 restatement's sequential loop (oracle/vtrace.py: the kernel keeps
  the reference's recurrence order, one rounding per operation), and element-wise within 1e-5
  of the fp64 scan with an absolute floor of 1e-6 * rms (|d| <= 1e-5 max(|x|, 0.1 rms)).  A
  pure element-wise 1e-5 is beyond fp32 for this recurrence: the fp32 sequential loop itself
  is 2-5e-5 from fp64 at its smallest outputs (differences that cancel to ~1e-3 rms); both
  figures are printed, and the kernel's must not exceed twice the fp32 loop's.
* Every gradient check runs under each V-trace gradient mode (oracle/vtrace.py GRAD_MODES,
  IMPALA_VTRACE_SG_*), against oracles run in the same mode.
* The loss and every metric within 1e-5 relative of fp64 and native (and of fp32, or of
  twice fp32's own error when that is larger: grad_norm at C2).
* The post-clip gradient within 1e-5 rel-L2 of fp64 (of the fp32 yardsticks: 1e-5 or twice
  their own distance from fp64); parameters after 1 step within 1e-6 of fp64 / native, after 3
  steps within 5e-5 of native (at most 100 parameters beyond 1e-6).
Achieved values: tools/parity_probe.py, profiles/r02a/parity_probe.json.
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu
from oracle.vtrace import DEFAULT_GRAD_MODE, GRAD_MODES

pytestmark = pytest.mark.gpu
NAMES = ("loss", "entropy", "td", "pg", "kl", "ratio", "grad_norm")
RTOL = 1e-5   # north_star bar: V-trace outputs and losses
GRAD_RL2 = 1e-5  # post-clip gradient, rel-L2


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


_CACHE = {}


def _oracle32(flat0, batch, A, native, mode):
    """fp32 oracle: 3 steps, step 1's intermediates captured."""
    with torch.backends.mkldnn.flags(enabled=not native):
        ref = ref_cpu.RefModel(A)
        ref_cpu.load_flat(ref, flat0)
        opt = ref_cpu.make_optimizer(ref)
        tb = [torch.from_numpy(x) for x in batch]
        cap = {}
        met = {k: float(v) for k, v in
               ref_cpu.train_step(ref, opt, tb, collated=True, capture=cap,
                                  grad_mode=mode).items()}
        out = {"met": met, "cap": {k: v.numpy() for k, v in cap.items()},
               "grad": ref_cpu.flat_grads(ref), "p": [ref_cpu.flat_params(ref)]}
        for _ in range(2):
            ref_cpu.train_step(ref, opt, tb, collated=True, grad_mode=mode)
        out["p"].append(ref_cpu.flat_params(ref))
    return out


def _run(B, mode=DEFAULT_GRAD_MODE, T=20, A=15, seed=1234):
    """HIP fp32 step (V-trace exported) and the three CPU yardsticks, all in V-trace gradient
    mode ``mode``; cached per shape and mode (the oracle takes ~0.1-0.7 s per step at C2)."""
    key = (B, mode, T, A, seed)
    if key in _CACHE:
        return _CACHE[key]
    from impala_amd.engine import Engine
    from impala_amd.model import AtariPPOModel
    dev = _dev()
    batch = ref_cpu.synthetic_batch(B, T, A, seed=seed)
    flat0 = ref_cpu.flat_params(ref_cpu.make_model(0, A))
    ys = {"fp32": _oracle32(flat0, batch, A, native=False, mode=mode),
          "native": _oracle32(flat0, batch, A, native=True, mode=mode)}
    cap64 = {}
    p64, g64, met64 = ref_cpu.train_step_fp64(flat0, batch, A, capture=cap64, grad_mode=mode)
    p64_3, _, _ = ref_cpu.train_step_fp64(flat0, batch, A, steps=3, grad_mode=mode)
    ys["fp64"] = {"met": met64, "cap": {k: v.numpy() for k, v in cap64.items()}, "grad": g64,
                  "p": [p64, p64_3]}
    m = AtariPPOModel((3, 64, 64), A, device=dev, dtype="fp32")
    m.load_flat(flat0)
    e = Engine(m, batch_size=B, rollout_length=T, vtrace_grad_mode=mode)
    m._train_engine = e
    dbg = e.debug_vtrace()
    db = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in batch]
    e.train_step(*db)
    torch.cuda.synchronize()
    hip = {"met": e.metrics.cpu().numpy().astype(np.float64),
           "vt": {k: v.cpu().numpy().copy() for k, v in dbg.items()},
           "grad": m.flat_grad.cpu().numpy().copy(), "p": [m.flat.cpu().numpy().copy()],
           "batch": batch}
    e.debug_vtrace(False)
    for _ in range(2):
        e.train_step(*db)
    torch.cuda.synchronize()
    hip["p"].append(m.flat.cpu().numpy().copy())
    hip["step"] = float(e.metrics[7])
    _CACHE[key] = (hip, ys)
    return hip, ys


CONFIGS = [pytest.param(8, id="C1_B8_T20"), pytest.param(64, id="C2_B64_T20")]
MODES = pytest.mark.parametrize("mode", GRAD_MODES)


@pytest.mark.parametrize("B", CONFIGS)
def test_step_vtrace_outputs_match_oracle(B):
    """The V-trace the fused head computed inside the step (not a standalone call) against the
    oracle step's batched_vtrace(values[:, :-1], values[:, 1:], r, g, rho) (learning.py:150) and
    rho (learning.py:148): normwise, |hip - x| <= 1e-5 * (|x| + rms(x)) per element.  The pure
    element-wise relative error (floor 1e-3 * rms) is printed for the record."""
    hip, ys = _run(B)
    for k in ("adv", "err", "q", "rho"):
        got = hip["vt"][k].astype(np.float64)
        for name, y in ys.items():
            want = y["cap"][k].astype(np.float64)
            rms = float(np.sqrt(np.mean(want ** 2)))
            worst = float(np.max(np.abs(got - want) / (np.abs(want) + rms)))
            elem = float(np.max(np.abs(got - want) / np.maximum(np.abs(want), 1e-3 * rms)))
            print(f"B={B} {k} vs {name}: normwise max |d| / (|x| + rms) = {worst:.2e}; "
                  f"element-wise max |d| / max(|x|, 1e-3 rms) = {elem:.2e}")
            assert worst <= RTOL, (k, name, worst)


@pytest.mark.parametrize("B", CONFIGS)
def test_step_vtrace_scan_elementwise_on_its_own_inputs(B):
    """The fused head's V-trace scan on the values and rho the kernel itself used (exported
    beside its outputs): bit-identical to the fp32 restatement's sequential loop
    (oracle/vtrace.py, the rlax equations of learning.py:150-153, numpy float32), and
    element-wise 1e-5 of the fp64 scan with an absolute floor of 1e-6 rms.  The pure
    element-wise error of both the kernel and the fp32 loop is printed; the kernel's must not
    exceed twice the fp32 loop's.  Also prints how far the step's values are from each
    yardstick's: that forward rounding, propagated through the scan, is the whole step-level
    V-trace deviation."""
    from oracle.vtrace import vtrace_numpy
    hip, ys = _run(B)
    vt = hip["vt"]
    v32, rho32 = vt["v"], vt["rho"]
    r32 = np.asarray(hip["batch"][2], dtype=np.float32).reshape(v32.shape)
    g32 = np.asarray(hip["batch"][3], dtype=np.float32).reshape(v32.shape)
    args = (v32[:, :-1], v32[:, 1:], r32[:, :-1], g32[:, :-1], rho32[:, :-1])
    seq32 = vtrace_numpy(*args)
    seq64 = vtrace_numpy(*[a.astype(np.float64) for a in args])
    for k, want32, want in zip(("adv", "err", "q"), seq32, seq64):
        got = vt[k]
        np.testing.assert_array_equal(got, want32, err_msg=f"{k}: kernel vs fp32 sequential loop")
        rms = float(np.sqrt(np.mean(want ** 2)))
        d = np.abs(got.astype(np.float64) - want)
        floored = float(np.max(d / np.maximum(np.abs(want), 0.1 * rms)))
        pure = float(np.max(d / np.abs(want)))
        pure32 = float(np.max(np.abs(want32.astype(np.float64) - want) / np.abs(want)))
        print(f"B={B} scan {k} on its own inputs vs fp64: max |d| / max(|x|, 0.1 rms) = "
              f"{floored:.2e}; pure element-wise {pure:.2e} (fp32 sequential loop: {pure32:.2e})")
        assert floored <= RTOL, (k, floored)
        assert pure <= 2 * pure32 + 1e-12, (k, pure, pure32)
    for name, y in ys.items():
        want = y["cap"]["values"].astype(np.float64)
        rms = float(np.sqrt(np.mean(want ** 2)))
        print(f"B={B} values vs {name}: max |d| {np.max(np.abs(v32 - want)):.2e} "
              f"(rms {rms:.3e}, max |d| / rms {np.max(np.abs(v32 - want)) / rms:.2e})")


def _rel(a, b):
    return abs(a - b) / max(abs(b), 1e-30)


@MODES
@pytest.mark.parametrize("B", CONFIGS)
def test_step_losses_and_metrics_match_oracle(B, mode):
    """loss = -pg + td - 0.01 * entropy and the logged metrics (learning.py:155-170)."""
    hip, ys = _run(B, mode)
    for i, k in enumerate(NAMES):
        got = hip["met"][i]
        x64 = ys["fp64"]["met"]["train/" + k]
        for name, y in ys.items():
            want = y["met"]["train/" + k]
            bound = RTOL
            if name == "fp32":  # the reference's own arithmetic: its error vs float64 counts
                bound = max(RTOL, 2 * _rel(want, x64))
            print(f"B={B} {mode} {k} vs {name}: rel {_rel(got, want):.2e} (bound {bound:.1e})")
            assert _rel(got, want) <= bound, (k, name, got, want)
    assert hip["step"] == 3


@MODES
@pytest.mark.parametrize("B", CONFIGS)
def test_step_gradients_and_params_match_oracle(B, mode):
    """Post-clip gradient (p.grad after clip_grad_norm_, as the learner leaves it) and the
    parameters after 1 and 3 Adam steps, in each V-trace gradient mode."""
    hip, ys = _run(B, mode)
    g = hip["grad"]
    x64 = ys["fp64"]["grad"]
    # float64 is the truth: 1e-5.  The two fp32 yardsticks carry their own rounding (torch's
    # oneDNN convolution gradients ~1e-3 at C2): against them 1e-5 or twice their own distance
    # from float64.  (The gradient is piecewise in the forward values -- ReLU masks -- and with
    # the targets live (sg_none) a pre-activation within fp32 rounding of zero moves it: native
    # fp32 lands 1.0e-4 from float64 at C2, and so did a conv2 run as bf16x3 passes, r04d; the
    # f32-MFMA kernels round that unit as float64 does, 8e-7.)
    own = {n: _rel_l2(ys[n]["grad"], x64) for n in ("native", "fp32")}
    checks = []
    for name in ("fp64", "native", "fp32"):
        y = ys[name]
        rl2 = _rel_l2(g, y["grad"])
        bound = GRAD_RL2 if name == "fp64" else max(GRAD_RL2, 2 * own[name])
        print(f"B={B} {mode} grad vs {name}: rel-L2 {rl2:.2e} (bound {bound:.1e})")
        checks.append((name, rl2, bound))
    for name, rl2, bound in checks:
        assert rl2 <= bound, (name, rl2, bound)
    # parameters after 1 step: within 1e-6 of float64; of the native fp32 oracle within 1e-6
    # or twice its own distance from float64 (its gradient with the targets live, sg_none, is
    # ~1e-4 from float64 where the kernels' is ~1e-6)
    p64 = ys["fp64"]["p"]
    d1 = np.abs(hip["p"][0] - p64[0])
    own1 = float(np.abs(ys["native"]["p"][0] - p64[0]).max())
    dn1 = float(np.abs(hip["p"][0] - ys["native"]["p"][0]).max())
    print(f"B={B} {mode} params step 1: max vs fp64 {d1.max():.2e}, vs native {dn1:.2e} "
          f"(native vs fp64 {own1:.2e})")
    assert d1.max() <= 1e-6, d1.max()
    assert dn1 <= max(1e-6, 2 * own1), (dn1, own1)
    # after 3 steps: Adam turns a rounding-level difference in a near-zero gradient element into
    # an O(lr) move (conv1 runs as three exact bf16 MFMA passes since round 3, the weight
    # gradients since round 4: in round 3, 29 of the 344,496 parameters landed 1e-6..2.1e-5 from
    # the native oracle).  Bounds pinned near the measured values: against float64 max 5e-5 and
    # at most 100 parameters (0.03 %) beyond 1e-6; against native the same or twice native's
    # own distance from float64.
    d3 = np.abs(hip["p"][1] - p64[1])
    n3 = int(np.sum(d3 > 1e-6))
    dn3 = np.abs(hip["p"][1] - ys["native"]["p"][1])
    own3 = np.abs(ys["native"]["p"][1] - p64[1])
    nn3, nown3 = int(np.sum(dn3 > 1e-6)), int(np.sum(own3 > 1e-6))
    print(f"B={B} {mode} params step 3: vs fp64 max {d3.max():.2e}, n > 1e-6 {n3}; vs native max "
          f"{dn3.max():.2e}, n > 1e-6 {nn3} (native vs fp64: max {own3.max():.2e}, n {nown3})")
    assert d3.max() <= 5e-5, d3.max()
    assert n3 <= 100, n3
    assert dn3.max() <= max(5e-5, 2 * own3.max()), (dn3.max(), own3.max())
    assert nn3 <= max(100, 2 * nown3), (nn3, nown3)
    # against torch's default fp32 (its conv gradients off by ~1e-3 at C2): Adam's first
    # steps move a parameter by ~lr * sign(m), so a gradient element near 0 can flip: one lr
    # step everywhere; away from 1e-6 no more often than fp32 itself is away from float64
    frac32 = np.mean(np.abs(ys["fp32"]["p"][0] - ys["fp64"]["p"][0]) > 1e-6)
    for i in range(2):
        d = np.abs(hip["p"][i] - ys["fp32"]["p"][i])
        print(f"B={B} params step {2 * i + 1} vs fp32: max {d.max():.2e}, "
              f"frac > 1e-6 {np.mean(d > 1e-6):.2e} (fp32 vs fp64 step 1: {frac32:.2e})")
        assert d.max() <= 2e-4, d.max()
        if i == 0:
            assert np.mean(d > 1e-6) <= 2 * frac32 + 1e-3, np.mean(d > 1e-6)
