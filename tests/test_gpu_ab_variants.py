"""The measured-slower alternative kernels kept for A/B runs (csrc/common.h IMPALA_AB:
fc_fwd_splitk_f32 / fc_fwd_wsplit_f32, fwd_chain_kernel, reduce_adam_kernel, wgrad23r_kernel)
against the default path.  They are compiled into ``libimpala_hip_ab.so`` only
(``python -m impala_amd.build --ab``), so this file runs only when that library is the one
loaded:

    IMPALA_HIP_LIB=$PWD/impala_amd/libimpala_hip_ab.so python -m pytest tests/test_gpu_ab_variants.py -m gpu

The product suite checks instead that libimpala_hip.so refuses the switches
(tests/test_gpu_parity.py::test_product_library_refuses_ab_variants).  Results and timings of
the variants: DESIGN.md §4.0 and §7.
"""
import numpy as np
import pytest
import torch

from impala_amd import _lib
from oracle import ref_cpu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not _lib.LIB_PATH.endswith("_ab.so"),
                                 reason="A/B variants: run with IMPALA_HIP_LIB=<libimpala_hip_ab.so>")]


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _model(dev, dtype="fp32", A=15, seed=0):
    from impala_amd.model import AtariPPOModel
    return AtariPPOModel((3, 64, 64), A, device=dev, dtype=dtype, seed=seed)


def _engine(m, B, T, **kw):
    from impala_amd.engine import Engine
    e = Engine(m, batch_size=B, rollout_length=T, **kw)
    m._train_engine = e
    return e


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fused_update_matches_reduce_then_adam(dtype, monkeypatch):
    """The fused slab reduction + clip + Adam launch (reduce_adam_kernel, world_size 1, opt-in
    IMPALA_FUSED_UPDATE=1) is bitwise equal to reduce_grads + adam at BASELINE config 2's size (B=64, T=20):
    params, post-clip grads, both Adam moments and every metric, over 3 steps."""
    dev = _dev()
    batches = [[_t(x, dev) for x in ref_cpu.synthetic_batch(64, 20, 15, seed=70 + i)]
               for i in range(3)]

    def run():
        m = _model(dev, dtype, seed=0)
        e = _engine(m, 64, 20)
        for b in batches:
            e.train_step(*b)
        torch.cuda.synchronize()
        return [x.cpu().numpy().copy() for x in (m.flat, m.flat_grad, e.exp_avg, e.exp_avg_sq,
                                                 e.metrics)]

    monkeypatch.setenv("IMPALA_FUSED_UPDATE", "1")
    fused = run()
    monkeypatch.setenv("IMPALA_FUSED_UPDATE", "0")
    ref = run()
    for a, b, name in zip(fused, ref, ("params", "grads", "exp_avg", "exp_avg_sq", "metrics")):
        np.testing.assert_array_equal(a, b, err_msg=name)
    assert np.isfinite(fused[4]).all() and fused[4][7] == 3.0  # step counter


@pytest.mark.parametrize("env", [{"IMPALA_FWD_CHAIN": "1"}, {"IMPALA_EARLY_RED": "1"}])
def test_ab_launch_modes_bitwise(env, monkeypatch):
    """The flag-joined trunk + FC forward and the early slab reduction: bit-identical to the
    default launches (bf16, B=8, 3 steps)."""
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
    np.testing.assert_array_equal(base[0], alt[0])
    np.testing.assert_array_equal(base[1], alt[1])


@pytest.mark.parametrize("mode", ["1", "2"])
def test_ab_fp32_fc_forward_split_k(mode, monkeypatch):
    """fp32 FC forward with K split over workgroups (1) or over the waves of a workgroup (2):
    the step's metrics within fp32 rounding of the default 32x32 tiles (C2, 2 steps)."""
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
    monkeypatch.setenv("IMPALA_FC_SPLITK", mode)
    alt = run()
    np.testing.assert_allclose(base[1], alt[1], rtol=1e-5, atol=1e-7)
    assert np.abs(base[0] - alt[0]).max() <= 1e-4
