"""ORACLE — test infrastructure only (never shipped, never on the product path).

CPU restatement of the V-trace arithmetic the reference learner calls.

The reference imports it from the third-party package ``rlego``
(``-e git+https://github.com/d3sm0/RLego.git#egg=rlego``, ``requirements.txt:7`` —
**no commit pin**; not installed here, not on disk, not fetchable offline).  Call sites:

* ``agents/impala/learning.py:18``  ``functorch.vmap(rlego.vtrace_td_error_and_advantage)``
* ``agents/impala/learning.py:24``  fallback loop over the batch
* ``agents/impala/learning.py:150-153``  ``adv, err, _ = batched_vtrace(v[:, :-1], v[:, 1:],
  r[:, :-1], discount_t[:, :-1], rho_tm1[:, :-1])``

rlego is a PyTorch port of rlax building blocks, so this restates rlax's published
``vtrace_td_error_and_advantage`` (defaults ``lambda_=1``, ``clip_rho_threshold=1``,
``clip_pg_rho_threshold=1``, ``stop_target_gradients=True``).  The return ORDER is taken
from the reference's four consistent unpackings ``adv, err, _`` (``learning.py:150``,
``losses.py:38,73,106``): ``(pg_advantage, td_error, q_estimate)``.

Gradient semantics (forward values do not depend on them).  rlax's function
stops gradients through the TARGETS only (``stop_target_gradients``); its pg advantage
``min(clip_pg_rho, rho) * (q - v_tm1)`` stays differentiable, and learning.py:148-155 detaches
neither rho nor the advantage.  ``GRAD_MODES`` names the three semantics the HIP learner
implements (``IMPALA_VTRACE_SG_*``); ``mode_kwargs`` maps a name to this function's flags:

* ``sg_advantage`` -- the default: ``stop_target_gradients=True`` and
  ``stop_advantage_gradients=True`` (the latter is not an rlax flag): targets and advantages
  constant, SURVEY.md §8(c)'s restatement (``adv_t = sg(...)``) and the IMPALA paper's
  estimator
* ``sg_targets``   -- ``stop_target_gradients=True`` alone (rlax's function taken literally,
  with the advantage learning.py:155 multiplies in left live)
* ``sg_none``      -- ``stop_target_gradients=False``

Per trajectory, t = 0 .. L-1 (L = T-1 in the learner)::

    c_t      = lambda * min(1, rho_t)
    d_t      = min(clip_rho, rho_t) * (r_t + g_t * v_t[t] - v_tm1[t])
    e_t      = d_t + g_t * c_t * e_{t+1},      e_L = 0           (reverse scan)
    target_t = sg(e_t + v_tm1[t])
    err_t    = target_t - v_tm1[t]
    q_t      = r_t + g_t * (lambda * target_{t+1} + (1 - lambda) * v_tm1[t+1])   t < L-1
    q_{L-1}  = r_{L-1} + g_{L-1} * v_t[L-1]
    adv_t    = min(clip_pg_rho, rho_t) * (q_t - v_tm1[t])     (sg only in sg_advantage)

Parity status: forward values are pinned only by this restatement (SURVEY.md §8(c):
"parity unpinned at the rlego boundary"); everything around it is pinned by the
reference's own code run in this container (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np
import torch


GRAD_MODES = ("sg_advantage", "sg_targets", "sg_none")
DEFAULT_GRAD_MODE = "sg_advantage"


def mode_kwargs(mode: str) -> dict:
    """Gradient-mode name (GRAD_MODES) -> flags of vtrace_td_error_and_advantage."""
    if mode not in GRAD_MODES:
        raise ValueError(f"unknown V-trace gradient mode {mode!r}")
    return {"sg_targets": dict(stop_target_gradients=True),
            "sg_advantage": dict(stop_target_gradients=True, stop_advantage_gradients=True),
            "sg_none": dict(stop_target_gradients=False)}[mode]


def vtrace_td_error_and_advantage(v_tm1, v_t, r_t, discount_t, rho_tm1,
                                  lambda_=1.0, clip_rho_threshold=1.0,
                                  clip_pg_rho_threshold=1.0,
                                  stop_target_gradients=True,
                                  stop_advantage_gradients=False):
    """Single trajectory (1-D tensors of length L).  torch, vmap-compatible.

    Returns ``(pg_advantage, td_error, q_estimate)`` (order per learning.py:150).
    """
    lam = float(lambda_) if lambda_ is not None else 1.0
    c_tm1 = torch.clamp(rho_tm1, max=1.0) * lam
    clipped_rho = torch.clamp(rho_tm1, max=clip_rho_threshold)
    td = clipped_rho * (r_t + discount_t * v_t - v_tm1)
    L = v_tm1.shape[0]
    errs = []
    acc = torch.zeros_like(td[0])
    for i in range(L - 1, -1, -1):
        acc = td[i] + discount_t[i] * c_tm1[i] * acc
        errs.append(acc)
    errs = torch.stack(errs[::-1])
    target = errs + v_tm1
    if stop_target_gradients:
        target = target.detach()
    boot = torch.cat([lam * target[1:] + (1.0 - lam) * v_tm1[1:], v_t[-1:]], dim=0)
    q = r_t + discount_t * boot
    adv = torch.clamp(rho_tm1, max=clip_pg_rho_threshold) * (q - v_tm1)
    if stop_advantage_gradients:
        adv = adv.detach()
    err = target - v_tm1
    return adv, err, q


def vtrace_numpy(v_tm1, v_t, r_t, discount_t, rho_tm1, lambda_=1.0,
                 clip_rho_threshold=1.0, clip_pg_rho_threshold=1.0):
    """Batched (B, L) float64-capable numpy restatement (same equations, explicit loop).

    Used by the known-answer tests and as an independent cross-check of the torch form.
    """
    v_tm1 = np.asarray(v_tm1)
    dt = v_tm1.dtype
    v_t, r_t, g, rho = (np.asarray(x, dtype=dt) for x in (v_t, r_t, discount_t, rho_tm1))
    lam = dt.type(lambda_)
    c = np.minimum(dt.type(1.0), rho) * lam
    td = np.minimum(dt.type(clip_rho_threshold), rho) * (r_t + g * v_t - v_tm1)
    B, L = v_tm1.shape
    e = np.zeros_like(td)
    acc = np.zeros(B, dtype=dt)
    for i in range(L - 1, -1, -1):
        acc = td[:, i] + g[:, i] * c[:, i] * acc
        e[:, i] = acc
    target = e + v_tm1
    boot = np.concatenate([lam * target[:, 1:] + (dt.type(1.0) - lam) * v_tm1[:, 1:],
                           v_t[:, -1:]], axis=1)
    q = r_t + g * boot
    adv = np.minimum(dt.type(clip_pg_rho_threshold), rho) * (q - v_tm1)
    err = target - v_tm1
    return adv, err, q
