// Non-GEMM kernels of the learner step: fused log-softmax / V-trace / loss head, LayerNorm
// forward and backward, gradient-slab reduction, global-norm clip + Adam, weight repacking.
#pragma once
#include "common.h"
#include "conv1.h"
#include "net.h"
#include "ops.h"

using namespace net;

// =========================================================================================
// V-trace (rlax/rlego vtrace_td_error_and_advantage as called through
// agents/impala/learning.py:15-26,150-153), one lane per (trajectory, t) of a wavefront segment
// of S lanes, L = T - 1 live lanes.
//
// Forward order.  Every operation rounds once, in the order of the fp32 restatement
// (oracle/vtrace.py: td = rho' * ((r + g v_t) - v_tm1); acc = td + (g c) * acc; target = acc +
// v_tm1; ...): floating-point contraction is off in these functions, so on identical inputs the
// outputs are bit-identical to the sequential fp32 loop.  The reverse recurrence
// e_t = b_t + a_t e_{t+1} runs as L sweeps over the segment, each lane recomputing its e from
// its neighbour's value of the previous sweep (DPP wave shift): after sweep k the lanes
// t >= L - k hold their final value, computed from the final e_{t+1} -- the sequential loop's
// own operations, so its own rounding (a log-depth composition of the affine maps would sum in
// tree order instead).  L <= 63 sweeps of 3 VALU operations.
//
// Return order (pg_advantage, td_error, q_estimate): taken from the reference's unpacking
// `adv, err, _ =` (learning.py:150); rlax's published VTraceOutput lists (errors,
// pg_advantage, q_estimate).  rlego itself is absent, so this order is an unpinned assumption
// pinned only by the reference's own call sites.
//
// Gradient semantics (IMPALA_VTRACE_SG_*, include/impala_hip.h).  learning.py:148-155 detaches
// neither rho nor the advantage; what is constant depends on rlego:
//   SG_ADVANTAGE (0)  targets and pg advantages constant (the IMPALA paper's estimator)
//   SG_TARGETS   (1)  rlax stop_target_gradients=True: targets constant, the advantage
//                     rho_pg (q - v_tm1) live -- through min(rho_pg, rho) into log pi(a), into
//                     v_tm1 and, via q's bootstrap, into v_t[L-1] ((1 - lambda) v_tm1[t+1])
//   SG_NONE      (2)  stop_target_gradients=False: also through the targets, i.e. the scan
// =========================================================================================
enum : int { VT_SG_ADVANTAGE = 0, VT_SG_TARGETS = 1, VT_SG_NONE = 2 };

DEV float seq_rev_scan(float a, float b, int t, int L) {
#pragma clang fp contract(off)
  const bool live = t < L, nxt = t + 1 < L;
  float e = 0.f;
  for (int k = 0; k < L; ++k) {
    const float en = shift_down1(e);
    e = live ? b + a * (nxt ? en : 0.f) : 0.f;
  }
  return e;
}
// the adjoint of seq_rev_scan: E_t = b_t + a_{t-1} E_{t-1}, E_0 = b_0 (forward in t)
DEV float seq_fwd_scan(float a, float b, int t, int L) {
  const bool live = t < L, prv = t >= 1;
  float E = 0.f;
  for (int k = 0; k < L; ++k) {
    const float p = shift_up1(a * E);
    E = live ? b + (prv ? p : 0.f) : 0.f;
  }
  return E;
}

struct VtLane {
  float a, td, e, tgt, err, q, adv;
};
// v = v_tm1[t], vt = v_t[t], vnx = v_tm1[t + 1] (only read for t < L - 1); lanes t >= L
// produce zeros.  In the learner v_t = values[:, 1:], so vt == vnx == the next lane's v.
DEV VtLane vtrace_lane(float v, float vt, float vnx, float r, float g, float rho, int t, int L,
                       float lam, float crho, float cpg) {
#pragma clang fp contract(off)
  const bool in = t < L;
  VtLane o;
  o.td = in ? fminf(crho, rho) * (r + g * vt - v) : 0.f;
  o.a = in ? g * (fminf(1.f, rho) * lam) : 0.f;
  o.e = seq_rev_scan(o.a, o.td, t, L);
  o.tgt = o.e + v;
  o.err = o.tgt - v;
  const float tgt_n = shift_down1(o.tgt);
  const float boot = (t < L - 1) ? lam * tgt_n + (1.f - lam) * vnx : vt;
  o.q = r + g * boot;
  o.adv = fminf(cpg, rho) * (o.q - v);
  return o;
}

// d loss / d log pi(a_t) and d loss / d v_t of the lane's frame t (t = 0 .. L, the last frame
// only through the bootstrap) for
//   loss = -c_pg sum_t log pi(a_t) adv_t + c_pg sum_t err_t^2 + (entropy term, elsewhere),
// c_pg = 1 / (B (T - 1)) (learning.py:155-159).  Every lane of the wavefront calls it.
struct VtGrad {
  float dlogpa, dv;
};
DEV VtGrad vtrace_grad_lane(const VtLane& o, int mode, float v, float vt, float r, float g,
                            float rho, float logpa, int t, int L, float lam, float crho,
                            float cpg, float c_pg) {
  const bool in = t < L;
  VtGrad d;
  d.dlogpa = in ? -c_pg * o.adv : 0.f;
  float dv = 0.f, dv_nx = 0.f, rbar = 0.f;  // -> v_t, -> v_{t+1}, -> rho_t
  if (mode != VT_SG_NONE) dv = in ? -2.f * c_pg * o.err : 0.f;  // err = sg(target) - v
  if (mode != VT_SG_ADVANTAGE) {
    const float abar = in ? -c_pg * logpa : 0.f;  // d loss / d adv_t
    const float qbar = fminf(cpg, rho) * abar;    // d loss / d q_t
    if (rho <= cpg) rbar += abar * (o.q - v);     // adv = min(cpg, rho) (q - v)
    dv -= qbar;
    dv_nx += (t < L - 1) ? (1.f - lam) * g * qbar : g * qbar;  // q's bootstrap
    if (mode == VT_SG_NONE) {
      // target_t = e_t + v_t enters err_t (whose own -v_t cancels target's +v_t) and q_{t-1}
      const float tq = shift_up1((t < L - 1) ? lam * g * qbar : 0.f);  // from q_{t-1}
      dv += (in && t >= 1) ? tq : 0.f;
      const float ebar = in ? 2.f * c_pg * o.err + (t >= 1 ? tq : 0.f) : 0.f;
      const float E = seq_fwd_scan(o.a, ebar, t, L);  // total adjoint of e_t
      // e_t = td_t + a_t e_{t+1};  td_t = min(crho, rho) (r + g v_{t+1} - v_t);
      // a_t = g min(1, rho) lambda
      const float rc = fminf(crho, rho);
      dv -= rc * E;
      dv_nx += rc * g * E;
      if (rho <= crho) rbar += E * (r + g * vt - v);
      const float e_n = shift_down1(o.e);
      if (rho <= 1.f) rbar += E * ((t + 1 < L) ? e_n : 0.f) * g * lam;
    }
    d.dlogpa += in ? rbar * rho : 0.f;  // rho = exp(log pi(a) - log mu(a))
  }
  const float from_prev = shift_up1(in ? dv_nx : 0.f);
  d.dv = (in ? dv : 0.f) + (t >= 1 && t <= L ? from_prev : 0.f);
  return d;
}

// Standalone batched V-trace on [B][L] inputs (impala_vtrace).
__global__ __launch_bounds__(256) void vtrace_kernel(const float* __restrict__ v_tm1,
                                                     const float* __restrict__ v_t,
                                                     const float* __restrict__ r_t,
                                                     const float* __restrict__ g_t,
                                                     const float* __restrict__ rho_t, int B,
                                                     int L, int S, float lam, float crho,
                                                     float cpg, float* __restrict__ adv,
                                                     float* __restrict__ err,
                                                     float* __restrict__ q) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int traj = gw * (64 / S) + lane / S;
  const int t = lane % S;
  const bool in = traj < B && t < L;
  const size_t i = (size_t)traj * L + t;
  const float v = in ? v_tm1[i] : 0.f, vt = in ? v_t[i] : 0.f, r = in ? r_t[i] : 0.f,
              g = in ? g_t[i] : 0.f, rho = in ? rho_t[i] : 0.f;
  const VtLane o = vtrace_lane(v, vt, shift_down1(v), r, g, rho, in ? t : L, L, lam, crho, cpg);
  if (in) {
    err[i] = o.err;
    q[i] = o.q;
    adv[i] = o.adv;
  }
}

// =========================================================================================
// Fused loss head (agents/impala/learning.py:144-170): per (b,t) lane: log-softmax of the
// policy and behaviour logits, log pi(a), rho, entropy, KL; per trajectory: V-trace scan over
// T-1 (the last step is dropped from pg/value, kept for entropy/KL/ratio, learning.py:150-157);
// analytic d loss / d logits and d loss / d value under the V-trace gradient mode vt_mode
// (VT_SG_*, vtrace_grad_lane):
//   loss = -mean_{B,T-1}(log pi(a) adv) + mean_{B,T-1}(err^2) - c_ent * mean_{B,T} H(pi)
//   dlogit_j = c_ent/(BT) pi_j (log pi_j + H)  +  kappa_t (1[j=a] - pi_j),
//   kappa_t = d loss / d log pi(a_t)  (= -[t<T-1] adv/(B(T-1)) with the advantage constant)
// Per-workgroup partial sums of (log pi(a) adv, err^2, H, KL, rho) go to `partials`.
// =========================================================================================
struct LossArgs {
  const float* logits; int lg_ld;
  const float* values; int v_ld;
  const int64_t* act; const float* rew; const float* disc; const float* mu;
  int B, T, A, S, vt_mode;
  float lam, crho, cpg, ent_coef;
  float* partials;  // [gridDim.x][8]
  float* dbg_adv; float* dbg_err; float* dbg_q; float* dbg_rho;
};

template <typename TO>
__global__ __launch_bounds__(256) void loss_head_kernel(const LossArgs a, TO* __restrict__ dl,
                                                        int dl_ld, TO* __restrict__ dv,
                                                        int dv_ld, int zero_to) {
  __shared__ float red[4][5];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int gw = blockIdx.x * 4 + wave;
  const int S = a.S, T = a.T, A = a.A, L = T - 1;
  const int traj = gw * (64 / S) + lane / S;
  const int t = lane % S;
  const bool valid = traj < a.B && t < T;
  const bool inL = valid && t < L;
  const size_t n = (size_t)(valid ? traj : 0) * T + (valid ? t : 0);

  float lg[MAX_A], logp[MAX_A];
  float H = 0.f, kl = 0.f, logpa = 0.f, rho = 0.f, v = 0.f, r = 0.f, g = 0.f;
  int act = 0;
  if (valid) {
    // all loads are issued unconditionally (clamped index) and masked afterwards: a
    // "load or constant" select per element would make the compiler wait on each load
    float m = -INFINITY, mu[MAX_A];
    const float* lrow = a.logits + n * a.lg_ld;
    const float* mrow = a.mu + n * A;
#pragma unroll
    for (int j = 0; j < MAX_A; ++j) {
      const int jj = j < A ? j : A - 1;
      lg[j] = lrow[jj];
      mu[j] = mrow[jj];
    }
    act = (int)a.act[n];
    v = a.values[n * a.v_ld];
    r = a.rew[n];
    g = a.disc[n];
#pragma unroll
    for (int j = 0; j < MAX_A; ++j) {
      if (j >= A) lg[j] = -INFINITY;
      m = fmaxf(m, lg[j]);
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAX_A; ++j) s += j < A ? expf(lg[j] - m) : 0.f;
    const float lse = m + logf(s);
    float mm = -INFINITY;
#pragma unroll
    for (int j = 0; j < MAX_A; ++j) {
      if (j >= A) mu[j] = -INFINITY;
      mm = fmaxf(mm, mu[j]);
    }
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < MAX_A; ++j) sm += j < A ? expf(mu[j] - mm) : 0.f;
    const float lse_mu = mm + logf(sm);
    float logmua = 0.f;
#pragma unroll
    for (int j = 0; j < MAX_A; ++j) {
      if (j < A) {
        logp[j] = lg[j] - lse;
        const float p = expf(logp[j]);
        const float lmu = mu[j] - lse_mu;
        H -= p * logp[j];
        kl += p * (logp[j] - lmu);
        if (j == act) { logpa = logp[j]; logmua = lmu; }
      } else {
        logp[j] = 0.f;
      }
    }
    rho = expf(logpa - logmua);
  }
  // ---- V-trace over the first T-1 steps of each trajectory segment ----
  const int tv = valid ? t : 64;     // lanes of missing trajectories are dead in the scans
  const float v_n = shift_down1(v);  // values[:, 1:]
  const VtLane o = vtrace_lane(v, v_n, v_n, r, g, rho, tv, L, a.lam, a.crho, a.cpg);
  const float err = o.err, qq = o.q, adv = o.adv;
  const float c_pg = 1.f / (float)(a.B * L), c_ent = 1.f / (float)(a.B * T);
  const VtGrad gr = vtrace_grad_lane(o, a.vt_mode, v, v_n, r, g, rho, logpa, tv, L, a.lam,
                                     a.crho, a.cpg, c_pg);

  if (valid) {
    const float ke = a.ent_coef * c_ent, kp = gr.dlogpa;
#pragma unroll
    for (int j = 0; j < MAX_A; ++j) {
      if (j < A) {
        const float p = expf(logp[j]);
        const float d = ke * p * (logp[j] + H) + kp * ((j == act ? 1.f : 0.f) - p);
        dl[n * dl_ld + j] = (TO)d;
      } else if (j < zero_to) {
        dl[n * dl_ld + j] = (TO)0.f;
      }
    }
    dv[n * dv_ld] = (TO)gr.dv;
    if (a.dbg_rho) a.dbg_rho[n] = rho;
    if (inL && a.dbg_adv) {
      const size_t k = (size_t)traj * L + t;
      a.dbg_adv[k] = adv;
      a.dbg_err[k] = err;
      a.dbg_q[k] = qq;
    }
  }
  float s0 = inL ? logpa * adv : 0.f, s1 = inL ? err * err : 0.f;
  float s2 = valid ? H : 0.f, s3 = valid ? kl : 0.f, s4 = valid ? rho : 0.f;
  s0 = wave_sum(s0); s1 = wave_sum(s1); s2 = wave_sum(s2); s3 = wave_sum(s3); s4 = wave_sum(s4);
  if (lane == 0) {
    red[wave][0] = s0; red[wave][1] = s1; red[wave][2] = s2; red[wave][3] = s3; red[wave][4] = s4;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    const int k = threadIdx.x;
    a.partials[blockIdx.x * 8 + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

// metrics[0..5] = loss, entropy, td, pg, kl, ratio from the loss-head partial sums
// Sum the per-workgroup partials [nparts][8] (first K values) across one wavefront: lane l
// sums partials l, l + 64, ... in order, then a fixed butterfly over the lanes -- every lane
// ends with the same totals (a one-thread load-add loop would be one L2 round trip per partial).
template <int K>
DEV void sum_partials(const float* part, int nparts, int lane, float (&s)[K]) {
  for (int p = lane; p < nparts; p += 64) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(part + (size_t)p * 8);
    const f32x4 b = *reinterpret_cast<const f32x4*>(part + (size_t)p * 8 + 4);
#pragma unroll
    for (int k = 0; k < K; ++k) s[k] += k < 4 ? a[k] : b[k - 4];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) s[k] = wave_sum(s[k]);
}

// (called by a whole wavefront; lane 0 writes the metrics)
DEV void finalize_loss_metrics(const float* part, int nparts, int B, int T, float ent_coef,
                               float* metrics, int lane) {
  float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  sum_partials<5>(part, nparts, lane, s);
  if (lane != 0) return;
  const float c_pg = 1.f / (float)(B * (T - 1)), c_ent = 1.f / (float)(B * T);
  const float pg = s[0] * c_pg, td = s[1] * c_pg, ent = s[2] * c_ent;
  metrics[0] = -pg + td - ent_coef * ent;
  metrics[1] = ent;
  metrics[2] = td;
  metrics[3] = pg;
  metrics[4] = s[3] * c_ent;
  metrics[5] = s[4] * c_ent;
  metrics[8] = 0.f;  // (PPO's train/target slot) every slot is written each step
}

__global__ void finalize_loss_kernel(const float* part, int nparts, int B, int T, float ent_coef,
                                     float* metrics) {
  if (threadIdx.x < 64) finalize_loss_metrics(part, nparts, B, T, ent_coef, metrics, (int)threadIdx.x);
}

// =========================================================================================
// PPO clipped surrogate (losses.py:131-155), per transition:
//   ratio r = exp(log pi(a) - log pi_ref(a)),  adv = v_target - v
//   pg_l = max(-adv r, -clamp(r, 1-eps, 1+eps) adv),  loss = mean(pg_l) + 0.5 mean(adv^2)
//                                                           - c_ent mean(H(pi))
// adv is detached in pg_l.  d pg_l / d r = -adv w, w = 1 where the unclipped term is the max,
// clamp'(r) (1 inside [lo, hi], bounds included, else 0) where the clipped term is, and their
// mean on a tie (torch.max splits the gradient evenly between equal inputs).
// =========================================================================================
struct PpoFrame {
  float adv, pgl, dr;  // advantage, surrogate term, d pg_l / d r
};
DEV PpoFrame ppo_frame(float r, float v, float tgt, float lo, float hi) {
  const float adv = tgt - v;
  const float l1 = -adv * r, l2 = -fminf(fmaxf(r, lo), hi) * adv;
  const float inside = (r >= lo && r <= hi) ? 1.f : 0.f;
  const float w = l1 > l2 ? 1.f : (l1 < l2 ? inside : 0.5f * (1.f + inside));
  return PpoFrame{adv, fmaxf(l1, l2), -adv * w};
}

// metrics from PPO partial sums (pg_l, adv^2, H, KL, r, target): slots 0..5 as IMPALA
// (loss, entropy, td, pg, kl, ratio) and slot 8 = train/target; kl is clamp_min(0)'d
DEV void finalize_ppo_metrics(const float* part, int nparts, int N, float ent_coef,
                              float* metrics, int lane) {
  float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  sum_partials<6>(part, nparts, lane, s);
  if (lane != 0) return;
  const float c = 1.f / (float)N;
  const float pg = s[0] * c, td = 0.5f * (s[1] * c), ent = s[2] * c;
  metrics[0] = pg + td - ent_coef * ent;
  metrics[1] = ent;
  metrics[2] = td;
  metrics[3] = pg;
  metrics[4] = fmaxf(s[3] * c, 0.f);
  metrics[5] = s[4] * c;
  metrics[8] = s[5] * c;
}

// Standalone PPO loss head on given outputs, one lane per transition (test / reuse entry).
__global__ __launch_bounds__(256) void ppo_loss_head_kernel(
    const float* __restrict__ logits, const float* __restrict__ values,
    const int64_t* __restrict__ act, const float* __restrict__ tgt,
    const float* __restrict__ mu, int N, int A, float ent_coef, float lo, float hi,
    float* __restrict__ dl, float* __restrict__ dv, float* __restrict__ partials) {
  __shared__ float red[4][6];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 256 + threadIdx.x;
  const bool valid = n0 < N;
  const int n = valid ? n0 : 0;
  float lg[MAX_A], mv[MAX_A], p[MAX_A], logp[MAX_A];
#pragma unroll
  for (int j = 0; j < MAX_A; ++j) {
    const int jj = j < A ? j : A - 1;
    lg[j] = logits[(size_t)n * A + jj];
    mv[j] = mu[(size_t)n * A + jj];
  }
  const int a = (int)act[n];
  const float v = values[n], t = tgt[n];
  float m = -INFINITY, mm = -INFINITY;
#pragma unroll
  for (int j = 0; j < MAX_A; ++j) {
    lg[j] = j < A ? lg[j] : -INFINITY;
    mv[j] = j < A ? mv[j] : -INFINITY;
    m = fmaxf(m, lg[j]);
    mm = fmaxf(mm, mv[j]);
  }
  float s = 0.f, sm = 0.f;
#pragma unroll
  for (int j = 0; j < MAX_A; ++j) {
    p[j] = j < A ? expf(lg[j] - m) : 0.f;
    s += p[j];
    sm += j < A ? expf(mv[j] - mm) : 0.f;
  }
  const float lse = m + logf(s), lse_mu = mm + logf(sm), inv_s = 1.f / s;
  float H = 0.f, kl = 0.f, logpa = 0.f, logmua = 0.f;
#pragma unroll
  for (int j = 0; j < MAX_A; ++j) {
    const bool on = j < A;
    logp[j] = on ? lg[j] - lse : 0.f;
    p[j] *= inv_s;
    const float lmu = on ? mv[j] - lse_mu : 0.f;
    H -= p[j] * logp[j];
    kl += p[j] * (logp[j] - lmu);
    logpa = j == a ? logp[j] : logpa;
    logmua = j == a ? lmu : logmua;
  }
  const float r = expf(logpa - logmua);
  const PpoFrame pf = ppo_frame(r, v, t, lo, hi);
  if (valid) {
    const float c = 1.f / (float)N, ke = ent_coef * c, kr = c * pf.dr * r;
#pragma unroll
    for (int j = 0; j < MAX_A; ++j)
      if (j < A) dl[(size_t)n * A + j] = ke * p[j] * (logp[j] + H) + kr * ((j == a ? 1.f : 0.f) - p[j]);
    dv[n] = -pf.adv * c;
  }
  float q[6] = {valid ? pf.pgl : 0.f, valid ? pf.adv * pf.adv : 0.f, valid ? H : 0.f,
                valid ? kl : 0.f, valid ? r : 0.f, valid ? t : 0.f};
#pragma unroll
  for (int k = 0; k < 6; ++k) q[k] = wave_sum(q[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 6; ++k) red[wave][k] = q[k];
  __syncthreads();
  if (threadIdx.x < 6) {
    const int k = threadIdx.x;
    partials[blockIdx.x * 8 + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

__global__ void finalize_ppo_kernel(const float* part, int nparts, int N, float ent_coef,
                                    float* metrics9) {
  if (threadIdx.x < 64) finalize_ppo_metrics(part, nparts, N, ent_coef, metrics9, (int)threadIdx.x);
}


// LayerNorm backward + conv3 ReLU mask; per-workgroup partials of d gamma, d beta.
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy,
                                                     const T* __restrict__ x,
                                                     const float* __restrict__ stats,
                                                     const float* __restrict__ gam,
                                                     T* __restrict__ dx,
                                                     float* __restrict__ slab, int N, int fpw) {
  __shared__ float red[4][2][FLAT / 4];  // reused in 4 passes of 256 columns
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dg[16], db[16], gm[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    dg[i] = 0.f;
    db[i] = 0.f;
    gm[i] = gam[lane * 16 + i];
  }
  // the next frame's x / dy / stats are loaded while the current one is computed
  const int nb = (blockIdx.x * 4 + wave) * fpw;
  const int nf = max(0, min(fpw, N - nb));
  float xn[16], dn[16], mn = 0.f, rn = 0.f;
  auto fetch = [&](int n) {
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
      load4(x + (size_t)n * FLAT + lane * 16 + i, xn + i);
      load4(dy + (size_t)n * FLAT + lane * 16 + i, dn + i);
    }
    mn = stats[2 * n];
    rn = stats[2 * n + 1];
  };
  if (nf > 0) fetch(nb);
  for (int f = 0; f < nf; ++f) {
    const int n = nb + f;
    float xv[16], d[16], xh[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) { xv[i] = xn[i]; d[i] = dn[i]; }
    const float mean = mn, rstd = rn;
    if (f + 1 < nf) fetch(n + 1);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      xh[i] = (xv[i] - mean) * rstd;
      const float gd = d[i] * gm[i];
      s1 += gd;
      s2 += gd * xh[i];
      dg[i] += d[i] * xh[i];
      db[i] += d[i];
    }
    s1 = wave_sum(s1) * (1.f / FLAT);
    s2 = wave_sum(s2) * (1.f / FLAT);
    float o[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float g = rstd * (d[i] * gm[i] - s1 - xh[i] * s2);
      o[i] = xv[i] > 0.f ? g : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 16; i += 4) store4(dx + (size_t)n * FLAT + lane * 16 + i, o + i);
  }
  // deterministic cross-wave reduction, 256 columns (16 lanes x 16) per pass
  for (int pass = 0; pass < 4; ++pass) {
    if ((lane >> 4) == pass) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        red[wave][0][(lane & 15) * 16 + i] = dg[i];
        red[wave][1][(lane & 15) * 16 + i] = db[i];
      }
    }
    __syncthreads();
    const int c = threadIdx.x;  // 0..255
    const float g = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    const float b = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    slab[(size_t)blockIdx.x * 2 * FLAT + pass * 256 + c] = g;
    slab[(size_t)blockIdx.x * 2 * FLAT + FLAT + pass * 256 + c] = b;
    __syncthreads();
  }
}

// =========================================================================================
// Shadow-weight emission: canonical (state_dict) index -> kernel layouts (see net.h).
// =========================================================================================
struct ShadowPtrs {
  void* base;   // T elements, layout net::shadow()
  float* vecs;  // net::Vecs
  int A;
};

template <typename T>
DEV void write_shadow(const ShadowPtrs& sp, const Canon& cn, const Shadow& sh, size_t i, float p) {
  T* w = reinterpret_cast<T*>(sp.base);
  float* vv = sp.vecs;
  const T pt = (T)p;
  if (i < cn.b1) {
    const int k = (int)i, oc = k / K1, rem = k - oc * K1;
    w[sh.w1 + oc * K1 + c1_kprime(rem >> 6, (rem >> 3) & 7, rem & 7)] = pt;
  } else if (i < cn.w2) {
    vv[Vecs::b1 + (i - cn.b1)] = p;
  } else if (i < cn.b2) {
    const int k = (int)(i - cn.w2), oc = k / K2, rem = k % K2, ci = rem >> 4, kh = (rem >> 2) & 3,
              kw = rem & 3;
    w[sh.w2 + oc * K2 + (kh * 4 + kw) * OC1 + ci] = pt;
    if constexpr (sizeof(T) == 4) w[sh.w2t + ((kh * 4 + kw) * OC1 + ci) * OC2 + oc] = pt;
  } else if (i < cn.w3) {
    vv[Vecs::b2 + (i - cn.b2)] = p;
  } else if (i < cn.b3) {
    const int k = (int)(i - cn.w3), oc = k / K3, rem = k % K3, ci = rem / 9, tap = rem % 9;
    w[sh.w3 + oc * K3 + tap * OC2 + ci] = pt;
    if constexpr (sizeof(T) == 4) w[sh.w3t + (tap * OC2 + ci) * OC3 + oc] = pt;
  } else if (i < cn.lng) {
    vv[Vecs::b3 + (i - cn.b3)] = p;
  } else if (i < cn.lnb) {
    const int j = (int)(i - cn.lng);
    vv[Vecs::lng + (j & 15) * OC3 + (j >> 4)] = p;
  } else if (i < cn.wfc) {
    const int j = (int)(i - cn.lnb);
    vv[Vecs::lnb + (j & 15) * OC3 + (j >> 4)] = p;
  } else if (i < cn.bfc) {
    const int k = (int)(i - cn.wfc), o = k >> 10, j = k & 1023;
    const int jj = (j & 15) * OC3 + (j >> 4);
    w[sh.wfc + (size_t)o * FLAT + jj] = pt;
  } else if (i < cn.wa) {
    vv[Vecs::bfc + (i - cn.bfc)] = p;
  } else if (i < cn.ba) {
    const int k = (int)(i - cn.wa), ar = k >> 8, j = k & 255;
    w[sh.wh + ar * HID + j] = pt;
    w[sh.wht + j * HPAD + ar] = pt;
  } else if (i < cn.wc) {
    vv[Vecs::bh + (i - cn.ba)] = p;
  } else if (i < cn.bc) {
    const int j = (int)(i - cn.wc);
    w[sh.wh + VCOL * HID + j] = pt;
    w[sh.wht + j * HPAD + VCOL] = pt;
  } else {
    vv[Vecs::bh + VCOL] = p;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pack_params_kernel(const float* __restrict__ params,
                                                          ShadowPtrs sp, Canon cn, Shadow sh) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < cn.total) write_shadow<T>(sp, cn, sh, i, params[i]);
}

// =========================================================================================
// Gradient-slab reduction into the canonical (state_dict) gradient buffer.  Work is laid out
// in KERNEL order (slab-contiguous: one float4 per thread, coalesced across the wave, all
// splits summed in a fixed order -> deterministic); the canonical index of each element is
// computed on the write side.  Also: per-block sum of squares (clip norm), loss-metric
// finalisation and the Adam step counter increment (block 0).
// =========================================================================================
enum RedKind { RK_ID = 0, RK_CONV2, RK_CONV3, RK_LN, RK_FC, RK_HEADS_W, RK_HEADS_B, RK_CONV1 };
constexpr int MAX_RED_SEGS = 12;
struct RedSeg {
  const float* slab;  // [S][count]
  int S, count, kind;
  long long canon;    // canonical offset (for RK_LN: lng offset; lnb follows)
  int sg;             // split groups per workgroup (power of two, <= 16)
};
struct RedArgs {
  RedSeg seg[MAX_RED_SEGS];
  int wg_start[MAX_RED_SEGS + 1];  // first workgroup of each segment
  int nseg;
  float* grads;
  Canon cn;
  float* sumsq_part;
  const float* loss_part;
  int n_loss_part, B, T, A;
  int algo;  // IMPALA_ALGO_*: which loss the partial sums belong to
  float ent_coef;
  float* metrics;
  int64_t* step;
  double lr, b1, b2;  // Adam bias corrections for the step this reduction completes
  float* adam_sc;     // [2]: lr / (1 - b1^t), sqrt(1 - b2^t)
};

DEV long long canon_index(const RedArgs& a, const RedSeg& sg, int k) {
  switch (sg.kind) {
    case RK_CONV1: {  // k = oc*192 + k' (s2d order)  ->  oc*192 + ci*64 + kh*8 + kw
      const int oc = k / K1;
      return sg.canon + oc * K1 + c1_canon_k(k - oc * K1);
    }
    case RK_CONV2: {  // k = oc*512 + tap*32 + ci  ->  oc*512 + ci*16 + tap
      const int oc = k >> 9, rem = k & 511, tap = rem >> 5, ci = rem & 31;
      return sg.canon + oc * K2 + ci * 16 + tap;
    }
    case RK_CONV3: {  // k = oc*576 + tap*64 + ci  ->  oc*576 + ci*9 + tap
      const int oc = k / K3, rem = k - oc * K3, tap = rem >> 6, ci = rem & 63;
      return sg.canon + oc * K3 + ci * 9 + tap;
    }
    case RK_LN: {  // k = which*1024 + p*64 + c  ->  lng/lnb + c*16 + p
      const int which = k >> 10, j = k & 1023, p = j >> 6, c = j & 63;
      return sg.canon + which * FLAT + c * 16 + p;
    }
    case RK_FC: {  // k = o*1024 + p*64 + c  ->  o*1024 + c*16 + p
      const int o = k >> 10, j = k & 1023, p = j >> 6, c = j & 63;
      return sg.canon + (long long)o * FLAT + c * 16 + p;
    }
    case RK_HEADS_W: {  // k = row*256 + j; rows 0..A-1 actor, row 15 critic, else padding
      const int row = k >> 8, j = k & 255;
      if (row < a.A) return (long long)a.cn.wa + row * HID + j;
      if (row == VCOL) return (long long)a.cn.wc + j;
      return -1;
    }
    case RK_HEADS_B: {
      if (k < a.A) return (long long)a.cn.ba + k;
      if (k == VCOL) return (long long)a.cn.bc;
      return -1;
    }
    default:
      return sg.canon + k;
  }
}

// Sum of splits grp, grp + SG, ... of one float4 column of a slab, in split order.  The loads
// are unconditional (split index clamped to S - 1) and out-of-range splits are dropped by a
// value select after them (a select, not a multiply by 0: an Inf in the clamped split must not
// become a NaN); a "load or zero" select per element compiles to a branch and a vmcnt(0) wait
// per load.
template <int R>
DEV f32x4 sum_splits(const float* p, int grp, int SG, int S, int count) {
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int q = grp; q < S; q += R * SG) {
    f32x4 v[R];
#pragma unroll
    for (int j = 0; j < R; ++j)
      v[j] = *reinterpret_cast<const f32x4*>(p + (size_t)min(q + j * SG, S - 1) * count);
#pragma unroll
    for (int j = 0; j < R; ++j) acc += q + j * SG < S ? v[j] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  return acc;
}

// torch Adam's step size lr / (1 - b1^t) and sqrt(1 - b2^t) for step t (double, as torch's
// python scalars), rounded to fp32
DEV void adam_scalars(const RedArgs& a, int64_t t, float& step_size, float& bc2s) {
  const double bc1 = 1.0 - pow(a.b1, (double)t), bc2 = 1.0 - pow(a.b2, (double)t);
  step_size = (float)(a.lr / bc1);
  bc2s = (float)sqrt(bc2);
}

// One reduction unit = one workgroup of reduce_grads_kernel (global index `u`), on 256 threads
// (`tid`): reduce_unit_sum gives each thread the sum of its split group, which the caller puts
// in part[tid]; after a barrier reduce_unit_finish combines the SG split groups from LDS --
// threads of split group 0 whose column is in range get the 4 reduced values and their
// canonical indices (-1: padding / out of range) -- and returns the thread's sum of squares.
struct RedUnit {
  int s, SG, cols, col, grp, v4;
  bool in;
};
DEV RedUnit reduce_unit_at(const RedArgs& a, int u, int tid) {
  RedUnit r;
  r.s = 0;
  while (u >= a.wg_start[r.s + 1]) ++r.s;
  const RedSeg& sg = a.seg[r.s];
  r.SG = sg.sg;
  r.cols = 256 / r.SG;
  r.col = tid % r.cols;
  r.grp = tid / r.cols;
  r.v4 = (u - a.wg_start[r.s]) * r.cols + r.col;  // float4 index in the segment
  r.in = r.v4 * 4 < sg.count;
  return r;
}
DEV f32x4 reduce_unit_sum(const RedArgs& a, const RedUnit& r) {
  const RedSeg& sg = a.seg[r.s];
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  if (r.in) {
    // R split loads in flight per round, R = 8 or 16 by the splits this thread sums (one
    // round for every segment at the default split-group rule)
    const float* p = sg.slab + (size_t)r.v4 * 4;
    acc = (sg.S + r.SG - 1) / r.SG <= 8 ? sum_splits<8>(p, r.grp, r.SG, sg.S, sg.count)
                                        : sum_splits<16>(p, r.grp, r.SG, sg.S, sg.count);
  }
  return acc;
}
DEV float reduce_unit_finish(const RedArgs& a, const RedUnit& r, const f32x4* part, f32x4& acc,
                             long long (&ci)[4]) {
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) ci[i] = -1;
  if (r.grp == 0 && r.in) {
    for (int g2 = 1; g2 < r.SG; ++g2) acc += part[g2 * r.cols + r.col];
    const int k = r.v4 * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ci[i] = canon_index(a, a.seg[r.s], k + i);
      if (ci[i] >= 0) sq += acc[i] * acc[i];
    }
  }
  return sq;
}
DEV float reduce_unit(const RedArgs& a, int wg, f32x4* part, f32x4& acc, long long (&ci)[4]) {
  const RedUnit r = reduce_unit_at(a, wg, (int)threadIdx.x);
  acc = reduce_unit_sum(a, r);
  part[threadIdx.x] = acc;
  __syncthreads();
  return reduce_unit_finish(a, r, part, acc, ci);
}

// Reduction units run by extra blocks of another launch (one unit per 256-thread quarter of a
// 256*Q-thread block; u < 0: the quarter has none but still takes part in the barriers).  Same
// arithmetic and sum-of-squares slot (the unit's global index) as reduce_grads_kernel.
template <int Q>
DEV void reduce_units_quarters(const RedArgs& a, int u, f32x4* part_all, float* red_all) {
  const int q = (int)threadIdx.x >> 8, tid = (int)threadIdx.x & 255;
  f32x4* part = part_all + q * 256;
  float* red = red_all + q * 4;
  RedUnit r{};
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  if (u >= 0) {
    r = reduce_unit_at(a, u, tid);
    acc = reduce_unit_sum(a, r);
  }
  part[tid] = acc;
  __syncthreads();
  long long ci[4];
  float sq = 0.f;
  if (u >= 0) {
    sq = reduce_unit_finish(a, r, part, acc, ci);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (ci[i] >= 0) a.grads[ci[i]] = acc[i];
  }
  sq = wave_sum(sq);
  if ((tid & 63) == 0) red[tid >> 6] = sq;
  __syncthreads();
  if (u >= 0 && tid == 0) a.sumsq_part[u] = red[0] + red[1] + red[2] + red[3];
}

// Each segment is processed by workgroups of 256 threads = (256/SG) float4 columns x SG
// split groups; split group g sums splits g, g+SG, ... and the SG partials are combined in
// LDS in a fixed order (deterministic for a given SG).  wg_start[] holds each segment's
// first workgroup.  One launch reduces segments [s_lo, s_hi) (grid = their workgroups), so
// each weight-gradient branch can be reduced as soon as its slab is complete; the workgroup's
// global index (wg_start[s_lo] + blockIdx.x) names its sum-of-squares partial, so the partial
// order -- and the norm -- does not depend on how the segments were grouped into launches.
__global__ __launch_bounds__(256) void reduce_grads_kernel(const RedArgs a, int s_lo, int fin) {
  __shared__ f32x4 part[256];
  __shared__ float red[4];
  const int wg = a.wg_start[s_lo] + (int)blockIdx.x;
  f32x4 acc;
  long long ci[4];
  float sq = reduce_unit(a, wg, part, acc, ci);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (ci[i] >= 0) a.grads[ci[i]] = acc[i];
  sq = wave_sum(sq);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) a.sumsq_part[wg] = red[0] + red[1] + red[2] + red[3];
  if (fin && blockIdx.x == 0 && (threadIdx.x >> 6) == 1) {  // wave 1
    if (a.algo == 1)
      finalize_ppo_metrics(a.loss_part, a.n_loss_part, a.B * a.T, a.ent_coef, a.metrics, threadIdx.x & 63);
    else
      finalize_loss_metrics(a.loss_part, a.n_loss_part, a.B, a.T, a.ent_coef, a.metrics, threadIdx.x & 63);
  }
  if (fin && blockIdx.x == 0 && threadIdx.x == 128) {  // step += 1 and its bias corrections
    const int64_t t = *a.step + 1;
    *a.step = t;
    adam_scalars(a, t, a.adam_sc[0], a.adam_sc[1]);
  }
}

// per-block sum of squares of an (all-reduced) gradient buffer
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, size_t n,
                                                    float* __restrict__ part) {
  __shared__ float red[4];
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    acc += g[i] * g[i];
  const float q = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// =========================================================================================
// clip_grad_norm_(max_norm) + torch.optim.Adam (agents/impala/learning.py:172-176,
// builder.py:43-44), then re-emission of the kernel-layout weights.  Every block re-sums
// the sum-of-squares partials itself (deterministic, no grid barrier).
// =========================================================================================
// impala_set_metrics_host: the word of the 16-float host row the Adam kernel sets last
constexpr int kMetricsHostFlag = 15;
struct AdamArgs {
  float *params, *grads, *m, *v, *metrics;
  float* metrics_host;  // (or null) page-locked host copy of the step's metrics vector
  const float* sumsq_part;
  int n_part;
  const int64_t* step;
  const float* sc;  // [2] step size and sqrt(bias correction 2), written by reduce_grads
  double b1, b2;
  float eps, max_norm, inv_world;
  ShadowPtrs sp;
  Canon cn;
  Shadow sh;
};

// torch.optim.Adam's update of one element (lerp form of exp_avg, sqrt(v) / sqrt(bc2) + eps),
// on the clipped gradient g * gscale; shared by the unfused and the fused update kernels so both
// compile the same arithmetic
DEV void adam_elem(const AdamArgs& a, float gscale, float step_size, float bc2s, float& g,
                   float& m, float& v, float& p) {
  // every multiply and add rounded on its own, as written: no FMA contraction, whose choice
  // depends on the surrounding code and would make the two kernels differ in the last bit
#pragma clang fp contract(off)
  const float w1 = (float)(1.0 - a.b1), b2f = (float)a.b2, w2 = (float)(1.0 - a.b2);
  g = g * gscale;
  m = m + w1 * (g - m);
  v = v * b2f + w2 * g * g;
  const float denom = sqrtf(v) / bc2s + a.eps;
  p = p - step_size * (m / denom);
}

// clip + Adam on 4 consecutive parameters per thread; re-emits the kernel-layout weights.
// Blocks [0, HID) each own one row o of the FC weight (canonical [wfc + o*FLAT, +FLAT): 64% of
// the parameters) and re-emit its kernel-layout row (jj = p*64 + c for canonical j = c*16 + p)
// through LDS as one 16-byte (fp32) / 8-byte (bf16) store per thread: the per-element
// scattered stores of write_shadow cost the step ~3 us (tools/var_specs/adamko.py,
// profiles/r05tail).  Blocks [HID, ..) take the other parameters, one per thread in canonical
// order with the FC rows skipped.
static_assert((OC1 * K1 + OC1 + OC2 * K2 + OC2 + OC3 * K3 + OC3 + 2 * FLAT) % 4 == 0,
              "adam_kernel: the FC weight rows start float4-aligned in the canonical buffer");
template <typename T>
__global__ __launch_bounds__(256) void adam_kernel(const AdamArgs a) {
  __shared__ float red[4];
  __shared__ __attribute__((aligned(16))) T fcrow[FLAT];
  // this thread's 4 parameters, the step scalars and the norm partials are all loaded up
  // front (one memory round trip), then one barrier combines the norm
  const bool fc = blockIdx.x < HID;
  size_t i0;
  if (fc) {
    i0 = a.cn.wfc + (size_t)blockIdx.x * FLAT + threadIdx.x * 4;
  } else {  // one parameter per thread: the scattered shadow stores of write_shadow (two per
            // conv2 / conv3 weight in fp32) spread over 4x the waves (profiles/r05tail)
    const size_t e = (size_t)(blockIdx.x - HID) * 256 + threadIdx.x;
    i0 = e < a.cn.wfc ? e : e + (a.cn.bfc - a.cn.wfc);
  }
  const int n = i0 < a.cn.total ? (fc ? 4 : 1) : 0;
  float g[4], m[4], v[4], p[4];
  if (n == 4) {
    const f32x4 G = *reinterpret_cast<const f32x4*>(a.grads + i0);
    const f32x4 M = *reinterpret_cast<const f32x4*>(a.m + i0);
    const f32x4 Vv = *reinterpret_cast<const f32x4*>(a.v + i0);
    const f32x4 P = *reinterpret_cast<const f32x4*>(a.params + i0);
#pragma unroll
    for (int k = 0; k < 4; ++k) { g[k] = G[k]; m[k] = M[k]; v[k] = Vv[k]; p[k] = P[k]; }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = k < n;
      g[k] = ok ? a.grads[i0 + k] : 0.f; m[k] = ok ? a.m[i0 + k] : 0.f;
      v[k] = ok ? a.v[i0 + k] : 0.f;     p[k] = ok ? a.params[i0 + k] : 0.f;
    }
  }
  const float step_size = a.sc[0], bc2s = a.sc[1];
  const int64_t step = a.step[0];  // for metrics[7] (block 0), loaded with everything else
  float sq = 0.f;  // partials are zero-padded to a multiple of 4 (see impala_create)
  // 4 float4 partial loads in flight per thread (unconditional, clamped; out-of-range ones
  // dropped by a select), same summation order as one at a time
  const int nq = (a.n_part + 3) / 4;
  for (int q0 = threadIdx.x; q0 < nq; q0 += 256 * 4) {
    f32x4 x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = *reinterpret_cast<const f32x4*>(a.sumsq_part + 4 * min(q0 + 256 * j, nq - 1));
#pragma unroll
    for (int j = 0; j < 4; ++j) sq += q0 + 256 * j < nq ? (x[j][0] + x[j][1]) + (x[j][2] + x[j][3]) : 0.f;
  }
  sq = wave_sum(sq);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]) * a.inv_world;
  const float coef = fminf(a.max_norm / (norm + 1e-6f), 1.f);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.metrics[6] = norm;
    a.metrics[7] = (float)step;
  }
  if (a.metrics_host && blockIdx.x == 0 && threadIdx.x == 0) {
    // the whole vector (slots other than 6 and 7 were final when the reduction kernel ended) to
    // host memory with system-scope stores, then a nonzero word at [15] after a system fence:
    // the caller (which zeroed that word before enqueueing the step) may read the vector as soon
    // as it sees the word -- before this kernel's other workgroups have finished -- or after an
    // event recorded behind the step (no device-to-host copy on the stream either way)
    unsigned* out = reinterpret_cast<unsigned*>(a.metrics_host);
    float x[IMPALA_NUM_METRICS];  // every load issued before the first store
#pragma unroll
    for (int i = 0; i < IMPALA_NUM_METRICS; ++i) x[i] = i == 6 ? norm : i == 7 ? (float)step : a.metrics[i];
#pragma unroll
    for (int i = 0; i < IMPALA_NUM_METRICS; ++i)
      __hip_atomic_store(out + i, __float_as_uint(x[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(out + kMetricsHostFlag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (n == 0) return;  // (never an FC block: those are full)
  const float gscale = a.inv_world * coef;
#pragma unroll
  for (int k = 0; k < 4; ++k) adam_elem(a, gscale, step_size, bc2s, g[k], m[k], v[k], p[k]);
  if (n == 4) {
    *reinterpret_cast<f32x4*>(a.grads + i0) = f32x4{g[0], g[1], g[2], g[3]};
    *reinterpret_cast<f32x4*>(a.m + i0) = f32x4{m[0], m[1], m[2], m[3]};
    *reinterpret_cast<f32x4*>(a.v + i0) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(a.params + i0) = f32x4{p[0], p[1], p[2], p[3]};
  } else {
    for (int k = 0; k < n; ++k) {
      a.grads[i0 + k] = g[k]; a.m[i0 + k] = m[k]; a.v[i0 + k] = v[k]; a.params[i0 + k] = p[k];
    }
  }
  if (fc) {
    // canonical j = 4 tid + k = c*16 + q  ->  kernel-layout jj = q*64 + c (write_shadow's RK_FC)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = 4 * (int)threadIdx.x + k;
      fcrow[(j & 15) * OC3 + (j >> 4)] = (T)p[k];
    }
    __syncthreads();
    T* w = reinterpret_cast<T*>(a.sp.base) + a.sh.wfc + (size_t)blockIdx.x * FLAT + 4 * threadIdx.x;
    if constexpr (sizeof(T) == 4)
      *reinterpret_cast<f32x4*>(w) = *reinterpret_cast<const f32x4*>(fcrow + 4 * threadIdx.x);
    else
      *reinterpret_cast<uint2*>(w) = *reinterpret_cast<const uint2*>(fcrow + 4 * threadIdx.x);
  } else {
    for (int k = 0; k < n; ++k) write_shadow<T>(a.sp, a.cn, a.sh, i0 + k, p[k]);
  }
}

// =========================================================================================
// Fused slab reduction + clip + Adam (world_size 1): one launch instead of reduce_grads and
// adam.  The workgroups run the reduction units of reduce_grads_kernel (unit u on workgroup
// u % grid, at most FU_MAX_UNITS each), keep each thread's reduced values and canonical indices in
// registers and issue that element's parameter / moment loads at once.  Each unit's sum of
// squares is published as one 8-byte {epoch, value} granule (an agent-scope relaxed atomic store:
// the data is its own flag, MI355X_MICROARCH.md "R2"); every workgroup then sweeps all granules
// until each carries this launch's epoch, sums them in adam_kernel's order (same norm bits), and
// updates its own elements -- no grid barrier and no other cross-workgroup payload.  Every
// workgroup must be resident at once: the grid is the CU count (one 256-thread workgroup per
// CU), and the sweep is bounded (a timeout sets `fault` and a NaN grad_norm instead of hanging).
// epoch = *epoch_ctr + 1 (never 0), read by every workgroup before it publishes; workgroup 0
// stores it back after its sweep has seen every granule, i.e. after every read.  The Adam step
// counter is handled the same way.  Bitwise equal to reduce_grads + adam (tests).
// =========================================================================================
constexpr int FU_MAX_UNITS = 1;  // units per workgroup (the grid is the unit count)
struct FusedSync {
  unsigned long long* gran;  // [n_units] {epoch << 32 | float bits}
  unsigned* epoch_ctr;
  unsigned* fault;
  int n_units;
  int n_part;          // clip-norm partials: the n_units granules, then part[n_units, n_part)
  const float* part;   // partials written by earlier launches (direct-mode weight gradients)
};

#if IMPALA_AB  // reduce_adam_kernel: measured slower, A/B builds only
template <typename T>
__global__ __launch_bounds__(256) void reduce_adam_kernel(const RedArgs a, const AdamArgs aa,
                                                          const FusedSync fs) {
  __shared__ f32x4 part[256];
  __shared__ float red[4];
  __shared__ unsigned s_epoch;
  __shared__ long long s_step;
  // the epoch counter and the step are read first but only waited for after the reduction
  unsigned e_ld = 0u;
  unsigned long long st_ld = 0ull;
  if (threadIdx.x == 0) {
    e_ld = __hip_atomic_load(fs.epoch_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st_ld = __hip_atomic_load(reinterpret_cast<unsigned long long*>(a.step), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
  }
  float g[FU_MAX_UNITS][4], m[FU_MAX_UNITS][4], v[FU_MAX_UNITS][4], p[FU_MAX_UNITS][4];
  long long ci[FU_MAX_UNITS][4];
  // ---- reduction units; the Adam operands of each element are loaded beside its slabs ----
#pragma unroll
  for (int j = 0; j < FU_MAX_UNITS; ++j) {
    const int u = (int)blockIdx.x + j * (int)gridDim.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) ci[j][i] = -1;
    if (u >= fs.n_units) continue;  // uniform over the workgroup
    {  // this thread's canonical indices (reduce_unit's column mapping) -> p, m, v loads now
      int s = 0;
      while (u >= a.wg_start[s + 1]) ++s;
      const RedSeg& sg = a.seg[s];
      const int cols = 256 / sg.sg, col = threadIdx.x % cols, grp = threadIdx.x / cols;
      const int v4 = (u - a.wg_start[s]) * cols + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long c = grp == 0 && v4 * 4 < sg.count ? canon_index(a, sg, v4 * 4 + i) : -1;
        const long long cc = c >= 0 ? c : 0;  // clamped address, value dropped later
        p[j][i] = aa.params[cc];
        m[j][i] = aa.m[cc];
        v[j][i] = aa.v[cc];
      }
    }
    f32x4 acc;
    float sq = reduce_unit(a, u, part, acc, ci[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) g[j][i] = acc[i];
    if (j == 0 && threadIdx.x == 0) {
      s_epoch = e_ld + 1u == 0u ? 1u : e_ld + 1u;
      s_step = (long long)st_ld;
    }
    sq = wave_sum(sq);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float part_sq = red[0] + red[1] + red[2] + red[3];
      __hip_atomic_store(fs.gran + u,
                         ((unsigned long long)s_epoch << 32) | (unsigned long long)__float_as_uint(part_sq),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();  // part / red are reused by the next unit
  }
  const unsigned epoch = s_epoch;
  const int64_t t = (int64_t)s_step + 1;
  if (blockIdx.x == 0 && (threadIdx.x >> 6) == 1) {  // wave 1
    if (a.algo == 1)
      finalize_ppo_metrics(a.loss_part, a.n_loss_part, a.B * a.T, a.ent_coef, a.metrics, threadIdx.x & 63);
    else
      finalize_loss_metrics(a.loss_part, a.n_loss_part, a.B, a.T, a.ent_coef, a.metrics, threadIdx.x & 63);
  }
  // step size and bias correction (double pow) by one lane, while the others start sweeping
  __shared__ float s_sc[2];
  if (threadIdx.x == 0) adam_scalars(a, t, s_sc[0], s_sc[1]);
  // ---- sweep the granules: thread q holds partials 4q .. 4q+3 (adam_kernel's float4 q) ----
  const int nq = (fs.n_part + 3) / 4;
  float x[4] = {0.f, 0.f, 0.f, 0.f};
  if ((int)threadIdx.x < nq) {  // partials of earlier launches (no wait needed)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = 4 * (int)threadIdx.x + k;
      if (q >= fs.n_units && q < fs.n_part) x[k] = fs.part[q];
    }
  }
  bool timed_out = false;
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
    if ((int)threadIdx.x < nq) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = 4 * (int)threadIdx.x + k;
        if (q < fs.n_units) {
          const unsigned long long w = __hip_atomic_load(fs.gran + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = ok && (unsigned)(w >> 32) == epoch;
          x[k] = __uint_as_float((unsigned)w);
        }
      }
    }
    if (__syncthreads_and(ok)) break;
    if (spins > (1u << 22)) {  // ~0.1 s: a workgroup never ran; give up instead of hanging
      timed_out = true;
      break;
    }
    __builtin_amdgcn_s_sleep(10);
  }
  float sq = 0.f;
  if ((int)threadIdx.x < nq) sq += (x[0] + x[1]) + (x[2] + x[3]);
  sq = wave_sum(sq);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  float norm = sqrtf(red[0] + red[1] + red[2] + red[3]) * aa.inv_world;
  if (timed_out) {
    norm = __builtin_nanf("");
    if (threadIdx.x == 0) __hip_atomic_store(fs.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const float coef = fminf(aa.max_norm / (norm + 1e-6f), 1.f);
  const float step_size = s_sc[0], bc2s = s_sc[1];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    aa.metrics[6] = norm;
    aa.metrics[7] = (float)t;
    *a.step = t;
    a.adam_sc[0] = step_size;
    a.adam_sc[1] = bc2s;
    __hip_atomic_store(fs.epoch_ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const float gscale = aa.inv_world * coef;
#pragma unroll
  for (int j = 0; j < FU_MAX_UNITS; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long c = ci[j][i];
      if (c < 0) continue;
      adam_elem(aa, gscale, step_size, bc2s, g[j][i], m[j][i], v[j][i], p[j][i]);
      aa.grads[c] = g[j][i];
      aa.m[c] = m[j][i];
      aa.v[c] = v[j][i];
      aa.params[c] = p[j][i];
      write_shadow<T>(aa.sp, aa.cn, aa.sh, (size_t)c, p[j][i]);
    }
}
#endif  // IMPALA_AB

// heads output [n][16] -> logits [n][A], values [n]
__global__ void split_heads_kernel(const float* __restrict__ heads, int n, int A,
                                   float* __restrict__ logits, float* __restrict__ values) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n * HEADS) return;
  const int f = i / HEADS, j = i % HEADS;
  if (j < A) logits[(size_t)f * A + j] = heads[i];
  else if (j == VCOL) values[f] = heads[i];
}

// Actor inference head (models/distributed_models.py:21-32 AtariPPOModel.act): one thread per
// frame splits the heads row into logits / value and picks the action -- argmax (first maximal
// index, as torch.argmax) where the frame's deterministic flag is set, else a draw from
// softmax(logits) by inverse CDF on a counter-based uniform (seed, counter, frame), the
// distribution torch's softmax(-1).multinomial(1) samples from.
DEV uint64_t act_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void act_heads_kernel(const float* __restrict__ heads, int n, int A,
                                                        const uint8_t* __restrict__ det, int det_all,
                                                        uint64_t seed, uint64_t counter,
                                                        int64_t* __restrict__ actions,
                                                        float* __restrict__ logits,
                                                        float* __restrict__ values) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= n) return;
  float l[HEADS];
#pragma unroll
  for (int j = 0; j < HEADS; j += 4) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(heads + (size_t)f * HEADS + j);
    l[j] = x[0]; l[j + 1] = x[1]; l[j + 2] = x[2]; l[j + 3] = x[3];
  }
  values[f] = l[VCOL];
  float mx = l[0];
  int am = 0;
  for (int j = 0; j < A; ++j) {
    logits[(size_t)f * A + j] = l[j];
    if (l[j] > mx) { mx = l[j]; am = j; }
  }
  int a = am;
  if (!(det ? det[f] != 0 : det_all != 0)) {
    float sum = 0.f;
    for (int j = 0; j < A; ++j) sum += expf(l[j] - mx);
    const uint64_t r = act_mix64(act_mix64(seed ^ act_mix64(counter)) + (uint64_t)f);
    const float u = (float)(uint32_t)(r >> 40) * (1.f / 16777216.f) * sum;  // [0, sum)
    float c = 0.f;
    a = A - 1;
    for (int j = 0; j < A; ++j) {
      c += expf(l[j] - mx);
      if (u < c) { a = j; break; }
    }
  }
  actions[f] = a;
}

// =========================================================================================
// Replay gather: dst_f[i] = src_f[idx[i]] for up to 8 fields of fixed row size (bytes, multiple
// of 4).  One workgroup per (row, field); 16-byte vector copies for the aligned bulk.
// =========================================================================================
// A row is copied in pieces of GATHER_PIECE bytes, one workgroup per (field, row, piece), so a
// 245 KB obs row is spread over 15 workgroups.  Indices come from device memory (idx) or, for
// up to GATHER_HIDX rows, from the launch's own arguments (hidx: no index upload).
constexpr int GATHER_PIECE = 16384;
constexpr int GATHER_HIDX = 256;
static_assert(GATHER_PIECE % (16 * 256) == 0, "whole 16-byte vectors per thread");
struct GatherArgs {
  const char* src[8];
  char* dst[8];
  long long row_bytes[8];
  int pieces[8];     // pieces per row of each field
  int unit0[9];      // first workgroup of each field: unit0[f] + row * pieces[f] + piece
  int nfields;
  const int64_t* idx;
  int n;
  int hidx[GATHER_HIDX];
};

// Host -> HBM pull copy for the staging ring (impala_stage, IMPALA_H2D_KERNEL=1): a few
// workgroups read page-locked host memory over PCIe with 4 x 16-byte loads in flight per lane
// (PCIe latency x bandwidth needs ~128 KB outstanding), on the copy stream beside the step.
struct PullArgs {
  const char* src[5];
  char* dst[5];
  long long bytes[5];
  int nf;
};
__global__ __launch_bounds__(1024) void h2d_pull_kernel(const PullArgs a) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (int f = 0; f < a.nf; ++f) {
    const long long nv = a.bytes[f] >> 4;
    const f32x4* s = reinterpret_cast<const f32x4*>(a.src[f]);
    f32x4* d = reinterpret_cast<f32x4*>(a.dst[f]);
    long long i = t;
    for (; i + 3 * stride < nv; i += 4 * stride) {
      const f32x4 v0 = __builtin_nontemporal_load(s + i), v1 = __builtin_nontemporal_load(s + i + stride);
      const f32x4 v2 = __builtin_nontemporal_load(s + i + 2 * stride);
      const f32x4 v3 = __builtin_nontemporal_load(s + i + 3 * stride);
      d[i] = v0;
      d[i + stride] = v1;
      d[i + 2 * stride] = v2;
      d[i + 3 * stride] = v3;
    }
    for (; i < nv; i += stride) d[i] = s[i];
    for (long long b = (nv << 4) + t; b < a.bytes[f]; b += stride) a.dst[f][b] = a.src[f][b];
  }
}

// Stands in for a learner step while impala_stage_init primes the copy path: one lane waits
// `ticks` of the 100 MHz real-time counter (bounded: at most 2^20 sleep rounds).
__global__ __launch_bounds__(64) void stage_prime_spin_kernel(long long ticks) {
  if (threadIdx.x != 0) return;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < (1 << 20); ++i) {
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(8);
  }
}

// the device step clock's closing stamp (impala_step_clock_end): one thread, one vector store
__global__ __launch_bounds__(64) void clock_stamp_kernel(unsigned long long* __restrict__ out) {
  if (threadIdx.x == 0) *out = __builtin_amdgcn_s_memrealtime();
}

__global__ __launch_bounds__(256) void gather_rows_kernel(const GatherArgs a) {
  const int u = blockIdx.x;
  int f = 0;
  while (f + 1 < a.nfields && u >= a.unit0[f + 1]) ++f;
  const int r = u - a.unit0[f];
  const int i = r / a.pieces[f], piece = r - i * a.pieces[f];
  if (f >= a.nfields || i >= a.n) return;
  const long long rb = a.row_bytes[f];
  const long long o0 = (long long)piece * GATHER_PIECE;
  const long long len = min((long long)GATHER_PIECE, rb - o0);
  const long long row = a.idx ? a.idx[i] : a.hidx[i];
  const char* s = a.src[f] + (size_t)row * rb + o0;
  char* d = a.dst[f] + (size_t)i * rb + o0;
  const bool al16 = ((((uintptr_t)s) | ((uintptr_t)d) | (uintptr_t)len) & 15) == 0;
  if (al16) {
    // every load of the piece issued before any store (a load-store pair per iteration waited
    // out one memory round trip each: source and destination may alias as far as the compiler
    // knows); the replay rows are read once (nontemporal)
    constexpr int NVT = GATHER_PIECE / 16 / 256;
    const int nv = (int)(len >> 4);
    const f32x4* s4 = reinterpret_cast<const f32x4*>(s);
    f32x4* d4 = reinterpret_cast<f32x4*>(d);
    f32x4 v[NVT];
#pragma unroll
    for (int k = 0; k < NVT; ++k) {
      const int e = (int)threadIdx.x + k * 256;
      if (e < nv) v[k] = __builtin_nontemporal_load(s4 + e);
    }
#pragma unroll
    for (int k = 0; k < NVT; ++k) {
      const int e = (int)threadIdx.x + k * 256;
      if (e < nv) d4[e] = v[k];
    }
  } else {
    const long long nw = len >> 2;
    for (long long v = threadIdx.x; v < nw; v += 256)
      reinterpret_cast<float*>(d)[v] = reinterpret_cast<const float*>(s)[v];
  }
}

#if IMPALA_AB  // wgrad23r_kernel: measured slower, A/B builds only
// conv3 + conv2 weight gradients (wgrad23_kernel's blocks) plus the reduction units of the
// slabs that are already final when they start -- conv1 / LayerNorm (the per-frame backward)
// and FC / heads -- as extra blocks, one unit per 256-thread quarter: the conv weight
// gradients' second round of blocks leaves CUs free, and the final reduce_grads launch keeps
// only the conv2 / conv3 units.  Units are the global indices [u0, u0 + n0) then [u1, u1 + n1).
template <typename T, int G>
__global__ __launch_bounds__(256 * G) void wgrad23r_kernel(
    const Conv3Wgrad<T> o3, float* __restrict__ s_w3, float* __restrict__ s_b3, int mps3, int g3x,
    int g3z, const Conv2Wgrad<T> o2, float* __restrict__ s_w2, float* __restrict__ s_b2, int mps2,
    int g2x, int g2z, const RedArgs ra, int u0, int n0, int u1, int n1) {
  constexpr int SM = Wg23Cfg<T, G>::SMEM * (int)sizeof(T);
  constexpr int SR = G * 256 * 16 + G * 4 * 4;
  __shared__ __attribute__((aligned(16))) char lds[SM > SR ? SM : SR];
  // the reduction blocks first: they are short, and the weight-gradient blocks fill the CUs
  // they free
  const int nr = (n0 + n1 + G - 1) / G;
  const int n3 = g3x * g3z, n2 = g2x * g2z, b = (int)blockIdx.x - nr;
  if (b < 0) {
    const int i = (int)blockIdx.x * G + ((int)threadIdx.x >> 8);
    const int u = i < n0 ? u0 + i : (i - n0 < n1 ? u1 + i - n0 : -1);
    reduce_units_quarters<G>(ra, u, reinterpret_cast<f32x4*>(lds),
                             reinterpret_cast<float*>(lds + G * 256 * 16));
  } else if (b < n3) {
    gemm_wg_body<T, 64, 64, 2, 2, 32, G, Conv3Wgrad<T>>(o3, s_w3, s_b3, mps3, b, g3x, 1, g3z,
                                                        reinterpret_cast<T*>(lds));
  } else if (b < n3 + n2) {
    gemm_wg_body<T, 64, Wg2Tile<T>::BC, Wg2Tile<T>::WR, Wg2Tile<T>::WC, 32, G, Conv2Wgrad<T>>(o2, s_w2, s_b2, mps2, b - n3, g2x, 1, g2z,
                                                         reinterpret_cast<T*>(lds));
  }
}
#endif  // IMPALA_AB
