// Device kernels of the SAC learner step (BASELINE config 5).
//
// Reference: agents/sac/learning.py:146-265 (SACLearner.train_step, critic_loss, actor_loss,
// alpha_loss), models/sac_model.py:19-203 (to_action, SoftQNetwork, ActorBody, ContionusHead,
// SoftCritic, SoftActor).  Every network is a 256-wide MLP and every batch is a few hundred
// transitions, so the step is a chain of small dependent contractions: it is latency-bound,
// and the kernels are shaped for the shortest dependency chain, not for MFMA throughput:
//
//  gemm_jobs   one launch = up to 8 independent GEMMs ("jobs"); one wave per 16x16 output
//              tile with the whole K range of both operands loaded into registers before the
//              first MFMA (one memory round trip per chunk of 8 k-steps).  Three epilogues:
//                E_FWD   D[o][n] = W[o]·X[n] + b[o] (+ReLU): Linear forward, stored row-major
//                        Y[n][o] (4 consecutive features per lane -> one vector store) and/or
//                        transposed Yt[o][n] for a later weight gradient;
//                E_DGRAD D[i][n] = Wt[i]·dY[n], masked by the forward ReLU output: the input
//                        gradient of Linear+ReLU;
//                E_WGRAD D[o][k] = sum_n dYt[o][n] · Xt[k][n]: weight gradient written straight
//                        into the canonical fp32 grad buffer; Xt carries a row of ones after its
//                        last feature, so the bias gradient is the last output column.  Each
//                        tile writes its sum of squares to a fixed slot (clip norm).
//  heads_kernel / critic_loss_kernel / actor_loss_kernel / actor_head_bwd_kernel
//              one wave per transition for everything that needs a whole 256-wide row: the
//              policy head + tanh-Normal sample and log-prob (to_action), Q = Linear(256,1),
//              the TD target and critic loss, the actor loss, and the closed-form backward of
//              the policy head.  Row reductions are DPP/permlane wave sums (fixed order).
//  adam_net_kernel   clip_grad_norm_ + torch Adam over one flat parameter buffer, Polyak
//              update of its target copy, re-emission of the kernel-layout (padded, T, and
//              transposed) weights of both.
//  finalize_kernel   one workgroup: fixed-order metric means, alpha loss + its Adam step,
//              step counters.
//
// Precision: operands in T (fp32 parity mode / bf16 perf mode), MFMA accumulates in fp32;
// heads, losses, gradients, master weights and Adam state are fp32.
#pragma once
#include "common.h"

namespace sac {

constexpr int H = 256;   // hidden width (models/sac_model.py)
constexpr int HT = 272;  // rows of a transposed hidden activation: 256 + ones row + padding
constexpr int MAXJ = 8;
constexpr int MAXK = 16;
constexpr float LOG_SQRT_2PI = 0.91893853320467274178f;  // math.log(math.sqrt(2 * math.pi))

enum Epi : int { E_FWD = 0, E_DGRAD = 1, E_WGRAD = 2 };

struct GJob {
  const void* A;  // [R][lda] (T), k-contiguous
  const void* B;  // [C][ldb] (T), k-contiguous
  int lda, ldb, R, C, K, epi;
  const float* bias;  // E_FWD: [R]
  void* Y;            // row-major [C][ldy] (T), nullable
  int ldy;
  void* Yt;  // transposed [R][ldyt] (T), nullable
  int ldyt;
  const void* M;  // E_DGRAD: forward ReLU output, row-major [C][ldm] (T)
  int ldm;
  float* gW;  // E_WGRAD: col c < kin -> gW[r * kin + c]; c == kin -> gB[r]
  float* gB;
  int kin;
  float* sq;  // E_WGRAD: sum-of-squares slot per tile
  int relu, tile0;
};
struct GArgs {
  GJob j[MAXJ];
  int nj, ntiles;
};

template <typename T>
__global__ __launch_bounds__(256) void gemm_jobs(const GArgs g) {
  using F = Frag<T>;
  typedef typename F::vec V;
  const int lane = threadIdx.x & 63;
  const int t = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
  if (t >= g.ntiles) return;
  int j = 0;
#pragma unroll 1
  while (j + 1 < g.nj && t >= g.j[j + 1].tile0) ++j;
  const GJob& J = g.j[j];
  const int ctn = (J.C + 15) >> 4;
  const int lt = t - J.tile0, rt = lt / ctn, ct = lt - rt * ctn;
  const int r0 = rt * 16, c0 = ct * 16;
  const int kl = F::KPL * (lane >> 4);
  const T* ap = (const T*)J.A + (size_t)min(r0 + (lane & 15), J.R - 1) * J.lda + kl;
  const T* bp = (const T*)J.B + (size_t)min(c0 + (lane & 15), J.C - 1) * J.ldb + kl;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int CH = 8;  // k-steps whose operands are in flight together
#pragma unroll 1
  for (int k0 = 0; k0 < J.K; k0 += CH * F::KSTEP) {
    V a[CH], b[CH];
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const int k = k0 + s * F::KSTEP;
      if (k < J.K) {
        a[s] = F::load(ap + k);
        b[s] = F::load(bp + k);
      } else {
        a[s] = F::zero();
        b[s] = F::zero();
      }
    }
#pragma unroll
    for (int s = 0; s < CH; ++s) acc = F::mma(a[s], b[s], acc);
  }
  const int c = c0 + (lane & 15);
  const int rb = r0 + 4 * (lane >> 4);
  float v[4] = {acc[0], acc[1], acc[2], acc[3]};
  if (J.epi == E_WGRAD) {
    float sq = 0.f;
    if (c <= J.kin) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rb + i;
        if (r < J.R) {
          if (c < J.kin) J.gW[(size_t)r * J.kin + c] = v[i];
          else J.gB[r] = v[i];
          sq += v[i] * v[i];
        }
      }
    }
    sq = wave_sum(sq);
    if (lane == 0) J.sq[lt] = sq;
    return;
  }
  if (c >= J.C) return;  // FWD / DGRAD jobs have R % 16 == 0 (checked by the host)
  if (J.epi == E_FWD) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] += J.bias[rb + i];
      if (J.relu) v[i] = fmaxf(v[i], 0.f);
    }
  } else {
    float m[4];
    load4((const T*)J.M + (size_t)c * J.ldm + rb, m);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = m[i] > 0.f ? v[i] : 0.f;
  }
  if (J.Y) store4((T*)J.Y + (size_t)c * J.ldy + rb, v);
  if (J.Yt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) ((T*)J.Yt)[(size_t)(rb + i) * J.ldyt + c] = to_t<T>(v[i]);
  }
}

// ---- row helpers: a 256-wide row, 4 features per lane (lane l owns 4l .. 4l+3) ----
template <typename T>
DEV void load_row(const void* base, int ld, int n, int lane, float h[4]) {
  load4((const T*)base + (size_t)n * ld + 4 * lane, h);
}
// canonical weight rows start at any float offset (e.g. q2 follows q1's odd-sized b3), so
// they are read with 4-byte loads
DEV f32x4 load4f(const float* w) { return f32x4{w[0], w[1], w[2], w[3]}; }
DEV float dot_row(const float* w, int lane, const float h[4]) {
  const f32x4 x = load4f(w + 4 * lane);
  return wave_sum(x[0] * h[0] + x[1] * h[1] + x[2] * h[2] + x[3] * h[3]);
}
// torch's rounding order, never contracted into fma
DEV float mul(float a, float b) { return __fmul_rn(a, b); }
DEV float add(float a, float b) { return __fadd_rn(a, b); }
DEV float sub(float a, float b) { return __fsub_rn(a, b); }

// ---- counter-based standard normal (device rsample noise) ----
DEV uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
DEV float normal_draw(uint64_t seed, uint64_t ctr, uint64_t i) {
  const uint64_t r = mix64(mix64(seed ^ mix64(ctr)) + i);
  const float u1 = ((float)(uint32_t)(r >> 40) + 1.f) * (1.f / 16777216.f);  // (0, 1]
  const float u2 = (float)(uint32_t)(r & 0xFFFFFFu) * (1.f / 16777216.f);
  return sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
}

// =========================================================================================
// Input packing: the sampled transitions (fp32, caller layout) into zero-padded operand rows
// (T) for the first layers and the transposed copies the first-layer weight gradients read.
// Also draws the three rsample noise blocks when the batch brings none.
// =========================================================================================
struct PackArgs {
  const float *s, *a, *s1;
  int N, D, K, ldd, ldc, ldt;
  void *xs, *xs1, *xc, *xt, *xp;  // [N][ldd] / [N][ldc]
  void *xst, *xct;                // [.][ldt]
  float* eps;                     // [3][N][K] when generated
  uint64_t seed;
  const int64_t* counter;
  const float* probs;  // sampler probabilities (nullable) -> *wmax = max probs^prio_exp (1 if none)
  float prio_exp;
  float* wmax;         // nullable
};

DEV float probs_pow_max(const float* probs, int N, float e, int lane);

template <typename T>
__global__ __launch_bounds__(256) void pack_kernel(const PackArgs p) {
  if (p.wmax && blockIdx.x == 0 && threadIdx.x < 64) {  // the IS-weight normaliser, once per step
    const float m = p.probs ? probs_pow_max(p.probs, p.N, p.prio_exp, threadIdx.x) : 1.f;
    if (threadIdx.x == 0) *p.wmax = m;
  }
  const int DK = p.D + p.K;
  const long long tot = (long long)p.N * DK;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < tot; i += (long long)gridDim.x * 256) {
    const int n = (int)(i / DK), k = (int)(i - (long long)n * DK);
    if (k < p.D) {
      const T s = to_t<T>(p.s[(size_t)n * p.D + k]), s1 = to_t<T>(p.s1[(size_t)n * p.D + k]);
      ((T*)p.xs)[(size_t)n * p.ldd + k] = s;
      ((T*)p.xs1)[(size_t)n * p.ldd + k] = s1;
      ((T*)p.xc)[(size_t)n * p.ldc + k] = s;
      ((T*)p.xt)[(size_t)n * p.ldc + k] = s1;
      ((T*)p.xp)[(size_t)n * p.ldc + k] = s;
      ((T*)p.xst)[(size_t)k * p.ldt + n] = s;
      ((T*)p.xct)[(size_t)k * p.ldt + n] = s;
    } else {
      const T a = to_t<T>(p.a[(size_t)n * p.K + (k - p.D)]);
      ((T*)p.xc)[(size_t)n * p.ldc + k] = a;
      ((T*)p.xct)[(size_t)k * p.ldt + n] = a;
    }
  }
  if (p.eps) {
    const uint64_t ctr = (uint64_t)*p.counter;
    const long long ne = 3LL * p.N * p.K;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < ne; i += (long long)gridDim.x * 256)
      p.eps[i] = normal_draw(p.seed, ctr, (uint64_t)i);
  }
}

// [obs | act] rows for a critic forward (sac_q_forward)
template <typename T>
__global__ __launch_bounds__(256) void pack_sa_kernel(const float* __restrict__ obs,
                                                      const float* __restrict__ act, int n, int D,
                                                      int K, int ld, T* __restrict__ x) {
  const int DK = D + K;
  const long long tot = (long long)n * DK;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < tot; i += (long long)gridDim.x * 256) {
    const int r = (int)(i / DK), k = (int)(i - (long long)r * DK);
    x[(size_t)r * ld + k] = to_t<T>(k < D ? obs[(size_t)r * D + k] : act[(size_t)r * K + k - D]);
  }
}

// plain row packing of observations for inference (sac_act / sac_policy)
template <typename T>
__global__ __launch_bounds__(256) void pack_obs_kernel(const float* __restrict__ obs, int n, int D,
                                                       int ld, T* __restrict__ x) {
  const long long tot = (long long)n * D;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < tot; i += (long long)gridDim.x * 256) {
    const int r = (int)(i / D), k = (int)(i - (long long)r * D);
    x[(size_t)r * ld + k] = to_t<T>(obs[i]);
  }
}

// =========================================================================================
// Heads: one wave per transition.
//   HK_POLICY  ContionusHead + to_action (sac_model.py:19-29,125-139) with rsample = mean +
//              eps * std: action (into the next layer's operand row and/or fp32), log-prob,
//              and the per-(n,k) values the closed-form backward needs.
//   HK_Q       Q = Linear(256, 1) (sac_model.py:80-88).
//   HK_ACT     SoftActor.act (sac_model.py:190-200): tanh(mu + std * noise * scale) * s + b.
// =========================================================================================
enum HeadKind : int { HK_POLICY = 0, HK_Q = 1, HK_ACT = 2 };
struct HeadJob {
  int kind;
  const void* h;  // row-major hidden [N][ldh] (T)
  int ldh;
  const float *wm, *bm, *wl, *bl;  // policy: fc_mean / fc_logstd [K][256], [K]; Q: W3 [256], b3
  const float* eps;                // [N][K]
  void* xout;                      // action into operand rows: xout[n * ldx + xoff + k] (T)
  int ldx, xoff;
  float* act;     // [N][K] fp32
  float* logp;    // [N]
  float* save;    // [4][N][K]: std, y = tanh(x), x - mean, tanh(u)
  float* stdrow;  // [N]: std.mean(-1)
  float* stdout_; // [N][K]
  float *mean_out, *ls_out;  // [N][K] raw head outputs (SoftActor.forward)
  float* q;       // HK_Q: [N]
  float noise_scale, act_scale, act_bias;
};
struct HeadArgs {
  HeadJob j[4];
  int N, K;
};

// one transition's head from its hidden-2 row (global or LDS), executed by one wave
// (operands wm / bm / wl / bl / eps passed separately so they can live in LDS; eps row `er`
// holds this transition's noise)
template <typename T>
DEV void head_row(const HeadJob& J, const float* wm, const float* bm, const float* wl,
                  const float* bl, const float* eps_, const T* hrow, int n, int N, int K, int lane,
                  int er) {
  float h[4];
  load4(hrow + 4 * lane, h);
  if (J.kind == HK_Q) {
    const float q = dot_row(wm, lane, h) + bm[0];
    if (lane == 0) J.q[n] = q;
    return;
  }
  float logp = 0.f, stdsum = 0.f;
  for (int k = 0; k < K; ++k) {
    const float mean = dot_row(wm + (size_t)k * H, lane, h) + bm[k];
    const float u = dot_row(wl + (size_t)k * H, lane, h) + bl[k];
    const float tu = tanhf(u);
    const float ls = add(-5.f, mul(3.5f, add(tu, 1.f)));  // LOG_STD_MIN + 0.5*(MAX-MIN)*(t+1)
    const float sd = expf(ls);
    const float e = eps_ ? eps_[(size_t)er * K + k] : 0.f;
    if (J.kind == HK_ACT) {
      const float x = add(mean, mul(mul(sd, e), J.noise_scale));
      const float y = add(mul(tanhf(x), J.act_scale), J.act_bias);
      if (lane == k) J.act[(size_t)n * K + k] = y;
      continue;
    }
    const float x = add(mean, mul(e, sd));
    const float y = tanhf(x);
    const float var = mul(sd, sd);
    const float xm = sub(x, mean);
    float lp = sub(sub(-__fdiv_rn(mul(xm, xm), mul(2.f, var)), logf(sd)), LOG_SQRT_2PI);
    lp = sub(lp, logf(add(sub(1.f, mul(y, y)), 1e-6f)));
    logp = add(logp, lp);
    stdsum = add(stdsum, sd);
    if (lane == k) {
      const size_t o = (size_t)n * K + k;
      if (J.xout) ((T*)J.xout)[(size_t)n * J.ldx + J.xoff + k] = to_t<T>(y);
      if (J.act) J.act[o] = y;
      if (J.stdout_) J.stdout_[o] = sd;
      if (J.mean_out) J.mean_out[o] = mean;
      if (J.ls_out) J.ls_out[o] = ls;
      if (J.save) {
        const size_t NK = (size_t)N * K;
        J.save[o] = sd;
        J.save[NK + o] = y;
        J.save[2 * NK + o] = xm;
        J.save[3 * NK + o] = tu;
      }
    }
  }
  if (lane == 0 && J.kind == HK_POLICY) {
    if (J.logp) J.logp[n] = logp;
    if (J.stdrow) J.stdrow[n] = __fdiv_rn(stdsum, (float)K);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void heads_kernel(const HeadArgs g) {
  const int lane = threadIdx.x & 63;
  const int n = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
  if (n >= g.N) return;
  const HeadJob& J = g.j[blockIdx.y];
  head_row<T>(J, J.wm, J.bm, J.wl, J.bl, J.eps, (const T*)J.h + (size_t)n * J.ldh, n, g.N, g.K, lane, n);
}

// =========================================================================================
// critic_loss (learning.py:233-248) per transition, and the start of its backward:
//   y = r + !done * gamma * (min(t1, t2) - alpha * logp1)          (no grad)
//   qfi_loss terms w * (y - qi)^2,  dqi = -(2 (y - qi)) * (w / N),  prio = |y - min(q1, q2)|
//   dh2_i = dqi * W3_i (.) [h2_i > 0]   (row-major + transposed), dqi into row 0 of dq_t.
// =========================================================================================
struct CLossArgs {
  const void *ht1, *ht2;  // target critic hidden-2 rows (T)
  const float *w3t1, *b3t1, *w3t2, *b3t2;
  const void *hc1, *hc2;  // critic hidden-2 rows (T)
  const float *w3c1, *w3c2;
  const float *q1, *q2, *logp1;
  const float* r;
  const uint8_t* done;
  const float* probs;
  const float* log_alpha;
  float gamma, prio_exp;
  int N, ldh, ldt;
  float* prio;
  void *dh1, *dh2;    // [N][256] (T)
  void *dh1t, *dh2t;  // [256][ldt] (T)
  void *dq1t, *dq2t;  // [16][ldt] (T), row 0
  float* rowm;        // [8][ldt]
  const float* wmax;  // fused path: the normaliser, computed by pack_kernel
};

// one transition's inputs to critic_loss (loaded together: one memory round trip)
struct CRow {
  float p, lp1, r, q1, q2;
  int done;
};
DEV CRow load_crow(const CLossArgs& a, int n) {
  CRow c;
  // pointer select, not value select (closs_row ignores p without probabilities): a "load or
  // constant" select becomes a branch with a full vmcnt wait
  c.p = (a.probs ? a.probs : a.r)[n];
  c.lp1 = a.logp1[n];
  c.r = a.r[n];
  c.q1 = a.q1[n];
  c.q2 = a.q2[n];
  c.done = a.done[n];
  return c;
}
// importance-weight normaliser max_i probabilities[i]^-0.4 (learning.py:197-199), by one wave
DEV float probs_pow_max(const float* probs, int N, float e, int lane) {
  float mx = 0.f;
  for (int base = 0; base < N; base += 8 * 64) {  // 8 loads in flight per lane per round
    // unconditional loads (indices past N re-read element N - 1), the range test at use
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = probs[min(base + lane + 64 * j, N - 1)];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (base + lane + 64 * j < N) mx = fmaxf(mx, powf(v[j], e));
  }
  return wave_max(mx);
}
DEV float weight_max(const CLossArgs& a, int lane) { return probs_pow_max(a.probs, a.N, a.prio_exp, lane); }
// TD target, weights, losses and dQ of one transition (t1, t2 = target-critic Q values,
// alpha = exp(log_alpha)); lane 0 writes the per-transition metric terms and priority when
// `emit`, and dQ into row 0 of both dq_t operands.
template <typename T>
DEV void closs_row(const CLossArgs& a, const CRow& c, float alpha, float wmax, float t1, float t2,
                   int n, int lane, bool emit, float& dq1, float& dq2) {
  const float w = a.probs ? __fdiv_rn(powf(c.p, a.prio_exp), wmax) : 1.f;
  const float mn = sub(fminf(t1, t2), mul(alpha, c.lp1));
  const float notd = c.done ? 0.f : a.gamma;
  const float y = add(c.r, mul(notd, mn));
  const float d1 = sub(y, c.q1), d2 = sub(y, c.q2);
  const float wn = mul(__fdiv_rn(1.f, (float)a.N), w);
  dq1 = -mul(wn, mul(2.f, d1));
  dq2 = -mul(wn, mul(2.f, d2));
  if (lane == 0) {
    if (emit) {
      if (a.prio) a.prio[n] = fabsf(sub(y, fminf(c.q1, c.q2)));
      a.rowm[0 * a.ldt + n] = mul(mul(d1, d1), w);
      a.rowm[1 * a.ldt + n] = mul(mul(d2, d2), w);
      a.rowm[2 * a.ldt + n] = c.q1;
      a.rowm[3 * a.ldt + n] = c.q2;
    }
    ((T*)a.dq1t)[n] = to_t<T>(dq1);
    ((T*)a.dq2t)[n] = to_t<T>(dq2);
  }
}
// dh2 = dq * W3 (.) [h2 > 0] for the lane's 4 features of one row (h = those h2 values)
DEV void dq_to_dh(float dq, const float* w3, const float h[4], int lane, float d[4]) {
  const f32x4 wv = load4f(w3 + 4 * lane);
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = h[i] > 0.f ? dq * wv[i] : 0.f;
}

template <typename T>
__global__ __launch_bounds__(256) void critic_loss_kernel(const CLossArgs a) {
  const int lane = threadIdx.x & 63;
  const int n = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
  if (n >= a.N) return;
  float h[4];
  load_row<T>(a.ht1, H, n, lane, h);
  const float t1 = dot_row(a.w3t1, lane, h) + a.b3t1[0];
  load_row<T>(a.ht2, H, n, lane, h);
  const float t2 = dot_row(a.w3t2, lane, h) + a.b3t2[0];
  float dq[2];
  const CRow c = load_crow(a, n);
  closs_row<T>(a, c, expf(a.log_alpha[0]), a.probs ? weight_max(a, lane) : 1.f, t1, t2, n, lane,
               true, dq[0], dq[1]);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    float d[4];
    load_row<T>(q ? a.hc2 : a.hc1, H, n, lane, h);
    dq_to_dh(dq[q], q ? a.w3c2 : a.w3c1, h, lane, d);
    store4((T*)(q ? a.dh2 : a.dh1) + (size_t)n * H + 4 * lane, d);
    T* dt = (T*)(q ? a.dh2t : a.dh1t);
#pragma unroll
    for (int i = 0; i < 4; ++i) dt[(size_t)(4 * lane + i) * a.ldt + n] = to_t<T>(d[i]);
  }
}

// =========================================================================================
// actor_loss (learning.py:251-257) per transition: qi on (s, pi) with the updated critic,
// loss term alpha * logp - min(q1, q2); d/dqi = -1/N to the smaller (halved on ties, as the
// torch.min backward); dh2_i row-major.
// =========================================================================================
struct ALossArgs {
  const void *hp1, *hp2;  // hidden-2 rows of the two Q networks on (s, pi) (T)
  const float *w3c1, *b3c1, *w3c2, *b3c2;
  const float* logp;
  const float* log_alpha;
  int N, ldt;
  void *dh1, *dh2;  // [N][256] (T)
  float* rowm;      // row 4: loss term
};

// actor loss term and the dQ of both networks for one transition (q1, q2 on (s, pi))
DEV void aloss_row(const ALossArgs& a, float q1, float q2, float logp, float alpha, int n, int lane,
                   float& dq1, float& dq2) {
  const float g = -__fdiv_rn(1.f, (float)a.N);
  dq1 = q1 < q2 ? g : (q1 == q2 ? 0.5f * g : 0.f);
  dq2 = q2 < q1 ? g : (q1 == q2 ? 0.5f * g : 0.f);
  if (lane == 0) a.rowm[4 * a.ldt + n] = sub(mul(alpha, logp), fminf(q1, q2));
}

template <typename T>
__global__ __launch_bounds__(256) void actor_loss_kernel(const ALossArgs a) {
  const int lane = threadIdx.x & 63;
  const int n = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
  if (n >= a.N) return;
  float h1[4], h2[4];
  load_row<T>(a.hp1, H, n, lane, h1);
  load_row<T>(a.hp2, H, n, lane, h2);
  const float q1 = dot_row(a.w3c1, lane, h1) + a.b3c1[0];
  const float q2 = dot_row(a.w3c2, lane, h2) + a.b3c2[0];
  float dq[2];
  aloss_row(a, q1, q2, a.logp[n], expf(a.log_alpha[0]), n, lane, dq[0], dq[1]);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    float d[4];
    dq_to_dh(dq[q], q ? a.w3c2 : a.w3c1, q ? h2 : h1, lane, d);
    store4((T*)(q ? a.dh2 : a.dh1) + (size_t)n * H + 4 * lane, d);
  }
}

// =========================================================================================
// Backward of the policy head for the actor loss, per transition.  dpi = sum over both Q
// networks of dh1_i · W1_i[:, D + k] (the action columns of the critic's first layer); then
// the closed form of autograd through to_action (x = mean + eps*std, y = tanh x, log-prob of
// Normal(mean, std) at x minus log(1 - y^2 + 1e-6)) and the log-std rescale, with
// c = alpha / N the weight of every log-prob term:
//   g_y    = dpi + c * 2y / (1 - y^2 + 1e-6)
//   g_x    = g_y (1 - y^2) - c (x - mean) / var
//   g_mean = g_x + c (x - mean) / var
//   g_std  = g_x eps + c (x - mean)^2 / std^3 - c / std,   g_u = g_std * std * 3.5 (1 - tanh^2 u)
//   dh2_actor = (g_mean · W_mean + g_u · W_logstd) (.) [h2 > 0]
// =========================================================================================
struct ABwdArgs {
  const void *dhp1, *dhp2;      // critic dh1 rows on (s, pi), [N][256] (T), ReLU-masked
  const float *w1c1, *w1c2;     // critic first layers, canonical [256][D+K]
  const float* save;            // [4][N][K] from heads_kernel
  const float* eps;             // [N][K]
  const float* log_alpha;
  const float *wm, *wl;         // actor fc_mean / fc_logstd weights [K][256]
  const void* ha2;              // actor hidden-2 rows (T)
  int D, K, N, ldt;
  int w1_so, w1_sk, w1_off;     // action column k of w1c at [o * w1_so + k * w1_sk + w1_off]
  void* dha2;                   // [N][256] (T)
  void* dha2t;                  // [256][ldt] (T)
  void *gmt, *gut;              // [16][ldt] (T): g_mean, g_u transposed
};

// one transition: d1/d2 = its ReLU-masked critic dh1 rows on (s, pi), ha2 = its actor hidden-2
// row; writes dha2 (row-major when dha2_row, transposed into a.dha2t) and g_mean / g_u.
// save / eps: row `si` of [4][NKs/K][K] / [.][K] blocks (global, or a row block staged in LDS).
// sg: this wave's 2*MAXK floats of LDS for g_mean / g_u (every lane holds the same values; the
// k loops stay rolled, so register use does not grow with MAXK).
// hv: the lane's 4 actor hidden-2 values of the row (dha2 mask); alpha = exp(log_alpha)
template <typename T>
DEV void ahead_row(const ABwdArgs& a, const T* d1row, const T* d2row, const float hv[4], T* dha2_row,
                   int n, int lane, const float* save, const float* eps, int si, size_t NKs,
                   float* sg, float alpha) {
  const int K = a.K;
  float d1[4], d2[4];
  load4(d1row + 4 * lane, d1);
  load4(d2row + 4 * lane, d2);
  const float c = mul(__fdiv_rn(1.f, (float)a.N), alpha);
#pragma unroll 1
  for (int k = 0; k < K; ++k) {
    float p1 = 0.f, p2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t w = (size_t)(4 * lane + i) * a.w1_so + (size_t)k * a.w1_sk + a.w1_off;
      p1 += d1[i] * a.w1c1[w];
      p2 += d2[i] * a.w1c2[w];
    }
    const float dpi = wave_sum(p1) + wave_sum(p2);
    const size_t o = (size_t)si * K + k;
    const float sd = save[o], y = save[NKs + o], xm = save[2 * NKs + o], tu = save[3 * NKs + o];
    const float e = eps[o];
    const float var = sd * sd, omy = 1.f - y * y;
    const float gy = dpi + c * (2.f * y / (omy + 1e-6f));
    const float gx = gy * omy - c * xm / var;
    const float gs = gx * e + c * (xm * xm) / (var * sd) - c / sd;
    sg[k] = gx + c * xm / var;
    sg[MAXK + k] = gs * sd * (3.5f * (1.f - tu * tu));
  }
  float sacc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int k = 0; k < K; ++k) {
    const float gm = sg[k], gu = sg[MAXK + k];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hcol = 4 * lane + i;
      sacc[i] += gm * a.wm[(size_t)k * H + hcol] + gu * a.wl[(size_t)k * H + hcol];
    }
  }
  float d[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = hv[i] > 0.f ? sacc[i] : 0.f;
  if (dha2_row) store4(dha2_row + 4 * lane, d);
#pragma unroll
  for (int i = 0; i < 4; ++i) ((T*)a.dha2t)[(size_t)(4 * lane + i) * a.ldt + n] = to_t<T>(d[i]);
  if (lane < K) {
    ((T*)a.gmt)[(size_t)lane * a.ldt + n] = to_t<T>(sg[lane]);
    ((T*)a.gut)[(size_t)lane * a.ldt + n] = to_t<T>(sg[MAXK + lane]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void actor_head_bwd_kernel(const ABwdArgs a) {
  __shared__ float sg[4][2 * MAXK];
  const int lane = threadIdx.x & 63;
  const int n = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
  if (n >= a.N) return;
  float hv[4];
  load_row<T>(a.ha2, H, n, lane, hv);
  ahead_row<T>(a, (const T*)a.dhp1 + (size_t)n * H, (const T*)a.dhp2 + (size_t)n * H, hv,
               (T*)a.dha2 + (size_t)n * H, n, lane, a.save, a.eps, n, (size_t)a.N * a.K,
               sg[threadIdx.x >> 6], expf(a.log_alpha[0]));
}

// =========================================================================================
// clip_grad_norm_ + torch.optim.Adam over one flat parameter buffer (learning.py:205-210 /
// :217-222, builder.py:42-47), the Polyak update of its target copy (learning.py:174-180),
// and re-emission of the kernel-layout weights (first layer padded to ld1, second layer and
// its transpose) of both.  update = 0: layouts only (bind / refresh).
// =========================================================================================
struct MlpK {
  void* w1;  // [256][ld1] (T)
  void* w2;  // [256][256] (T)
  void* w2t; // [256][256] (T), nullable
};
struct NetDesc {
  long long base;  // flat offset of the first layer's weight
  int in1, ld1;    // first layer fan-in (D or D+K) and its padded row length
};
struct AdamNetArgs {
  float *p, *g, *m, *v, *tgt;
  long long n;
  const float* sq;
  int nsq, nnet, update, polyak;
  const int64_t* step;
  double lr, b1, b2;
  float eps, max_norm, tau;
  float* norm_out;
  NetDesc net[2];
  MlpK k[2], kt[2];
};

template <typename T>
DEV void emit_layout(const NetDesc& nd, const MlpK& mk, long long i, float val) {
  long long l = i - nd.base;
  const long long n1 = (long long)H * nd.in1;
  if (l < 0) return;
  if (l < n1) {
    const int o = (int)(l / nd.in1), k = (int)(l - (long long)o * nd.in1);
    ((T*)mk.w1)[(size_t)o * nd.ld1 + k] = to_t<T>(val);
    return;
  }
  l -= n1 + H;  // skip b1
  if (l >= 0 && l < (long long)H * H) {
    const int o = (int)(l >> 8), k = (int)(l & 255);
    ((T*)mk.w2)[(size_t)o * H + k] = to_t<T>(val);
    if (mk.w2t) ((T*)mk.w2t)[(size_t)k * H + o] = to_t<T>(val);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void adam_net_kernel(const AdamNetArgs a) {
  __shared__ float red[4];
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  // Every global load is issued first, unconditionally (index clamped, pointer -- not value --
  // selects), so the whole prologue is one memory round trip: the parameter's state, then the
  // norm partials 8 at a time (a "load or 0" select per element would become a branch and a
  // vmcnt(0) wait per load).  Arithmetic and summation order are unchanged.
  const bool in = i < a.n;
  const long long ic = in ? i : a.n - 1;
  float p = a.p[ic];
  const float* gp = a.update ? a.g : a.p;
  const float* mp = a.update ? a.m : a.p;
  const float* vp = a.update ? a.v : a.p;
  float g = gp[ic], m = mp[ic], v = vp[ic];
  float tv = (a.tgt ? a.tgt : a.p)[ic];
  float coef = 1.f;
  if (a.update && a.max_norm > 0.f) {
    float sq = 0.f;
    for (int q0 = threadIdx.x; q0 < a.nsq; q0 += 256 * 8) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = a.sq[min(q0 + 256 * j, a.nsq - 1)];
#pragma unroll
      for (int j = 0; j < 8; ++j) sq += q0 + 256 * j < a.nsq ? x[j] : 0.f;
    }
    sq = wave_sum(sq);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
    __syncthreads();
    const float norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    coef = fminf(__fdiv_rn(a.max_norm, norm + 1e-6f), 1.f);
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.norm_out) *a.norm_out = norm;
  }
  if (!in) return;
  if (a.update) {
    const double t = (double)(*a.step + 1);
    const double bc1 = 1.0 - pow(a.b1, t), bc2 = 1.0 - pow(a.b2, t);
    const float step_size = (float)(a.lr / bc1), bc2s = (float)sqrt(bc2);
    if (a.max_norm > 0.f) g = mul(g, coef);
    const float w1 = (float)(1.0 - a.b1), b2f = (float)a.b2, w2 = (float)(1.0 - a.b2);
    m = add(m, mul(w1, sub(g, m)));
    v = add(mul(v, b2f), mul(mul(w2, g), g));
    const float denom = add(__fdiv_rn(sqrtf(v), bc2s), a.eps);
    p = sub(p, mul(step_size, __fdiv_rn(m, denom)));
    a.g[i] = g;
    a.m[i] = m;
    a.v[i] = v;
    a.p[i] = p;
  }
  const int q = (a.nnet > 1 && i >= a.net[1].base) ? 1 : 0;
  emit_layout<T>(a.net[q], a.k[q], i, p);
  if (a.tgt) {
    if (a.polyak) {
      const float tau = a.tau, omt = (float)(1.0 - (double)a.tau);
      tv = add(mul(tau, p), mul(omt, tv));
      a.tgt[i] = tv;
    }
    emit_layout<T>(a.net[q], a.kt[q], i, tv);
  }
}

// =========================================================================================
// Step finalisation (one workgroup): fixed-order means of the per-transition terms, the
// alpha loss and its Adam step (learning.py:225-230,260-265), the step counters.
// =========================================================================================
struct FinArgs {
  const float* rowm;  // [8][ldt]
  int ldt, N, tune_alpha;
  const float* logp2;  // [N]
  float* la;           // {log_alpha, grad, exp_avg, exp_avg_sq}
  float* metrics;
  int64_t* steps;      // [4]: critic, actor, alpha, learner
  double lr, b1, b2;
  float eps, target_entropy;
};

DEV float block_sum(float v, float* red) {  // 256 threads, fixed order
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void finalize_kernel(const FinArgs a) {
  __shared__ float red[4];
  float s[6];
  const float invN = __fdiv_rn(1.f, (float)a.N);
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    float acc = 0.f;
    for (int n = threadIdx.x; n < a.N; n += 256) acc += a.rowm[r * a.ldt + n];
    s[r] = block_sum(acc, red);
  }
  const float la = a.la[0];
  float sv = 0.f, slv = 0.f;
  if (a.tune_alpha) {
    float acc = 0.f, acc2 = 0.f;
    for (int n = threadIdx.x; n < a.N; n += 256) {
      const float v = add(a.logp2[n], a.target_entropy);
      acc += v;
      acc2 += mul(la, v);
    }
    sv = block_sum(acc, red);
    slv = block_sum(acc2, red);
  }
  if (threadIdx.x != 0) return;
  float* M = a.metrics;
  const float l1 = __fdiv_rn(s[0], (float)a.N), l2 = __fdiv_rn(s[1], (float)a.N);
  M[0] = l1;
  M[1] = l2;
  M[2] = __fdiv_rn(s[2], (float)a.N);
  M[3] = __fdiv_rn(s[3], (float)a.N);
  M[4] = __fdiv_rn(add(l1, l2), 2.f);
  M[6] = __fdiv_rn(s[4], (float)a.N);
  M[7] = __fdiv_rn(s[5], (float)a.N);
  a.steps[0] += 1;
  a.steps[1] += 1;
  if (a.tune_alpha) {
    M[9] = -__fdiv_rn(slv, (float)a.N);
    M[10] = expf(la);
    const float g = mul(-invN, sv);
    const int64_t t = a.steps[2] + 1;
    a.steps[2] = t;
    const double bc1 = 1.0 - pow(a.b1, (double)t), bc2 = 1.0 - pow(a.b2, (double)t);
    const float step_size = (float)(a.lr / bc1), bc2s = (float)sqrt(bc2);
    const float w1 = (float)(1.0 - a.b1), b2f = (float)a.b2, w2 = (float)(1.0 - a.b2);
    float m = a.la[2], v = a.la[3];
    m = add(m, mul(w1, sub(g, m)));
    v = add(mul(v, b2f), mul(mul(w2, g), g));
    const float denom = add(__fdiv_rn(sqrtf(v), bc2s), a.eps);
    a.la[0] = sub(la, mul(step_size, __fdiv_rn(m, denom)));
    a.la[1] = g;
    a.la[2] = m;
    a.la[3] = v;
  }
  a.steps[3] += 1;
  M[11] = (float)a.steps[3];
}

// =========================================================================================
// Uniform replay sampling (one workgroup): idx[i] = hash(seed, counter, i, round) % size,
// redrawn while it collides with an earlier index (without replacement when n <= size).
// =========================================================================================
constexpr int SAMPLE_MAX_UNIQUE = 4096;  // n above this (or size >= 2^31): with replacement
constexpr int SAMPLE_TS = 8192;          // LDS hash table slots (>= 2 n)
DEV int64_t draw_index(uint64_t seed, uint64_t counter, int i, int round, int64_t size) {
  return (int64_t)(mix64(mix64(seed ^ mix64(counter)) + (uint64_t)i + ((uint64_t)round << 40)) %
                   (uint64_t)size);
}
// Every position draws a key; a round inserts all keys into an LDS hash table (linear probing,
// atomicCAS on the key, atomicMin on the owning position), and every position whose key is
// owned by an earlier position redraws.  atomicMin makes the winner order-independent, so the
// result is deterministic; rounds repeat until no position redraws (bounded).
__global__ __launch_bounds__(256) void sample_kernel(uint64_t seed, uint64_t counter, int64_t size,
                                                     int n, int64_t* idx, float* probs) {
  __shared__ uint32_t key[SAMPLE_TS];
  __shared__ int owner[SAMPLE_TS];
  constexpr int PER = SAMPLE_MAX_UNIQUE / 256;
  const bool unique = (int64_t)n <= size && n <= SAMPLE_MAX_UNIQUE && size < (1LL << 31);
  if (probs)
    for (int i = threadIdx.x; i < n; i += 256) probs[i] = __fdiv_rn(1.f, (float)size);
  if (!unique) {
    for (int i = threadIdx.x; i < n; i += 256) idx[i] = draw_index(seed, counter, i, 0, size);
    return;
  }
  uint32_t v[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = threadIdx.x + 256 * q;
    v[q] = i < n ? (uint32_t)draw_index(seed, counter, i, 0, size) : 0u;
  }
  for (int round = 1; round < 64; ++round) {
    for (int t = threadIdx.x; t < SAMPLE_TS; t += 256) {
      key[t] = 0xFFFFFFFFu;
      owner[t] = 0x7FFFFFFF;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + 256 * q;
      if (i >= n) continue;
      uint32_t h = (uint32_t)mix64(v[q]) & (SAMPLE_TS - 1);
      for (int probe = 0; probe < SAMPLE_TS; ++probe) {
        const uint32_t old = atomicCAS(&key[h], 0xFFFFFFFFu, v[q]);
        if (old == 0xFFFFFFFFu || old == v[q]) {
          atomicMin(&owner[h], i);
          break;
        }
        h = (h + 1) & (SAMPLE_TS - 1);
      }
    }
    __syncthreads();
    int redraw = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + 256 * q;
      if (i >= n) continue;
      uint32_t h = (uint32_t)mix64(v[q]) & (SAMPLE_TS - 1);
      for (int probe = 0; probe < SAMPLE_TS && key[h] != v[q]; ++probe) h = (h + 1) & (SAMPLE_TS - 1);
      if (owner[h] != i) {
        v[q] = (uint32_t)draw_index(seed, counter, i, round, size);
        redraw = 1;
      }
    }
    if (!__syncthreads_or(redraw)) break;
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = threadIdx.x + 256 * q;
    if (i < n) idx[i] = (int64_t)v[q];
  }
}

// row gather for sac_sample: dst_f[i] = src_f[idx[i]], any row size (4-byte copies when the
// row size and both addresses allow it, bytes otherwise)
struct SGather {
  const char* src[8];
  char* dst[8];
  long long rb[8];
  int nf, n;
  const int64_t* idx;
};
__global__ __launch_bounds__(64) void sample_gather_kernel(const SGather g) {
  const int i = blockIdx.x, f = blockIdx.y;
  if (i >= g.n || f >= g.nf) return;
  const long long rb = g.rb[f];
  const char* s = g.src[f] + (size_t)g.idx[i] * rb;
  char* d = g.dst[f] + (size_t)i * rb;
  if (((((uintptr_t)s) | ((uintptr_t)d) | (uintptr_t)rb) & 3) == 0) {
    for (long long w = threadIdx.x; w < (rb >> 2); w += 64)
      reinterpret_cast<uint32_t*>(d)[w] = reinterpret_cast<const uint32_t*>(s)[w];
  } else {
    for (long long w = threadIdx.x; w < rb; w += 64) d[w] = s[w];
  }
}

}  // namespace sac
