// SAC learner C-ABI (include/sac_hip.h), linked into libimpala_hip.so beside the IMPALA/PPO
// learner.  SURVEY.md §8(f) row 4 / BASELINE config 5.
//
// One handle = one SAC learner on one device.  The caller owns the canonical parameters,
// gradients, Adam moments, target copies, log_alpha and metrics (sac_bind_state), so the
// Python host exposes them as torch tensors; the handle owns the activation workspaces and
// the kernel-layout weight copies (T, padded, and transposed where a dgrad reads them), which
// the Adam kernels re-emit every step.
//
// One train step is a fixed chain of launches (phase names in kPhase): the critic step
// (learning.py:195-211), the actor step (:213-223), the alpha step (:225-230), Polyak (:174-180)
// folded into the two Adam launches.  Default: 10 launches of per-row-block chain kernels
// (sac_fused.h); SAC_FUSED=0: 22 launches of one kernel per layer (bitwise-equal results).
// The chain is replayed from a hipGraph (SAC_GRAPH=0 disables it): every launch is a few
// microseconds, so host enqueue would otherwise bound the step.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/sac_hip.h"
#include "sac.h"
#include "sac_fused.h"

namespace impala_internal {
int set_error(int code, const std::string& msg);
}

namespace {
using namespace sac;

int fail(int code, const std::string& msg) { return impala_internal::set_error(code, msg); }

#define SCK(x)                                                                         \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return fail((int)e_, std::string(#x) + ": " + hipGetErrorString(e_));           \
  } while (0)

#define SCK_LAUNCH(name)                                                               \
  do {                                                                                 \
    hipError_t e_ = hipGetLastError();                                                 \
    if (e_ != hipSuccess)                                                              \
      return fail((int)e_, std::string("launch ") + (name) + ": " + hipGetErrorString(e_)); \
  } while (0)

inline int rup(int x, int m) { return (x + m - 1) / m * m; }
inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
inline double dec(float x) {  // the decimal constant a float config value was written as
  if (x == 0.f) return 0.0;
  const double e = std::floor(std::log10(std::fabs((double)x)));
  const double s = std::pow(10.0, 7.0 - e);
  return std::round((double)x * s) / s;
}

enum Phase {
  P_PACK = 0, P_FWD1, P_FWD2, P_HEADS, P_TFWD1, P_TFWD2, P_CLOSS, P_CBWD2, P_CBWD1, P_CADAM,
  P_AFWD1, P_AFWD2, P_ALOSS, P_ABWD2, P_AHEAD, P_ABWD1, P_AW1, P_AADAM, P_LFWD1, P_LFWD2,
  P_LHEAD, P_FIN,
  // fused path (sac_fused.h)
  P_CFWD, P_CCHAIN, P_CWGRAD, P_ACHAIN, P_AWGRAD, P_LCHAIN, P_COUNT
};
const char* kPhase[P_COUNT] = {
    "pack", "fwd_l1", "fwd_l2", "heads", "target_critic_l1", "target_critic_l2", "critic_loss",
    "critic_bwd_l2", "critic_wgrad_l1", "critic_adam", "actor_q_l1", "actor_q_l2", "actor_loss",
    "actor_q_dgrad", "actor_head_bwd", "actor_bwd_l2", "actor_wgrad_l1", "actor_adam",
    "alpha_fwd_l1", "alpha_fwd_l2", "alpha_head", "finalize", "critic_fwd_chain",
    "critic_loss_chain", "critic_wgrad", "actor_chain", "actor_wgrad", "alpha_chain"};

inline const char* pname(int ph) { return ph >= 0 && ph < P_COUNT ? kPhase[ph] : "sac_forward"; }

struct Offs {  // canonical flat offsets
  long long a_w1, a_b1, a_w2, a_b2, a_wm, a_bm, a_wl, a_bl, a_total;
  long long q_per, q_w1, q_b1, q_w2, q_b2, q_w3, q_b3, c_total;
};
Offs offsets(int D, int K) {
  Offs o;
  const long long DK = D + K;
  o.a_w1 = 0;
  o.a_b1 = (long long)H * D;
  o.a_w2 = o.a_b1 + H;
  o.a_b2 = o.a_w2 + (long long)H * H;
  o.a_wm = o.a_b2 + H;
  o.a_bm = o.a_wm + (long long)H * K;
  o.a_wl = o.a_bm + K;
  o.a_bl = o.a_wl + (long long)H * K;
  o.a_total = o.a_bl + K;
  o.q_w1 = 0;
  o.q_b1 = (long long)H * DK;
  o.q_w2 = o.q_b1 + H;
  o.q_b2 = o.q_w2 + (long long)H * H;
  o.q_w3 = o.q_b2 + H;
  o.q_b3 = o.q_w3 + H;
  o.q_per = o.q_b3 + 1;
  o.c_total = 2 * o.q_per;
  return o;
}

template <typename T>
__global__ void fill_row_kernel(T* p, int n, float v) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = to_t<T>(v);
}

}  // namespace

struct sac_learner {
  sac_config cfg{};
  int device = 0;
  bool bf16 = false;
  int N = 0, Np = 0, D = 0, K = 0, DK = 0, Dp = 0, Cp = 0, Dt = 0, Ct = 0;
  size_t esz = 4;
  Offs off{};
  sac_state st{};
  bool bound = false;
  void* arena = nullptr;
  size_t arena_used = 0, arena_size = 0;
  // operands (T)
  void *xs = nullptr, *xs1 = nullptr, *xc = nullptr, *xt = nullptr, *xp = nullptr, *xi = nullptr;
  void* xi2 = nullptr;  // [obs | act] rows of sac_q_forward
  void *xst = nullptr, *xct = nullptr;
  void *hta1 = nullptr, *hta2 = nullptr, *ha1 = nullptr, *ha2 = nullptr, *hb1 = nullptr, *hb2 = nullptr;
  void *hc1[2]{}, *hc2[2]{}, *htc1[2]{}, *htc2[2]{}, *hp1[2]{}, *hp2[2]{};
  void *hc1t[2]{}, *hc2t[2]{}, *ha1t = nullptr, *ha2t = nullptr;
  void *dh2[2]{}, *dh2t[2]{}, *dhc1t[2]{}, *dhp2[2]{}, *dhp1[2]{}, *dqt[2]{};
  void *dha2 = nullptr, *dha2t = nullptr, *dha1t = nullptr, *gmt = nullptr, *gut = nullptr;
  // fp32 scratch
  float *q1 = nullptr, *q2 = nullptr, *logp1 = nullptr, *logp = nullptr, *logp2 = nullptr;
  float *save = nullptr, *rowm = nullptr, *eps = nullptr, *sq_c = nullptr, *sq_a = nullptr, *wmax = nullptr;
  int nsq_c = 0, nsq_a = 0;
  int64_t* steps = nullptr;  // critic, actor, alpha, learner
  MlpK ka{}, kta{}, kq[2]{}, ktq[2]{};
  bool fused = true;  // per-row-block chain kernels (SAC_FUSED=0: one launch per layer)
  // graph cache
  bool use_graph = true;
  hipStream_t cap = nullptr;
  struct GraphSlot {
    hipGraphExec_t exec = nullptr;
    sac_batch key{};
    unsigned long long used = 0;
  } graphs[4];
  unsigned long long tick = 0;
  // live launch timer
  int timer_phase = -1, timer_max = 0, timer_n = 0;
  std::vector<hipEvent_t> ev;

  void* take(size_t bytes) {
    const size_t a = (arena_used + 255) & ~(size_t)255;
    arena_used = a + bytes;
    return arena ? (char*)arena + a : nullptr;
  }
};

namespace {

void carve(sac_learner* h) {
  h->arena_used = 0;
  const size_t E = h->esz;
  const int N = h->N, Np = h->Np;
  auto T2 = [&](long long rows, long long cols) { return h->take((size_t)rows * cols * E); };
  auto F = [&](long long n) { return (float*)h->take((size_t)n * 4); };
  h->xs = T2(Np, h->Dp);
  h->xs1 = T2(Np, h->Dp);
  h->xi = T2(Np, h->Dp);
  h->xc = T2(Np, h->Cp);
  h->xt = T2(Np, h->Cp);
  h->xp = T2(Np, h->Cp);
  h->xi2 = T2(Np, h->Cp);
  h->xst = T2(h->Dt, Np);
  h->xct = T2(h->Ct, Np);
  h->hta1 = T2(Np, H);
  h->hta2 = T2(Np, H);
  h->ha1 = T2(Np, H);
  h->ha2 = T2(Np, H);
  h->hb1 = T2(Np, H);
  h->hb2 = T2(Np, H);
  for (int q = 0; q < 2; ++q) {
    h->hc1[q] = T2(Np, H);
    h->hc2[q] = T2(Np, H);
    h->htc1[q] = T2(Np, H);
    h->htc2[q] = T2(Np, H);
    h->hp1[q] = T2(Np, H);
    h->hp2[q] = T2(Np, H);
    h->hc1t[q] = T2(HT, Np);
    h->hc2t[q] = T2(HT, Np);
    h->dh2[q] = T2(Np, H);
    h->dh2t[q] = T2(H, Np);
    h->dhc1t[q] = T2(H, Np);
    h->dhp2[q] = T2(Np, H);
    h->dhp1[q] = T2(Np, H);
    h->dqt[q] = T2(16, Np);
  }
  h->ha1t = T2(HT, Np);
  h->ha2t = T2(HT, Np);
  h->dha2 = T2(Np, H);
  h->dha2t = T2(H, Np);
  h->dha1t = T2(H, Np);
  h->gmt = T2(16, Np);
  h->gut = T2(16, Np);
  const long long NK = (long long)N * h->K;
  h->q1 = F(Np);
  h->q2 = F(Np);
  h->logp1 = F(Np);
  h->logp = F(Np);
  h->logp2 = F(Np);
  h->save = F(4 * NK);
  h->rowm = F(8LL * Np);
  h->eps = F(3 * NK);
  h->wmax = F(4);
  // norm slots: one per weight-gradient tile
  const int t_w2 = 16 * cdiv(H + 1, 16), t_w3 = cdiv(H + 1, 16);
  const int t_w1c = 16 * cdiv(h->DK + 1, 16), t_w1a = 16 * cdiv(h->D + 1, 16);
  const int t_head = cdiv(h->K, 16) * cdiv(H + 1, 16);
  h->nsq_c = 2 * (t_w2 + t_w3 + t_w1c);
  h->nsq_a = t_w2 + 2 * t_head + t_w1a;
  h->sq_c = F(h->nsq_c);
  h->sq_a = F(h->nsq_a);
  h->steps = (int64_t*)h->take(4 * sizeof(int64_t));
  auto mk = [&](int ld1, bool tr) {
    MlpK k;
    k.w1 = T2(H, ld1);
    k.w2 = T2(H, H);
    k.w2t = tr ? T2(H, H) : nullptr;
    return k;
  };
  h->ka = mk(h->Dp, true);
  h->kta = mk(h->Dp, false);
  for (int q = 0; q < 2; ++q) {
    h->kq[q] = mk(h->Cp, true);
    h->ktq[q] = mk(h->Cp, false);
  }
}

template <typename T>
int fill_ones(sac_learner* h, void* base, int row, int ld) {
  fill_row_kernel<T><<<cdiv(h->N, 256), 256>>>((T*)base + (size_t)row * ld, h->N, 1.f);
  SCK_LAUNCH("fill_ones");
  return 0;
}

// ---- launch helpers -------------------------------------------------------------------
void timer_begin(sac_learner* h, int ph, hipStream_t st) {
  if (ph >= 0 && h->timer_phase == ph && h->timer_n < h->timer_max)
    (void)hipEventRecord(h->ev[2 * h->timer_n], st);
}
void timer_end(sac_learner* h, int ph, hipStream_t st) {
  if (ph >= 0 && h->timer_phase == ph && h->timer_n < h->timer_max) {
    (void)hipEventRecord(h->ev[2 * h->timer_n + 1], st);
    ++h->timer_n;
  }
}

GJob fwd_job(const void* W, int ldw, const void* X, int ldx, int K, const float* bias, void* Y,
             void* Yt, int ldt, int N) {
  GJob j{};
  j.A = W; j.lda = ldw; j.B = X; j.ldb = ldx; j.R = H; j.C = N; j.K = K; j.epi = E_FWD;
  j.bias = bias; j.Y = Y; j.ldy = H; j.Yt = Yt; j.ldyt = ldt; j.relu = 1;
  return j;
}
GJob dgrad_job(const void* Wt, const void* dY, const void* Mfwd, void* Y, void* Yt, int ldt, int N) {
  GJob j{};
  j.A = Wt; j.lda = H; j.B = dY; j.ldb = H; j.R = H; j.C = N; j.K = H; j.epi = E_DGRAD;
  j.M = Mfwd; j.ldm = H; j.Y = Y; j.ldy = H; j.Yt = Yt; j.ldyt = ldt;
  return j;
}
GJob wgrad_job(const void* dYt, int R, const void* Xt, int kin, int Np, float* gW, float* gB,
               float* sq) {
  GJob j{};
  j.A = dYt; j.lda = Np; j.B = Xt; j.ldb = Np; j.R = R; j.C = kin + 1; j.K = Np; j.epi = E_WGRAD;
  j.gW = gW; j.gB = gB; j.kin = kin; j.sq = sq;
  return j;
}
inline int job_tiles(const GJob& j) { return cdiv(j.R, 16) * cdiv(j.C, 16); }

template <typename T>
int launch_gemm(sac_learner* h, int ph, std::initializer_list<GJob> jobs, hipStream_t st) {
  GArgs g{};
  int t = 0;
  for (const GJob& j : jobs) {
    if (g.nj >= MAXJ) return fail(IMPALA_E_INVALID, "sac: too many jobs in one launch");
    g.j[g.nj] = j;
    g.j[g.nj].tile0 = t;
    t += job_tiles(j);
    ++g.nj;
  }
  g.ntiles = t;
  timer_begin(h, ph, st);
  gemm_jobs<T><<<cdiv(t, 4), 256, 0, st>>>(g);
  timer_end(h, ph, st);
  SCK_LAUNCH(pname(ph));
  return 0;
}

HeadJob policy_job(const void* hrow, const float* params, const Offs& o, const float* eps) {
  HeadJob j{};
  j.kind = HK_POLICY;
  j.h = hrow; j.ldh = H;
  j.wm = params + o.a_wm; j.bm = params + o.a_bm; j.wl = params + o.a_wl; j.bl = params + o.a_bl;
  j.eps = eps;
  return j;
}
HeadJob q_job(const void* hrow, const float* critic, long long qbase, const Offs& o, float* q) {
  HeadJob j{};
  j.kind = HK_Q;
  j.h = hrow; j.ldh = H;
  j.wm = critic + qbase + o.q_w3; j.bm = critic + qbase + o.q_b3;
  j.q = q;
  return j;
}

template <typename T>
int launch_heads(sac_learner* h, int ph, std::initializer_list<HeadJob> jobs, int n, hipStream_t st) {
  HeadArgs a{};
  int nj = 0;
  for (const HeadJob& j : jobs) a.j[nj++] = j;
  a.N = n;
  a.K = h->K;
  timer_begin(h, ph, st);
  heads_kernel<T><<<dim3(cdiv(n, 4), nj), 256, 0, st>>>(a);
  timer_end(h, ph, st);
  SCK_LAUNCH(pname(ph));
  return 0;
}

AdamNetArgs adam_args(sac_learner* h, bool critic, int update) {
  const sac_state& s = h->st;
  const Offs& o = h->off;
  AdamNetArgs a{};
  a.update = update;
  a.polyak = update;
  a.b1 = dec(h->cfg.adam_beta1);
  a.b2 = dec(h->cfg.adam_beta2);
  a.eps = h->cfg.adam_eps;
  a.max_norm = h->cfg.max_grad_norm;
  a.tau = h->cfg.tau;
  if (critic) {
    a.p = s.critic; a.g = s.critic_grad; a.m = s.critic_m; a.v = s.critic_v; a.tgt = s.target_critic;
    a.n = o.c_total;
    a.sq = h->sq_c; a.nsq = h->nsq_c;
    a.step = h->steps + 0;
    a.lr = dec(h->cfg.critic_lr);
    a.norm_out = s.metrics + SAC_M_CRITIC_GRAD_NORM;
    a.nnet = 2;
    for (int q = 0; q < 2; ++q) {
      a.net[q] = NetDesc{q * o.q_per, h->DK, h->Cp};
      a.k[q] = h->kq[q];
      a.kt[q] = h->ktq[q];
    }
  } else {
    a.p = s.actor; a.g = s.actor_grad; a.m = s.actor_m; a.v = s.actor_v; a.tgt = s.target_actor;
    a.n = o.a_total;
    a.sq = h->sq_a; a.nsq = h->nsq_a;
    a.step = h->steps + 1;
    a.lr = dec(h->cfg.actor_lr);
    a.norm_out = s.metrics + SAC_M_ACTOR_GRAD_NORM;
    a.nnet = 1;
    a.net[0] = NetDesc{0, h->D, h->Dp};
    a.k[0] = h->ka;
    a.kt[0] = h->kta;
  }
  return a;
}

template <typename T>
int launch_adam(sac_learner* h, bool critic, int update, hipStream_t st) {
  const AdamNetArgs a = adam_args(h, critic, update);
  const int ph = critic ? P_CADAM : P_AADAM;
  timer_begin(h, ph, st);
  adam_net_kernel<T><<<cdiv(a.n, 256), 256, 0, st>>>(a);
  timer_end(h, ph, st);
  SCK_LAUNCH(pname(ph));
  return 0;
}

// the whole learner step (learning.py:146-193) on stream `st`
template <typename T>
int enqueue_step(sac_learner* h, const sac_batch* b, hipStream_t st) {
  const sac_state& S = h->st;
  const Offs& o = h->off;
  const int N = h->N, Np = h->Np, D = h->D, K = h->K;
  const long long NK = (long long)N * K;
  const long long qb[2] = {0, o.q_per};
  const float* eps = b->noise ? b->noise : h->eps;
  const float *eps0 = eps, *eps1 = eps + NK, *eps2 = eps + 2 * NK;
  int r;
  {  // 0: operand rows (+ device noise)
    PackArgs p{};
    p.s = b->s; p.a = b->a; p.s1 = b->s1;
    p.N = N; p.D = D; p.K = K; p.ldd = h->Dp; p.ldc = h->Cp; p.ldt = Np;
    p.xs = h->xs; p.xs1 = h->xs1; p.xc = h->xc; p.xt = h->xt; p.xp = h->xp;
    p.xst = h->xst; p.xct = h->xct;
    p.eps = b->noise ? nullptr : h->eps;
    p.seed = h->cfg.seed;
    p.counter = h->steps + 3;
    timer_begin(h, P_PACK, st);
    pack_kernel<T><<<std::max(1, std::min(256, cdiv(std::max((long long)N * h->DK, 3 * NK), 256))), 256, 0, st>>>(p);
    timer_end(h, P_PACK, st);
    SCK_LAUNCH("pack");
  }
  // ---------------- critic step (learning.py:195-211, critic_loss :233-248) ----------------
  if ((r = launch_gemm<T>(h, P_FWD1, {
           fwd_job(h->kta.w1, h->Dp, h->xs1, h->Dp, h->Dp, S.target_actor + o.a_b1, h->hta1, nullptr, Np, N),
           fwd_job(h->kq[0].w1, h->Cp, h->xc, h->Cp, h->Cp, S.critic + qb[0] + o.q_b1, h->hc1[0], h->hc1t[0], Np, N),
           fwd_job(h->kq[1].w1, h->Cp, h->xc, h->Cp, h->Cp, S.critic + qb[1] + o.q_b1, h->hc1[1], h->hc1t[1], Np, N),
           fwd_job(h->ka.w1, h->Dp, h->xs, h->Dp, h->Dp, S.actor + o.a_b1, h->ha1, h->ha1t, Np, N)}, st)))
    return r;
  if ((r = launch_gemm<T>(h, P_FWD2, {
           fwd_job(h->kta.w2, H, h->hta1, H, H, S.target_actor + o.a_b2, h->hta2, nullptr, Np, N),
           fwd_job(h->kq[0].w2, H, h->hc1[0], H, H, S.critic + qb[0] + o.q_b2, h->hc2[0], h->hc2t[0], Np, N),
           fwd_job(h->kq[1].w2, H, h->hc1[1], H, H, S.critic + qb[1] + o.q_b2, h->hc2[1], h->hc2t[1], Np, N),
           fwd_job(h->ka.w2, H, h->ha1, H, H, S.actor + o.a_b2, h->ha2, h->ha2t, Np, N)}, st)))
    return r;
  {
    HeadJob tj = policy_job(h->hta2, S.target_actor, o, eps0);
    tj.xout = h->xt; tj.ldx = h->Cp; tj.xoff = D; tj.logp = h->logp1;
    HeadJob aj = policy_job(h->ha2, S.actor, o, eps1);
    aj.xout = h->xp; aj.ldx = h->Cp; aj.xoff = D; aj.logp = h->logp; aj.save = h->save;
    aj.stdrow = h->rowm + 5 * Np;
    if ((r = launch_heads<T>(h, P_HEADS, {tj, aj, q_job(h->hc2[0], S.critic, qb[0], o, h->q1),
                                          q_job(h->hc2[1], S.critic, qb[1], o, h->q2)}, N, st)))
      return r;
  }
  if ((r = launch_gemm<T>(h, P_TFWD1, {
           fwd_job(h->ktq[0].w1, h->Cp, h->xt, h->Cp, h->Cp, S.target_critic + qb[0] + o.q_b1, h->htc1[0], nullptr, Np, N),
           fwd_job(h->ktq[1].w1, h->Cp, h->xt, h->Cp, h->Cp, S.target_critic + qb[1] + o.q_b1, h->htc1[1], nullptr, Np, N)}, st)))
    return r;
  if ((r = launch_gemm<T>(h, P_TFWD2, {
           fwd_job(h->ktq[0].w2, H, h->htc1[0], H, H, S.target_critic + qb[0] + o.q_b2, h->htc2[0], nullptr, Np, N),
           fwd_job(h->ktq[1].w2, H, h->htc1[1], H, H, S.target_critic + qb[1] + o.q_b2, h->htc2[1], nullptr, Np, N)}, st)))
    return r;
  {
    CLossArgs a{};
    a.ht1 = h->htc2[0]; a.ht2 = h->htc2[1];
    a.w3t1 = S.target_critic + qb[0] + o.q_w3; a.b3t1 = S.target_critic + qb[0] + o.q_b3;
    a.w3t2 = S.target_critic + qb[1] + o.q_w3; a.b3t2 = S.target_critic + qb[1] + o.q_b3;
    a.hc1 = h->hc2[0]; a.hc2 = h->hc2[1];
    a.w3c1 = S.critic + qb[0] + o.q_w3; a.w3c2 = S.critic + qb[1] + o.q_w3;
    a.q1 = h->q1; a.q2 = h->q2; a.logp1 = h->logp1;
    a.r = b->r; a.done = b->done; a.probs = b->probabilities; a.log_alpha = S.log_alpha;
    a.gamma = h->cfg.gamma; a.prio_exp = -h->cfg.prio_exponent;
    a.N = N; a.ldh = H; a.ldt = Np;
    a.prio = b->priorities;
    a.dh1 = h->dh2[0]; a.dh2 = h->dh2[1]; a.dh1t = h->dh2t[0]; a.dh2t = h->dh2t[1];
    a.dq1t = h->dqt[0]; a.dq2t = h->dqt[1];
    a.rowm = h->rowm;
    timer_begin(h, P_CLOSS, st);
    critic_loss_kernel<T><<<cdiv(N, 4), 256, 0, st>>>(a);
    timer_end(h, P_CLOSS, st);
    SCK_LAUNCH("critic_loss");
  }
  float* cg = S.critic_grad;
  if ((r = launch_gemm<T>(h, P_CBWD2, {
           dgrad_job(h->kq[0].w2t, h->dh2[0], h->hc1[0], nullptr, h->dhc1t[0], Np, N),
           dgrad_job(h->kq[1].w2t, h->dh2[1], h->hc1[1], nullptr, h->dhc1t[1], Np, N),
           wgrad_job(h->dh2t[0], H, h->hc1t[0], H, Np, cg + qb[0] + o.q_w2, cg + qb[0] + o.q_b2, h->sq_c),
           wgrad_job(h->dh2t[1], H, h->hc1t[1], H, Np, cg + qb[1] + o.q_w2, cg + qb[1] + o.q_b2,
                     h->sq_c + 16 * cdiv(H + 1, 16)),
           wgrad_job(h->dqt[0], 1, h->hc2t[0], H, Np, cg + qb[0] + o.q_w3, cg + qb[0] + o.q_b3,
                     h->sq_c + 32 * cdiv(H + 1, 16)),
           wgrad_job(h->dqt[1], 1, h->hc2t[1], H, Np, cg + qb[1] + o.q_w3, cg + qb[1] + o.q_b3,
                     h->sq_c + 33 * cdiv(H + 1, 16))}, st)))
    return r;
  {
    float* sq1 = h->sq_c + 34 * cdiv(H + 1, 16);
    const int t1 = 16 * cdiv(h->DK + 1, 16);
    if ((r = launch_gemm<T>(h, P_CBWD1, {
             wgrad_job(h->dhc1t[0], H, h->xct, h->DK, Np, cg + qb[0] + o.q_w1, cg + qb[0] + o.q_b1, sq1),
             wgrad_job(h->dhc1t[1], H, h->xct, h->DK, Np, cg + qb[1] + o.q_w1, cg + qb[1] + o.q_b1, sq1 + t1)}, st)))
      return r;
  }
  if ((r = launch_adam<T>(h, true, 1, st))) return r;
  // ---------------- actor step (learning.py:213-223, actor_loss :251-257) ----------------
  if ((r = launch_gemm<T>(h, P_AFWD1, {
           fwd_job(h->kq[0].w1, h->Cp, h->xp, h->Cp, h->Cp, S.critic + qb[0] + o.q_b1, h->hp1[0], nullptr, Np, N),
           fwd_job(h->kq[1].w1, h->Cp, h->xp, h->Cp, h->Cp, S.critic + qb[1] + o.q_b1, h->hp1[1], nullptr, Np, N)}, st)))
    return r;
  if ((r = launch_gemm<T>(h, P_AFWD2, {
           fwd_job(h->kq[0].w2, H, h->hp1[0], H, H, S.critic + qb[0] + o.q_b2, h->hp2[0], nullptr, Np, N),
           fwd_job(h->kq[1].w2, H, h->hp1[1], H, H, S.critic + qb[1] + o.q_b2, h->hp2[1], nullptr, Np, N)}, st)))
    return r;
  {
    ALossArgs a{};
    a.hp1 = h->hp2[0]; a.hp2 = h->hp2[1];
    a.w3c1 = S.critic + qb[0] + o.q_w3; a.b3c1 = S.critic + qb[0] + o.q_b3;
    a.w3c2 = S.critic + qb[1] + o.q_w3; a.b3c2 = S.critic + qb[1] + o.q_b3;
    a.logp = h->logp; a.log_alpha = S.log_alpha;
    a.N = N; a.ldt = Np;
    a.dh1 = h->dhp2[0]; a.dh2 = h->dhp2[1];
    a.rowm = h->rowm;
    timer_begin(h, P_ALOSS, st);
    actor_loss_kernel<T><<<cdiv(N, 4), 256, 0, st>>>(a);
    timer_end(h, P_ALOSS, st);
    SCK_LAUNCH("actor_loss");
  }
  if ((r = launch_gemm<T>(h, P_ABWD2, {
           dgrad_job(h->kq[0].w2t, h->dhp2[0], h->hp1[0], h->dhp1[0], nullptr, Np, N),
           dgrad_job(h->kq[1].w2t, h->dhp2[1], h->hp1[1], h->dhp1[1], nullptr, Np, N)}, st)))
    return r;
  {
    ABwdArgs a{};
    a.dhp1 = h->dhp1[0]; a.dhp2 = h->dhp1[1];
    a.w1c1 = S.critic + qb[0] + o.q_w1; a.w1c2 = S.critic + qb[1] + o.q_w1;
    a.save = h->save; a.eps = eps1; a.log_alpha = S.log_alpha;
    a.wm = S.actor + o.a_wm; a.wl = S.actor + o.a_wl;
    a.ha2 = h->ha2;
    a.D = D; a.K = K; a.N = N; a.ldt = Np;
    a.w1_so = h->DK; a.w1_sk = 1; a.w1_off = D;
    a.dha2 = h->dha2; a.dha2t = h->dha2t; a.gmt = h->gmt; a.gut = h->gut;
    timer_begin(h, P_AHEAD, st);
    actor_head_bwd_kernel<T><<<cdiv(N, 4), 256, 0, st>>>(a);
    timer_end(h, P_AHEAD, st);
    SCK_LAUNCH("actor_head_bwd");
  }
  float* ag = S.actor_grad;
  {
    const int t_w2 = 16 * cdiv(H + 1, 16), t_head = cdiv(K, 16) * cdiv(H + 1, 16);
    if ((r = launch_gemm<T>(h, P_ABWD1, {
             dgrad_job(h->ka.w2t, h->dha2, h->ha1, nullptr, h->dha1t, Np, N),
             wgrad_job(h->dha2t, H, h->ha1t, H, Np, ag + o.a_w2, ag + o.a_b2, h->sq_a),
             wgrad_job(h->gmt, K, h->ha2t, H, Np, ag + o.a_wm, ag + o.a_bm, h->sq_a + t_w2),
             wgrad_job(h->gut, K, h->ha2t, H, Np, ag + o.a_wl, ag + o.a_bl, h->sq_a + t_w2 + t_head)}, st)))
      return r;
    if ((r = launch_gemm<T>(h, P_AW1, {
             wgrad_job(h->dha1t, H, h->xst, D, Np, ag + o.a_w1, ag + o.a_b1, h->sq_a + t_w2 + 2 * t_head)}, st)))
      return r;
  }
  if ((r = launch_adam<T>(h, false, 1, st))) return r;
  // ---------------- alpha step (learning.py:225-230, alpha_loss :260-265) ----------------
  if (h->cfg.tune_alpha) {
    if ((r = launch_gemm<T>(h, P_LFWD1, {
             fwd_job(h->ka.w1, h->Dp, h->xs, h->Dp, h->Dp, S.actor + o.a_b1, h->hb1, nullptr, Np, N)}, st)))
      return r;
    if ((r = launch_gemm<T>(h, P_LFWD2, {
             fwd_job(h->ka.w2, H, h->hb1, H, H, S.actor + o.a_b2, h->hb2, nullptr, Np, N)}, st)))
      return r;
    HeadJob lj = policy_job(h->hb2, S.actor, o, eps2);
    lj.logp = h->logp2;
    if ((r = launch_heads<T>(h, P_LHEAD, {lj}, N, st))) return r;
  }
  {
    FinArgs f{};
    f.rowm = h->rowm; f.ldt = Np; f.N = N; f.tune_alpha = h->cfg.tune_alpha;
    f.logp2 = h->logp2; f.la = S.log_alpha; f.metrics = S.metrics; f.steps = h->steps;
    f.lr = dec(h->cfg.critic_lr); f.b1 = dec(h->cfg.adam_beta1); f.b2 = dec(h->cfg.adam_beta2);
    f.eps = h->cfg.adam_eps; f.target_entropy = h->cfg.target_entropy;
    timer_begin(h, P_FIN, st);
    finalize_kernel<<<1, 256, 0, st>>>(f);
    timer_end(h, P_FIN, st);
    SCK_LAUNCH("finalize");
  }
  return 0;
}

ChainJob chain_job(const void* x, int ldx, int K1, const MlpK& k, const float* b1, const float* b2,
                   HeadJob head) {
  ChainJob c{};
  c.x = x; c.ldx = ldx; c.K1 = K1;
  c.w1 = k.w1; c.b1 = b1; c.w2 = k.w2; c.b2 = b2;
  c.head = head;
  return c;
}

template <typename T>
int launch_chain(sac_learner* h, int ph, std::initializer_list<ChainJob> jobs, int n, hipStream_t st) {
  ChainArgs a{};
  int nj = 0;
  for (const ChainJob& j : jobs) a.j[nj++] = j;
  a.N = n;
  a.K = h->K;
  a.ldt = h->Np;
  timer_begin(h, ph, st);
  chain_fwd_kernel<T><<<dim3(cdiv(n, 16), nj), 64 * FW, 0, st>>>(a);
  timer_end(h, ph, st);
  SCK_LAUNCH(pname(ph));
  return 0;
}

// the fused learner step: 12 launches (sac_fused.h), bitwise equal to enqueue_step
template <typename T>
int enqueue_step_fused(sac_learner* h, const sac_batch* b, hipStream_t st) {
  const sac_state& S = h->st;
  const Offs& o = h->off;
  const int N = h->N, Np = h->Np, D = h->D, K = h->K;
  const long long NK = (long long)N * K;
  const long long qb[2] = {0, o.q_per};
  const float* eps = b->noise ? b->noise : h->eps;
  const float *eps0 = eps, *eps1 = eps + NK, *eps2 = eps + 2 * NK;
  int r;
  {  // operand rows (+ device noise)
    PackArgs p{};
    p.s = b->s; p.a = b->a; p.s1 = b->s1;
    p.N = N; p.D = D; p.K = K; p.ldd = h->Dp; p.ldc = h->Cp; p.ldt = Np;
    p.xs = h->xs; p.xs1 = h->xs1; p.xc = h->xc; p.xt = h->xt; p.xp = h->xp;
    p.xst = h->xst; p.xct = h->xct;
    p.eps = b->noise ? nullptr : h->eps;
    p.seed = h->cfg.seed;
    p.counter = h->steps + 3;
    p.probs = b->probabilities; p.prio_exp = -h->cfg.prio_exponent; p.wmax = h->wmax;
    timer_begin(h, P_PACK, st);
    pack_kernel<T><<<std::max(1, std::min(256, cdiv(std::max((long long)N * h->DK, 3 * NK), 256))), 256, 0, st>>>(p);
    timer_end(h, P_PACK, st);
    SCK_LAUNCH("pack");
  }
  // critic step: forward chains (target actor -> a1, Q1, Q2, actor -> pi) ...
  {
    HeadJob tj = policy_job(nullptr, S.target_actor, o, eps0);
    tj.xout = h->xt; tj.ldx = h->Cp; tj.xoff = D; tj.logp = h->logp1;
    HeadJob aj = policy_job(nullptr, S.actor, o, eps1);
    aj.xout = h->xp; aj.ldx = h->Cp; aj.xoff = D; aj.logp = h->logp; aj.save = h->save;
    aj.stdrow = h->rowm + 5 * Np;
    ChainJob j0 = chain_job(h->xs1, h->Dp, h->Dp, h->kta, S.target_actor + o.a_b1, S.target_actor + o.a_b2, tj);
    ChainJob jq[2];
    for (int q = 0; q < 2; ++q) {
      jq[q] = chain_job(h->xc, h->Cp, h->Cp, h->kq[q], S.critic + qb[q] + o.q_b1, S.critic + qb[q] + o.q_b2,
                        q_job(nullptr, S.critic, qb[q], o, q ? h->q2 : h->q1));
      jq[q].h1 = h->hc1[q]; jq[q].h1t = h->hc1t[q]; jq[q].h2 = h->hc2[q]; jq[q].h2t = h->hc2t[q];
    }
    ChainJob j3 = chain_job(h->xs, h->Dp, h->Dp, h->ka, S.actor + o.a_b1, S.actor + o.a_b2, aj);
    j3.h1 = h->ha1; j3.h1t = h->ha1t; j3.h2 = h->ha2; j3.h2t = h->ha2t;
    if ((r = launch_chain<T>(h, P_CFWD, {j0, jq[0], jq[1], j3}, N, st))) return r;
  }
  {  // ... target critic chains, critic loss, row-local critic backward ...
    CChainArgs c{};
    CLossArgs& a = c.L;
    a.w3t1 = S.target_critic + qb[0] + o.q_w3; a.b3t1 = S.target_critic + qb[0] + o.q_b3;
    a.w3t2 = S.target_critic + qb[1] + o.q_w3; a.b3t2 = S.target_critic + qb[1] + o.q_b3;
    a.hc1 = h->hc2[0]; a.hc2 = h->hc2[1];
    a.w3c1 = S.critic + qb[0] + o.q_w3; a.w3c2 = S.critic + qb[1] + o.q_w3;
    a.q1 = h->q1; a.q2 = h->q2; a.logp1 = h->logp1;
    a.r = b->r; a.done = b->done; a.probs = b->probabilities; a.log_alpha = S.log_alpha;
    a.gamma = h->cfg.gamma; a.prio_exp = -h->cfg.prio_exponent;
    a.N = N; a.ldh = H; a.ldt = Np;
    a.prio = b->priorities;
    a.dh1t = h->dh2t[0]; a.dh2t = h->dh2t[1];
    a.dq1t = h->dqt[0]; a.dq2t = h->dqt[1];
    a.rowm = h->rowm;
    a.wmax = h->wmax;
    c.xt = h->xt; c.ldx = h->Cp; c.K1 = h->Cp;
    for (int q = 0; q < 2; ++q) {
      c.tw1[q] = h->ktq[q].w1; c.tw2[q] = h->ktq[q].w2;
      c.tb1[q] = S.target_critic + qb[q] + o.q_b1; c.tb2[q] = S.target_critic + qb[q] + o.q_b2;
      c.w2t[q] = h->kq[q].w2t; c.h1[q] = h->hc1[q]; c.dh1t[q] = h->dhc1t[q];
    }
    timer_begin(h, P_CCHAIN, st);
    critic_chain_kernel<T><<<dim3(cdiv(N, 16), 2), 64 * FW, 0, st>>>(c);
    timer_end(h, P_CCHAIN, st);
    SCK_LAUNCH("critic_loss_chain");
  }
  float* cg = S.critic_grad;
  {  // ... every critic weight gradient, clip + Adam + Polyak
    const int t2 = cdiv(H + 1, 16);
    float* sq1 = h->sq_c + 34 * t2;
    const int t1 = 16 * cdiv(h->DK + 1, 16);
    if ((r = launch_gemm<T>(h, P_CWGRAD, {
             wgrad_job(h->dh2t[0], H, h->hc1t[0], H, Np, cg + qb[0] + o.q_w2, cg + qb[0] + o.q_b2, h->sq_c),
             wgrad_job(h->dh2t[1], H, h->hc1t[1], H, Np, cg + qb[1] + o.q_w2, cg + qb[1] + o.q_b2, h->sq_c + 16 * t2),
             wgrad_job(h->dqt[0], 1, h->hc2t[0], H, Np, cg + qb[0] + o.q_w3, cg + qb[0] + o.q_b3, h->sq_c + 32 * t2),
             wgrad_job(h->dqt[1], 1, h->hc2t[1], H, Np, cg + qb[1] + o.q_w3, cg + qb[1] + o.q_b3, h->sq_c + 33 * t2),
             wgrad_job(h->dhc1t[0], H, h->xct, h->DK, Np, cg + qb[0] + o.q_w1, cg + qb[0] + o.q_b1, sq1),
             wgrad_job(h->dhc1t[1], H, h->xct, h->DK, Np, cg + qb[1] + o.q_w1, cg + qb[1] + o.q_b1, sq1 + t1)}, st)))
      return r;
  }
  if ((r = launch_adam<T>(h, true, 1, st))) return r;
  {  // actor step: Q chains on (s, pi) with the updated critic, actor loss, row-local backward
    AChainArgs c{};
    ALossArgs& a = c.L;
    a.logp = h->logp; a.log_alpha = S.log_alpha; a.N = N; a.ldt = Np; a.rowm = h->rowm;
    ABwdArgs& bb = c.B;
    bb.w1c1 = S.critic + qb[0] + o.q_w1; bb.w1c2 = S.critic + qb[1] + o.q_w1;
    bb.save = h->save; bb.eps = eps1; bb.log_alpha = S.log_alpha;
    bb.wm = S.actor + o.a_wm; bb.wl = S.actor + o.a_wl;
    bb.ha2 = h->ha2;
    bb.D = D; bb.K = K; bb.N = N; bb.ldt = Np;
    bb.w1_so = h->DK; bb.w1_sk = 1; bb.w1_off = D;  // the chain kernel restages them in LDS
    bb.dha2t = h->dha2t; bb.gmt = h->gmt; bb.gut = h->gut;
    c.xp = h->xp; c.ldx = h->Cp; c.K1 = h->Cp;
    for (int q = 0; q < 2; ++q) {
      c.w1[q] = h->kq[q].w1; c.w2[q] = h->kq[q].w2; c.w2t[q] = h->kq[q].w2t;
      c.b1[q] = S.critic + qb[q] + o.q_b1; c.b2[q] = S.critic + qb[q] + o.q_b2;
      c.w3[q] = S.critic + qb[q] + o.q_w3; c.b3[q] = S.critic + qb[q] + o.q_b3;
    }
    c.aw2t = h->ka.w2t; c.ha1 = h->ha1; c.dha1t = h->dha1t;
    timer_begin(h, P_ACHAIN, st);
    actor_chain_kernel<T><<<cdiv(N, 16), 64 * FW, 0, st>>>(c);
    timer_end(h, P_ACHAIN, st);
    SCK_LAUNCH("actor_chain");
  }
  float* ag = S.actor_grad;
  {
    const int t_w2 = 16 * cdiv(H + 1, 16), t_head = cdiv(K, 16) * cdiv(H + 1, 16);
    if ((r = launch_gemm<T>(h, P_AWGRAD, {
             wgrad_job(h->dha2t, H, h->ha1t, H, Np, ag + o.a_w2, ag + o.a_b2, h->sq_a),
             wgrad_job(h->gmt, K, h->ha2t, H, Np, ag + o.a_wm, ag + o.a_bm, h->sq_a + t_w2),
             wgrad_job(h->gut, K, h->ha2t, H, Np, ag + o.a_wl, ag + o.a_bl, h->sq_a + t_w2 + t_head),
             wgrad_job(h->dha1t, H, h->xst, D, Np, ag + o.a_w1, ag + o.a_b1, h->sq_a + t_w2 + 2 * t_head)}, st)))
      return r;
  }
  if ((r = launch_adam<T>(h, false, 1, st))) return r;
  if (h->cfg.tune_alpha) {  // alpha step: a fresh sample from the updated actor
    HeadJob lj = policy_job(nullptr, S.actor, o, eps2);
    lj.logp = h->logp2;
    if ((r = launch_chain<T>(h, P_LCHAIN, {chain_job(h->xs, h->Dp, h->Dp, h->ka, S.actor + o.a_b1,
                                                     S.actor + o.a_b2, lj)}, N, st)))
      return r;
  }
  {
    FinArgs f{};
    f.rowm = h->rowm; f.ldt = Np; f.N = N; f.tune_alpha = h->cfg.tune_alpha;
    f.logp2 = h->logp2; f.la = S.log_alpha; f.metrics = S.metrics; f.steps = h->steps;
    f.lr = dec(h->cfg.critic_lr); f.b1 = dec(h->cfg.adam_beta1); f.b2 = dec(h->cfg.adam_beta2);
    f.eps = h->cfg.adam_eps; f.target_entropy = h->cfg.target_entropy;
    timer_begin(h, P_FIN, st);
    finalize_kernel<<<1, 256, 0, st>>>(f);
    timer_end(h, P_FIN, st);
    SCK_LAUNCH("finalize");
  }
  return 0;
}

template <typename T>
int enqueue_forward(sac_learner* h, const float* obs, int n, hipStream_t st, HeadJob job) {
  const Offs& o = h->off;
  pack_obs_kernel<T><<<std::max(1, std::min(256, cdiv((long long)n * h->D, 256))), 256, 0, st>>>(
      obs, n, h->D, h->Dp, (T*)h->xi);
  SCK_LAUNCH("pack_obs");
  if (h->fused)
    return launch_chain<T>(h, -1, {chain_job(h->xi, h->Dp, h->Dp, h->ka, h->st.actor + o.a_b1,
                                             h->st.actor + o.a_b2, job)}, n, st);
  int r;
  if ((r = launch_gemm<T>(h, -1, {fwd_job(h->ka.w1, h->Dp, h->xi, h->Dp, h->Dp, h->st.actor + o.a_b1,
                                           h->hb1, nullptr, h->Np, n)}, st)))
    return r;
  if ((r = launch_gemm<T>(h, -1, {fwd_job(h->ka.w2, H, h->hb1, H, H, h->st.actor + o.a_b2, h->hb2,
                                           nullptr, h->Np, n)}, st)))
    return r;
  job.h = h->hb2;
  job.ldh = H;
  return launch_heads<T>(h, -1, {job}, n, st);
}

template <typename T>
int enqueue_q_forward(sac_learner* h, const float* obs, const float* act, int n, bool target,
                      float* q1, float* q2, hipStream_t st) {
  const Offs& o = h->off;
  const float* P = target ? h->st.target_critic : h->st.critic;
  const MlpK* k = target ? h->ktq : h->kq;
  pack_sa_kernel<T><<<std::max(1, std::min(256, cdiv((long long)n * h->DK, 256))), 256, 0, st>>>(
      obs, act, n, h->D, h->K, h->Cp, (T*)h->xi2);
  SCK_LAUNCH("pack_sa");
  if (h->fused)
    return launch_chain<T>(h, -1, {
        chain_job(h->xi2, h->Cp, h->Cp, k[0], P + o.q_b1, P + o.q_b2, q_job(nullptr, P, 0, o, q1)),
        chain_job(h->xi2, h->Cp, h->Cp, k[1], P + o.q_per + o.q_b1, P + o.q_per + o.q_b2,
                  q_job(nullptr, P, o.q_per, o, q2))}, n, st);
  int r;
  if ((r = launch_gemm<T>(h, -1, {
           fwd_job(k[0].w1, h->Cp, h->xi2, h->Cp, h->Cp, P + o.q_b1, h->hp1[0], nullptr, h->Np, n),
           fwd_job(k[1].w1, h->Cp, h->xi2, h->Cp, h->Cp, P + o.q_per + o.q_b1, h->hp1[1], nullptr, h->Np, n)}, st)))
    return r;
  if ((r = launch_gemm<T>(h, -1, {
           fwd_job(k[0].w2, H, h->hp1[0], H, H, P + o.q_b2, h->hp2[0], nullptr, h->Np, n),
           fwd_job(k[1].w2, H, h->hp1[1], H, H, P + o.q_per + o.q_b2, h->hp2[1], nullptr, h->Np, n)}, st)))
    return r;
  return launch_heads<T>(h, -1, {q_job(h->hp2[0], P, 0, o, q1), q_job(h->hp2[1], P, o.q_per, o, q2)}, n, st);
}

bool same_batch(const sac_batch& a, const sac_batch& b) { return std::memcmp(&a, &b, sizeof(a)) == 0; }

int run_step(sac_learner* h, const sac_batch* b, hipStream_t st) {
  auto body = [&](hipStream_t s) {
    if (h->fused)
      return h->bf16 ? enqueue_step_fused<__bf16>(h, b, s) : enqueue_step_fused<float>(h, b, s);
    return h->bf16 ? enqueue_step<__bf16>(h, b, s) : enqueue_step<float>(h, b, s);
  };
  if (!h->use_graph || h->timer_phase >= 0) return body(st);
  for (auto& g : h->graphs)
    if (g.exec && same_batch(g.key, *b)) {
      g.used = ++h->tick;
      SCK(hipGraphLaunch(g.exec, st));
      return 0;
    }
  SCK(hipStreamBeginCapture(h->cap, hipStreamCaptureModeThreadLocal));
  const int r = body(h->cap);
  hipGraph_t graph = nullptr;
  const hipError_t ee = hipStreamEndCapture(h->cap, &graph);
  if (r || ee != hipSuccess) {
    if (graph) (void)hipGraphDestroy(graph);
    return r ? r : fail((int)ee, std::string("hipStreamEndCapture: ") + hipGetErrorString(ee));
  }
  hipGraphExec_t exec = nullptr;
  const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (ei != hipSuccess) return fail((int)ei, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
  auto* slot = &h->graphs[0];
  for (auto& g : h->graphs) {
    if (!g.exec) { slot = &g; break; }
    if (g.used < slot->used) slot = &g;
  }
  if (slot->exec) (void)hipGraphExecDestroy(slot->exec);
  slot->exec = exec;
  slot->key = *b;
  slot->used = ++h->tick;
  SCK(hipGraphLaunch(exec, st));
  return 0;
}

void drop_graphs(sac_learner* h) {
  for (auto& g : h->graphs) {
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    g = sac_learner::GraphSlot{};
  }
}

int check_bound(sac_learner* h) {
  if (!h) return fail(IMPALA_E_INVALID, "sac: null handle");
  if (!h->bound) return fail(IMPALA_E_STATE, "sac: state not bound (sac_bind_state)");
  return 0;
}

}  // namespace

extern "C" {

int sac_config_default(sac_config* c) {
  if (!c) return fail(IMPALA_E_INVALID, "sac_config_default: null");
  std::memset(c, 0, sizeof(*c));
  c->obs_dim = 17;
  c->act_dim = 6;
  c->batch_size = 256;
  c->dtype = IMPALA_DTYPE_F32;
  c->critic_lr = 0.003f;
  c->actor_lr = 0.0003f;
  c->adam_beta1 = 0.9f;
  c->adam_beta2 = 0.999f;
  c->adam_eps = 1e-5f;
  c->max_grad_norm = 40.f;
  c->tau = 0.005f;
  c->gamma = 0.99f;
  c->tune_alpha = 1;
  c->target_entropy = -6.f;
  c->prio_exponent = 0.4f;
  c->seed = 0;
  return 0;
}

size_t sac_actor_param_count(int D, int K) { return (size_t)offsets(D, K).a_total; }
size_t sac_critic_param_count(int D, int K) { return (size_t)offsets(D, K).c_total; }

int sac_create(const sac_config* cfg, int device, sac_learner** out) {
  if (!cfg || !out) return fail(IMPALA_E_INVALID, "sac_create: null argument");
  *out = nullptr;
  if (cfg->obs_dim < 1 || cfg->obs_dim > 4096) return fail(IMPALA_E_INVALID, "sac_create: obs_dim out of range");
  if (cfg->act_dim < 1 || cfg->act_dim > SAC_MAX_ACT)
    return fail(IMPALA_E_INVALID, "sac_create: act_dim must be 1..16");
  if (cfg->batch_size < 1 || cfg->batch_size > (1 << 16))
    return fail(IMPALA_E_INVALID, "sac_create: batch_size out of range");
  if (cfg->dtype != IMPALA_DTYPE_F32 && cfg->dtype != IMPALA_DTYPE_BF16)
    return fail(IMPALA_E_INVALID, "sac_create: dtype");
  sac_learner* h = new (std::nothrow) sac_learner();
  if (!h) return fail(IMPALA_E_INVALID, "sac_create: out of host memory");
  h->cfg = *cfg;
  h->device = device;
  h->bf16 = cfg->dtype == IMPALA_DTYPE_BF16;
  h->esz = h->bf16 ? 2 : 4;
  h->N = cfg->batch_size;
  h->Np = rup(h->N, 32);
  h->D = cfg->obs_dim;
  h->K = cfg->act_dim;
  h->DK = h->D + h->K;
  h->Dp = rup(h->D, 32);
  h->Cp = rup(h->DK, 32);
  h->Dt = rup(h->D + 1, 16);
  h->Ct = rup(h->DK + 1, 16);
  h->off = offsets(h->D, h->K);
  const char* g = std::getenv("SAC_GRAPH");
  h->use_graph = !(g && g[0] == '0');
  const char* fz = std::getenv("SAC_FUSED");
  h->fused = !(fz && fz[0] == '0') && h->Cp <= H;  // the chain kernels stage K1 <= 256
  auto cleanup = [&](int code) {
    if (h->arena) (void)hipFree(h->arena);
    if (h->cap) (void)hipStreamDestroy(h->cap);
    delete h;
    return code;
  };
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return cleanup(fail((int)e, std::string("hipSetDevice: ") + hipGetErrorString(e)));
  carve(h);  // size pass
  h->arena_size = h->arena_used;
  e = hipMalloc(&h->arena, h->arena_size);
  if (e != hipSuccess) return cleanup(fail((int)e, std::string("hipMalloc: ") + hipGetErrorString(e)));
  carve(h);
  e = hipMemset(h->arena, 0, h->arena_size);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->cap, hipStreamNonBlocking);
  if (e != hipSuccess) return cleanup(fail((int)e, std::string("sac_create: ") + hipGetErrorString(e)));
  // rows of ones (bias gradients) after the last feature of every weight-gradient operand
  int r = 0;
  auto ones = [&](void* base, int row, int ld) {
    return h->bf16 ? fill_ones<__bf16>(h, base, row, ld) : fill_ones<float>(h, base, row, ld);
  };
  r = r ? r : ones(h->xst, h->D, h->Np);
  r = r ? r : ones(h->xct, h->DK, h->Np);
  for (int q = 0; q < 2 && !r; ++q) {
    r = ones(h->hc1t[q], H, h->Np);
    r = r ? r : ones(h->hc2t[q], H, h->Np);
  }
  r = r ? r : ones(h->ha1t, H, h->Np);
  r = r ? r : ones(h->ha2t, H, h->Np);
  if (!r) {
    e = hipDeviceSynchronize();
    if (e != hipSuccess) r = fail((int)e, std::string("sac_create: ") + hipGetErrorString(e));
  }
  if (r) return cleanup(r);
  *out = h;
  return 0;
}

int sac_destroy(sac_learner* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  drop_graphs(h);
  for (auto& e : h->ev) (void)hipEventDestroy(e);
  if (h->arena) (void)hipFree(h->arena);
  if (h->cap) (void)hipStreamDestroy(h->cap);
  delete h;
  return 0;
}

int sac_bind_state(sac_learner* h, const sac_state* s, void* stream) {
  if (!h || !s) return fail(IMPALA_E_INVALID, "sac_bind_state: null argument");
  if (!s->actor || !s->actor_grad || !s->actor_m || !s->actor_v || !s->target_actor || !s->critic ||
      !s->critic_grad || !s->critic_m || !s->critic_v || !s->target_critic || !s->log_alpha ||
      !s->metrics)
    return fail(IMPALA_E_INVALID, "sac_bind_state: every buffer is required");
  SCK(hipSetDevice(h->device));
  drop_graphs(h);
  h->st = *s;
  h->bound = true;
  return sac_refresh_weights(h, stream);
}

int sac_refresh_weights(sac_learner* h, void* stream) {
  if (int r = check_bound(h)) return r;
  SCK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  for (int c = 0; c < 2; ++c) {
    const AdamNetArgs a = adam_args(h, c == 1, 0);
    if (h->bf16) adam_net_kernel<__bf16><<<cdiv(a.n, 256), 256, 0, st>>>(a);
    else adam_net_kernel<float><<<cdiv(a.n, 256), 256, 0, st>>>(a);
    SCK_LAUNCH("sac_refresh_weights");
  }
  return 0;
}

int sac_set_steps(sac_learner* h, int64_t cs, int64_t as, int64_t ls, void* stream) {
  if (!h) return fail(IMPALA_E_INVALID, "sac_set_steps: null handle");
  SCK(hipSetDevice(h->device));
  static thread_local int64_t v[4];
  v[0] = cs; v[1] = as; v[2] = ls; v[3] = cs;
  SCK(hipMemcpyAsync(h->steps, v, sizeof(v), hipMemcpyHostToDevice, (hipStream_t)stream));
  SCK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

int sac_train_step(sac_learner* h, const sac_batch* b, void* stream) {
  if (int r = check_bound(h)) return r;
  if (!b || !b->s || !b->a || !b->r || !b->s1 || !b->done)
    return fail(IMPALA_E_INVALID, "sac_train_step: s, a, r, s1, done are required");
  SCK(hipSetDevice(h->device));
  return run_step(h, b, (hipStream_t)stream);
}

int sac_act(sac_learner* h, const float* obs, int n, const float* noise, float noise_scale,
            float action_scale, float action_bias, float* action, void* stream) {
  if (int r = check_bound(h)) return r;
  if (!obs || !action || n < 1 || n > h->N)
    return fail(IMPALA_E_INVALID, "sac_act: need obs/action and 1 <= n <= batch_size");
  SCK(hipSetDevice(h->device));
  HeadJob j = policy_job(nullptr, h->st.actor, h->off, noise);
  j.kind = HK_ACT;
  j.noise_scale = noise_scale;
  j.act_scale = action_scale;
  j.act_bias = action_bias;
  j.act = action;
  hipStream_t st = (hipStream_t)stream;
  return h->bf16 ? enqueue_forward<__bf16>(h, obs, n, st, j) : enqueue_forward<float>(h, obs, n, st, j);
}

int sac_policy(sac_learner* h, const float* obs, int n, const float* noise, float* mean,
               float* log_std, float* action, float* log_prob, float* std_out, void* stream) {
  if (int r = check_bound(h)) return r;
  if (!obs || n < 1 || n > h->N)
    return fail(IMPALA_E_INVALID, "sac_policy: need obs and 1 <= n <= batch_size");
  SCK(hipSetDevice(h->device));
  HeadJob j = policy_job(nullptr, h->st.actor, h->off, noise);
  j.act = action;
  j.logp = log_prob;
  j.stdout_ = std_out;
  j.mean_out = mean;
  j.ls_out = log_std;
  hipStream_t st = (hipStream_t)stream;
  return h->bf16 ? enqueue_forward<__bf16>(h, obs, n, st, j) : enqueue_forward<float>(h, obs, n, st, j);
}

int sac_q_forward(sac_learner* h, const float* obs, const float* act, int n, int target, float* q1,
                  float* q2, void* stream) {
  if (int r = check_bound(h)) return r;
  if (!obs || !act || !q1 || !q2 || n < 1 || n > h->N)
    return fail(IMPALA_E_INVALID, "sac_q_forward: need obs/act/q1/q2 and 1 <= n <= batch_size");
  SCK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  return h->bf16 ? enqueue_q_forward<__bf16>(h, obs, act, n, target != 0, q1, q2, st)
                 : enqueue_q_forward<float>(h, obs, act, n, target != 0, q1, q2, st);
}

int sac_phase_count(void) { return P_COUNT; }
const char* sac_phase_name(int p) { return (p >= 0 && p < P_COUNT) ? kPhase[p] : nullptr; }

int sac_timer_start(sac_learner* h, int phase, int max_launches) {
  if (!h || phase < 0 || phase >= P_COUNT || max_launches < 1)
    return fail(IMPALA_E_INVALID, "sac_timer_start: bad argument");
  SCK(hipSetDevice(h->device));
  while ((int)h->ev.size() < 2 * max_launches) {
    hipEvent_t e;
    SCK(hipEventCreate(&e));
    h->ev.push_back(e);
  }
  h->timer_phase = phase;
  h->timer_max = max_launches;
  h->timer_n = 0;
  return 0;
}

int sac_timer_read(sac_learner* h, float* total_ms, int* launches) {
  if (!h || !total_ms || !launches) return fail(IMPALA_E_INVALID, "sac_timer_read: null argument");
  SCK(hipSetDevice(h->device));
  float tot = 0.f;
  for (int i = 0; i < h->timer_n; ++i) {
    SCK(hipEventSynchronize(h->ev[2 * i + 1]));
    float ms = 0.f;
    SCK(hipEventElapsedTime(&ms, h->ev[2 * i], h->ev[2 * i + 1]));
    tot += ms;
  }
  *total_ms = tot;
  *launches = h->timer_n;
  h->timer_phase = -1;
  h->timer_n = 0;
  return 0;
}

int sac_sample(uint64_t seed, uint64_t counter, int64_t size, int n, int64_t* idx,
               float* probabilities, const void* const* src, void* const* dst,
               const size_t* row_bytes, int nfields, void* stream) {
  if (!idx || n < 1 || size < 1) return fail(IMPALA_E_INVALID, "sac_sample: need idx, n >= 1, size >= 1");
  if (nfields < 0 || nfields > 8 || (nfields && (!src || !dst || !row_bytes)))
    return fail(IMPALA_E_INVALID, "sac_sample: nfields must be 0..8 with src/dst/row_bytes");
  hipStream_t st = (hipStream_t)stream;
  sample_kernel<<<1, 256, 0, st>>>(seed, counter, size, n, idx, probabilities);
  SCK_LAUNCH("sample");
  if (nfields == 0) return 0;
  SGather g{};
  for (int f = 0; f < nfields; ++f) {
    if (!src[f] || !dst[f] || row_bytes[f] == 0) return fail(IMPALA_E_INVALID, "sac_sample: bad field");
    g.src[f] = (const char*)src[f];
    g.dst[f] = (char*)dst[f];
    g.rb[f] = (long long)row_bytes[f];
  }
  g.nf = nfields;
  g.n = n;
  g.idx = idx;
  sample_gather_kernel<<<dim3(n, nfields), 64, 0, st>>>(g);
  SCK_LAUNCH("sample_gather");
  return 0;
}

}  // extern "C"
