// Fused learner head: actor/critic heads forward, log-softmax / ratio / V-trace / loss
// (agents/impala/learning.py:144-170), the heads' input gradient through GELU (dz) and the
// heads' weight-gradient partial -- one workgroup per group of whole trajectories.
//
//   phase 1  stage h[F][256] of the group's F frames in LDS; heads = Wh . h + bh (MFMA)
//   phase 2a all four waves, a quad of threads per frame, four actions per thread: log-softmax
//            of the policy and behaviour logits, entropy, KL, log pi(a), rho (quad DPP sums)
//   phase 2b wave 0, one lane per (trajectory, t) = one frame: the V-trace in the reference's
//            sequential order (kernels.h vtrace_lane) -> d loss / d value and d loss / d log
//            pi(a) under the gradient mode (vtrace_grad_lane), the loss partials
//   phase 2c the quads again: the frame's d loss / d heads row -> dH[F][32] in LDS
//            (the statistics on wave 0 alone, one lane per frame over all 15 actions, took
//            6.3k cycles of one SIMD: hstamps5, r04f; frame x 16-action lanes with row
//            reductions 4k cycles for the statistics alone: headstamps4, r04c)
//   phase 3  dz[f][j] = gelu'(z[f][j]) * sum_o' dH[f][o'] Wh[o'][j]        (MFMA, K = 32;
//            gelu'(z) comes precomputed from the FC forward epilogue)
//   phase 4  dWh[o'][j] += sum_f dH[f][o'] h[f][j]  (MFMA over frames, LDS transpose reads)
//            -> fp32 partial slab per workgroup (+ bias sums), reduced by reduce_grads
//
// F = (64 / S) * T <= 64 frames (S = segment = next pow2 >= T), i.e. one wavefront of lanes.
#pragma once
#include "gemm.h"
#include "kernels.h"
#include "net.h"

using namespace net;

// the hardware exp2 / log2 (v_exp_f32 / v_log_f32, ~1 ulp): exp2f / log2f add a denormal
// range reduction around them that costs 4 instructions per call and changes nothing here
DEV float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
DEV float fast_log(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }

struct HeadArgs {
  // phase 1 inputs
  const void* h;      // T [N][256]
  const float* zg;    // [N][256] gelu'(pre-GELU), from the FC forward
  const void* wh;     // T [16][256]
  const void* wht;    // T [256][32]
  const float* bh;    // [16]
  // batch
  const int64_t* act; const float* rew; const float* disc; const float* mu;
  int B, T, A, S, TPW;  // TPW = trajectories per workgroup = 64 / S
  int vt_mode;          // VT_SG_* (kernels.h): what the V-trace gradient treats as constant
  float lam, crho, cpg, ent_coef;
  float clip_lo, clip_hi;  // PPO: ratio clamp bounds (1 -+ clip_coeff)
  // outputs
  void* dz;             // T [N][256]
  float* partials;      // [gridDim.x][8] loss partial sums
  float* slab_h;        // [gridDim.x][16][256]
  float* slab_bh;       // [gridDim.x][16]
  float* heads_out;     // optional [N][16] (logits + value), nullptr = skip
  float* vt_dbg;        // optional debug export (IMPALA only): adv, err, q [3][B][T-1] then
                        // rho [B][T] and the values v [B][T] the scan ran on -- the step's own
                        // V-trace inputs / outputs (impala_set_debug_vtrace)
};

// workgroups per trajectory group (hidden-column slices).  fp32 8: 32 columns each, so the
// kernel fills the 256 CUs at B = 64 (32 groups), and phases 3 / 4 run half the columns per
// workgroup (the waves split the frame tiles / the frame range instead): 7.9 -> 7.35 us.  bf16
// 4 (64 columns, one tile per wave): 8 measured 5.7 -> 6.0 us (profiles/r05hs8)
template <typename T> constexpr int head_split() { return sizeof(T) == 4 ? 8 : 4; }

// grid (groups, head_split): all head_split workgroups of a group redo phases 1-2 (cheap: h is an
// L2 hit and the loss is one wavefront), then each takes a 64-column slice of dz / dWh.
// PPO = true: the PPO clipped-surrogate loss (kernels.h::ppo_frame) on flat transitions (T = 1,
// one lane per transition, targets in `rew`, `disc` unused) instead of V-trace.
template <typename T, bool PPO = false, class O = ObsDirect>
__global__ __launch_bounds__(256) void head_step_kernel(const HeadArgs a, const O fm) {
  constexpr int HEAD_JC = HID / head_split<T>();  // hidden columns per workgroup in phases 3/4
  static_assert(HEAD_JC == 64 || HEAD_JC == 32, "phase 3 / 4 wave map");
  constexpr int HEAD_CW = HEAD_JC / 16;           // column tiles per workgroup (4 or 2)
  using F = Frag<T>;
  typedef typename F::vec V;
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int LDH = HID + VEC;     // h tile row (elements)
  constexpr int LDD = HPAD + VEC;    // dH tile row
  __shared__ __attribute__((aligned(16))) T hs[64 * LDH];
  __shared__ __attribute__((aligned(16))) T dHs[64 * LDD];
  __shared__ float lg_s[64][HEADS + 1];
  __shared__ __attribute__((aligned(16))) float zs[64 * (HEAD_JC + 4)];  // z slice (phase 3)
  __shared__ float bred[4][HEADS];
  // the heads weights [16][256 + VEC], staged once per workgroup (each wave used to load all 16
  // KB of fragments itself: 64 KB of the ~155 KB a workgroup loaded, headstamps4 r04c)
  __shared__ __attribute__((aligned(16))) T whs[HEADS * LDH];
  __shared__ f32x4 fst[64];    // per frame: H, KL, log pi(a), rho (phase 2a -> 2b)
  __shared__ float kd[64][2];  // per frame: d loss / d log pi(a), d loss / d value (2b -> 2c)
  __shared__ f32x4 p4[HEAD_CW == 2 ? 2 : 1][64];  // phase 4 (2 column tiles): the second frame half's partials
  // the wave index as a scalar: `wave == 0` branches are uniform (no exec-mask joins)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T_ = a.T, S = a.S;
  const int traj0 = blockIdx.x * a.TPW;
  const int ntraj = min(a.TPW, a.B - traj0);
  const int nf = ntraj * T_;                       // valid frames of this workgroup (>= 1)
  const size_t f0 = (size_t)traj0 * T_;            // first global frame
  const T* hg = reinterpret_cast<const T*>(a.h);
  const int jw = blockIdx.y * HEAD_JC;            // this workgroup's hidden-column slice
  const bool lead = blockIdx.y == 0;              // writes the per-group outputs
  const int A = a.A, L = T_ - 1;
  // wave 0, phase 2b: one lane per (trajectory, t)
  const int tl = lane / S, t = lane % S;
  const bool valid = wave == 0 && tl < ntraj && t < T_;
  const bool inL = valid && t < L;
  const int fl = valid ? tl * T_ + t : 0;
  // phases 2a / 2c: a quad of threads per frame fq, four actions 4 q .. 4 q + 3 each
  const int fq = tid >> 2, q4 = (tid & 3) * 4;
  const size_t nq = f0 + min(fq, nf - 1);
  // ---- every global load of the kernel is issued here, unconditionally, in one round trip:
  // the batch values, h rows, this workgroup's z slice, the heads weights (both orientations)
  // and bias.  Row indices are clamped into the group: rows past the group's frames hold a
  // copy of its last frame, which only meets zero dH rows (phase 4, bias sums) or outputs
  // nobody stores.  (Guarded loads made the compiler wait for each one inside its branch:
  // three serial round trips, 4.8k cycles before phase 1, hstamps5 r04f.)  The action is read
  // as the low word of the int64 (actions are in [0, A)): a 64-bit load whose dead high half
  // gets its register reused costs a wait for the load. ----
  // (fm.map: the frame's row in the batch arrays -- a replay ring's row for ObsRows)
  const size_t nqb = fm.map(nq);
  const int act_q = reinterpret_cast<const int*>(a.act)[2 * nqb];
  float mub[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) mub[u] = a.mu[nqb * A + min(q4 + u, A - 1)];
  float r = 0.f, g = 0.f;
  if (wave == 0) {
    const size_t fb = fm.map(f0 + fl);
    r = a.rew[fb];
    if constexpr (!PPO) g = a.disc[fb];
  }
  constexpr int NHV = 64 * (HID / VEC) / 256, NZV = 64 * (HEAD_JC / 4) / 256;
  constexpr int NKH = HID / F::KSTEP, NKT = HPAD / F::KSTEP;
  const int kl = F::KPL * (lane >> 4);
  V hv[NHV];
  f32x4 zv[NZV];
#pragma unroll
  for (int i = 0; i < NHV; ++i) {
    const int e = tid + i * 256, f = min(e / (HID / VEC), nf - 1), c = (e % (HID / VEC)) * VEC;
    hv[i] = *reinterpret_cast<const V*>(hg + (f0 + f) * HID + c);
  }
#pragma unroll
  for (int i = 0; i < NZV; ++i) {
    const int e = tid + i * 256, f = min(e / (HEAD_JC / 4), nf - 1), c = (e % (HEAD_JC / 4)) * 4;
    zv[i] = *reinterpret_cast<const f32x4*>(a.zg + (f0 + f) * HID + jw + c);
  }
  constexpr int NWV = HEADS * (HID / VEC) / 256;  // 16-byte vectors of Wh per thread
  V whv[NWV], wtf[NKT];
  {
    const T* wh = reinterpret_cast<const T*>(a.wh);
    const T* wht = reinterpret_cast<const T*>(a.wht);
#pragma unroll
    for (int i = 0; i < NWV; ++i) whv[i] = F::load(wh + (size_t)(tid + i * 256) * VEC);
#pragma unroll
    for (int ks = 0; ks < NKT; ++ks)
      wtf[ks] = F::load(wht + (jw + (wave % HEAD_CW) * 16 + (lane & 15)) * HPAD + ks * F::KSTEP + kl);
  }
  float bhv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bhv[q] = a.bh[4 * (lane >> 4) + q];
  // ---- phase 1: stage h and z, zero dH, heads forward ----
#pragma unroll
  for (int i = 0; i < NHV; ++i) {
    const int e = tid + i * 256, f = e / (HID / VEC), c = (e % (HID / VEC)) * VEC;
    *reinterpret_cast<V*>(hs + f * LDH + c) = hv[i];
  }
#pragma unroll
  for (int i = 0; i < NZV; ++i) {
    const int e = tid + i * 256, f = e / (HEAD_JC / 4), c = (e % (HEAD_JC / 4)) * 4;
    *reinterpret_cast<f32x4*>(zs + f * (HEAD_JC + 4) + c) = zv[i];
  }
#pragma unroll
  for (int i = 0; i < NWV; ++i) {
    const int e = tid + i * 256, r = e / (HID / VEC), c = (e % (HID / VEC)) * VEC;
    *reinterpret_cast<V*>(whs + r * LDH + c) = whv[i];
  }
  for (int e = tid; e < 64 * LDD / VEC; e += 256) *reinterpret_cast<V*>(dHs + e * VEC) = F::zero();
  __syncthreads();
  {
    // four accumulators over interleaved k-steps (ks % 4), summed in a fixed order: the MFMAs
    // issue back to back instead of waiting on one accumulator's dependent latency
    const int f = wave * 16 + (lane & 15);
    constexpr int NA = NKH >= 4 ? 4 : 1;
    f32x4 acc[NA];
#pragma unroll
    for (int u = 0; u < NA; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k4 = 0; k4 < NKH; k4 += NA) {
      V w[NA], hf[NA];
#pragma unroll
      for (int u = 0; u < NA; ++u) {
        w[u] = *reinterpret_cast<const V*>(whs + (lane & 15) * LDH + (k4 + u) * F::KSTEP + kl);
        hf[u] = *reinterpret_cast<const V*>(hs + f * LDH + (k4 + u) * F::KSTEP + kl);
      }
#pragma unroll
      for (int e = 0; e < F::NE; ++e)
#pragma unroll
        for (int u = 0; u < NA; ++u) acc[u] = F::mma_e(e, w[u], hf[u], acc[u]);
    }
    f32x4 hsum = acc[0];
    if constexpr (NA == 4) hsum = (acc[0] + acc[1]) + (acc[2] + acc[3]);
#pragma unroll
    for (int q = 0; q < 4; ++q) lg_s[f][4 * (lane >> 4) + q] = hsum[q] + bhv[q];
  }
  __syncthreads();
  if (a.heads_out && lead) {
    for (int e = tid; e < nf * HEADS; e += 256)
      a.heads_out[(f0 + e / HEADS) * HEADS + e % HEADS] = lg_s[e / HEADS][e % HEADS];
  }
  // ---- phase 2a: per-frame statistics, a quad of threads per frame (all four waves) ----
  const int aa = min(act_q, A - 1);
  float pq[4], lpq[4];  // this thread's p_j and log p_j, kept for phase 2c
  float Hq;
  {
    float lg[4], ex[4];
    bool in[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      in[u] = q4 + u < A;
      lg[u] = lg_s[fq][min(q4 + u, A - 1)];
    }
    float m = -INFINITY, mm = -INFINITY;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (in[u]) {
        m = fmaxf(m, lg[u]);
        mm = fmaxf(mm, mub[u]);
      }
    m = quad_max(m);
    mm = quad_max(mm);
    float s = 0.f, sm = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ex[u] = in[u] ? fast_exp(lg[u] - m) : 0.f;
      s += ex[u];
      sm += in[u] ? fast_exp(mub[u] - mm) : 0.f;
    }
    s = quad_sum(s);
    sm = quad_sum(sm);
    const float lse = m + fast_log(s), lse_mu = mm + fast_log(sm), inv = 1.f / s;
    float H = 0.f, kld = 0.f, logpa = 0.f, logmua = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float logp = lg[u] - lse, pp = ex[u] * inv, lmu = mub[u] - lse_mu;
      pq[u] = pp;
      lpq[u] = logp;
      if (in[u]) {
        H -= pp * logp;
        kld += pp * (logp - lmu);
        if (q4 + u == aa) {
          logpa = logp;
          logmua = lmu;
        }
      }
    }
    // the one thread holding action a contributes log pi(a) / log mu(a), the others 0
    H = quad_sum(H);
    kld = quad_sum(kld);
    logpa = quad_sum(logpa);
    logmua = quad_sum(logmua);
    Hq = H;
    if ((tid & 3) == 0) fst[fq] = f32x4{H, kld, logpa, fast_exp(logpa - logmua)};
  }
  __syncthreads();
  // ---- phase 2b: wave 0, one lane per frame: V-trace / PPO, d loss / d log pi(a), d loss /
  // d value, the loss partials ----
  if (wave == 0) {
    const int f = fl;
    const f32x4 st = fst[f];
    float H = st[0], kld = st[1], logpa = st[2];
    float rho = valid ? st[3] : 0.f;
    if (!valid) { H = 0.f; kld = 0.f; logpa = 0.f; r = 0.f; g = 0.f; }
    const float v = valid ? lg_s[f][VCOL] : 0.f;
    float kappa = 0.f, dv = 0.f;  // d loss / d log pi(a), d loss / d value of this frame
    if constexpr (PPO) {
      const PpoFrame pf = ppo_frame(rho, v, r, a.clip_lo, a.clip_hi);
      const float c = 1.f / (float)a.B;
      kappa = c * pf.dr * rho;
      dv = -pf.adv * c;
      float q[6] = {valid ? pf.pgl : 0.f, valid ? pf.adv * pf.adv : 0.f, H, kld, rho, r};
#pragma unroll
      for (int k = 0; k < 6; ++k) q[k] = wave_sum(q[k]);
      if (lane == 0 && lead) {
        float* pp = a.partials + blockIdx.x * 8;
#pragma unroll
        for (int k = 0; k < 6; ++k) pp[k] = q[k];
      }
    } else {
      const int tv = valid ? t : 64;  // lanes of missing trajectories are dead in the scans
      const float v_n = shift_down1(v);
      const VtLane o = vtrace_lane(v, v_n, v_n, r, g, rho, tv, L, a.lam, a.crho, a.cpg);
      const float err = o.err, qq = o.q, adv = o.adv;
      const float c_pg = 1.f / (float)(a.B * L);
      const VtGrad gr = vtrace_grad_lane(o, a.vt_mode, v, v_n, r, g, rho, logpa, tv, L, a.lam,
                                         a.crho, a.cpg, c_pg);
      kappa = gr.dlogpa;
      dv = gr.dv;
      if (a.vt_dbg && lead && valid) {
        const size_t BL = (size_t)a.B * L, ob = (size_t)(traj0 + tl) * L + t;
        if (inL) {
          a.vt_dbg[ob] = adv;
          a.vt_dbg[BL + ob] = err;
          a.vt_dbg[2 * BL + ob] = qq;
        }
        a.vt_dbg[3 * BL + f0 + fl] = rho;
        a.vt_dbg[3 * BL + (size_t)a.B * T_ + f0 + fl] = v;
      }
      float s0 = inL ? logpa * adv : 0.f, s1 = inL ? err * err : 0.f;
      s0 = wave_sum(s0); s1 = wave_sum(s1);
      const float s2 = wave_sum(H), s3 = wave_sum(kld), s4 = wave_sum(rho);
      if (lane == 0 && lead) {
        float* pp = a.partials + blockIdx.x * 8;
        pp[0] = s0; pp[1] = s1; pp[2] = s2; pp[3] = s3; pp[4] = s4;
      }
    }
    if (valid) {
      kd[f][0] = kappa;
      kd[f][1] = dv;
    }
  }
  __syncthreads();
  // ---- phase 2c: dH[f][j] = ke p_j (log p_j + H) + kappa ([j == a] - p_j), dH[f][value] = dv
  // (quads again; rows of frames outside the group stay zero) ----
  if (fq < nf) {
    const float ke = a.ent_coef * (1.f / (float)(a.B * T_));  // d(-ent_coef * mean H) / d H
    const float kappa = kd[fq][0], dv = kd[fq][1];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = q4 + u;
      if (j < A)
        dHs[fq * LDD + j] = (T)(ke * pq[u] * (lpq[u] + Hq) + kappa * ((j == aa ? 1.f : 0.f) - pq[u]));
      else if (j == VCOL)
        dHs[fq * LDD + j] = (T)dv;
    }
  }
  __syncthreads();
  // ---- phase 3: dz = gelu'(z) * (dH . Wh)   rows j (256: wave w -> 4 row tiles), cols f ----
  {
    T* dz = reinterpret_cast<T*>(a.dz);
    {
      // wave: column tile wave % HEAD_CW, frame tiles wave / HEAD_CW, + 4 / HEAD_CW, ...
      const int j0 = jw + (wave % HEAD_CW) * 16;
#pragma unroll
      for (int ct = wave / HEAD_CW; ct < 4; ct += 4 / HEAD_CW) {
        if (ct * 16 >= nf) break;  // frame tiles past the group's frames (uniform)
        const int f = ct * 16 + (lane & 15);
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < HPAD / F::KSTEP; ++ks)
          acc = F::mma(wtf[ks], *reinterpret_cast<const V*>(dHs + f * LDD + ks * F::KSTEP + kl), acc);
        if (f < nf) {
          const int j = j0 + 4 * (lane >> 4);
          const f32x4 zz = *reinterpret_cast<const f32x4*>(zs + f * (HEAD_JC + 4) + j - jw);
          float o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = acc[q] * zz[q];
          store4(dz + (f0 + f) * HID + j, o);
        }
      }
    }
  }
  // ---- phase 4: dWh partial = dH^T . h over this group's frames (k = frame) ----
  {
    // wave: column tile wave % HEAD_CW over frames [k0, k0 + KR): all 64 (4 tiles), or the
    // half wave / HEAD_CW (2 tiles: the halves summed in order through LDS)
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const int c0 = jw + (wave % HEAD_CW) * 16;
    constexpr int KR = 64 * HEAD_CW / 4;
    const int k0 = (wave / HEAD_CW) * KR;
#pragma unroll
    for (int kk = 0; kk < KR; kk += F::KSTEP)  // k-steps past the group's frames: dH rows 0
      if (k0 + kk < nf)
        acc = F::mma(lds_frag_k(dHs + (k0 + kk) * LDD, LDD, lane),
                     lds_frag_k(hs + (k0 + kk) * LDH + c0, LDH, lane), acc);
    if constexpr (HEAD_CW == 2) {
      if (wave >= 2) p4[wave - 2][lane] = acc;
      __syncthreads();
      if (wave < 2) acc += p4[wave][lane];
    }
    float* sl = a.slab_h + (size_t)blockIdx.x * HEADS * HID;
    if (wave < HEAD_CW) {
#pragma unroll
      for (int q = 0; q < 4; ++q) sl[(4 * (lane >> 4) + q) * HID + c0 + (lane & 15)] = acc[q];
    }
    if (lead) {
    {  // bias = sum over frames of dH: 16 frame groups x 16 heads, fixed-order tree
      const int o = tid & 15, fg = tid >> 4;
      float b = 0.f;
      for (int f = fg; f < nf; f += 16) b += (float)dHs[f * LDD + o];
      b = xor32_sum(xor16_sum(b));
      if ((lane >> 4) == 0) bred[wave][o] = b;
      __syncthreads();
      if (tid < HEADS)
        a.slab_bh[(size_t)blockIdx.x * HEADS + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];
    }
    }
  }
}
