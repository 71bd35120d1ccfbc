// libimpala_hip.so — C-ABI of the MI355X-native IMPALA learner (see include/impala_hip.h).
//
// One handle = one learner replica on one device.  The handle owns the activation, gradient
// slab and kernel-layout weight workspaces (hipMalloc'd once at create, sized for B*T
// frames); the caller owns the canonical parameters, gradients, Adam moments and the metrics
// buffer (bound with impala_bind_state), so the Python host exposes them as ordinary torch
// tensors (state_dict, checkpoint, RCCL all-reduce) without copies.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <cctype>
#include <type_traits>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/impala_hip.h"
#include "head.h"
#include "hostpool.h"
#include "kernels.h"
#include "lnc3.h"
#include "ops.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

}  // namespace

// shared with the SAC translation unit (sac.hip): one last-error slot per thread for the library
namespace impala_internal {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace impala_internal

namespace {

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return fail((int)e_, std::string(#x) + ": " + hipGetErrorString(e_));           \
  } while (0)

#define CK_LAUNCH(name)                                                                \
  do {                                                                                 \
    hipError_t e_ = hipGetLastError();                                                 \
    if (e_ != hipSuccess)                                                              \
      return fail((int)e_, std::string("launch ") + name + ": " + hipGetErrorString(e_)); \
  } while (0)

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}
// recover the decimal constant a float config value was written as (0.9f -> 0.9)
inline double dec(float x) {
  if (x == 0.f) return 0.0;
  const double e = std::floor(std::log10(std::fabs((double)x)));
  const double s = std::pow(10.0, 7.0 - e);
  return std::round((double)x * s) / s;
}

struct Split {
  int S = 1, mps = 32;  // splits, m per split
};
// direct (one-split) FC weight-gradient tile: BR x BC outputs, WR x WC waves, G 4-wave groups
constexpr int FCD_BR = 32, FCD_BC = 64, FCD_WR = 2, FCD_WC = 2, FCD_G = 4, FCD_PD = 2;
// fp32 FC forward K loop: chunks held ahead, accumulator chains (gemm.h gemm_tile_body).
// PF / KACC 1 / 1: 13.97 us, 2 / 1: 13.40, 1 / 2: 14.20, 2 / 2: 13.67-13.69 (r04v2,
// tools/var_specs/fcpf.py); 2 / 1 keeps the summation order, so the output bits are unchanged
constexpr int FCF_PF = 2, FCF_KACC = 1;
// fp32 FC forward: FCF_BR (hidden) x FCF_BC (frames) tiles whose FCF_NW waves split each
// chunk's k-steps (gemm_tile_body KW).  16 x 80 on 8 waves: 256 tiles at N = 1280, one per CU,
// two waves per SIMD (the 32 x 32 tiles put two on 64 CUs, whose MFMA time bounds the kernel;
// 32 x 48 on 4 / 8 waves: 12.3 / 11.7 us, 16 x 80 on 8: 11.4 us; profiles/r05kw)
constexpr bool FCF_KW = true;
constexpr int FCF_BR = 16, FCF_BC = 80;
constexpr int FCF_NW = 8;
Split plan_split(long M, int tiles, int target_wgs, int chunk = 64) {
  Split s;
  const long chunks = (M + chunk - 1) / chunk;
  long S = (target_wgs + tiles - 1) / tiles;
  if (S < 1) S = 1;
  if (S > chunks) S = chunks;
  long mps = ((M + S - 1) / S + chunk - 1) / chunk * chunk;
  s.mps = (int)mps;
  s.S = (int)((M + mps - 1) / mps);
  return s;
}

}  // namespace

// kernel ids for the live launch timer (impala_timer_*)
enum KernelId {
  K_CONV1_FWD = 0, K_CONV2_FWD, K_CONV12_FWD, K_CONV3_FWD, K_FC_FWD, K_HEADS_FWD, K_HEAD_STEP, K_FC_DGRAD,
  K_LN_BWD, K_CONV3_DGRAD, K_LNC3_BWD, K_FC_WGRAD, K_CONV3_WGRAD, K_CONV2_WGRAD, K_CONV12_BWD, K_REDUCE,
  K_SUMSQ, K_ADAM, K_REDUCE_ADAM, K_FC_BWD, K_WGRAD23, K_CONV123_FWD, K_LNC12_BWD, K_FWD_CHAIN,
  K_COUNT
};
const char* const kKernelNames[K_COUNT] = {
    "conv1_fwd", "conv2_fwd", "conv1_fwd_conv2_fwd", "conv3_fwd", "fc_fwd", "heads_fwd", "head_step", "fc_dgrad",
    "ln_bwd", "conv3_dgrad", "ln_bwd_conv3_dgrad", "fc_wgrad", "conv3_wgrad", "conv2_wgrad",
    "conv2_dgrad_conv1_wgrad", "reduce_grads", "sumsq", "adam", "reduce_grads_adam", "fc_wgrad_fc_dgrad",
    "conv3_wgrad_conv2_wgrad", "conv1_conv2_conv3_fwd", "ln_conv3_conv2_dgrad_conv1_wgrad",
    "conv123_fwd_fc_fwd"};

struct impala_learner {
  impala_config cfg;
  int device = 0;
  int N = 0;  // frames per step = B * T
  int A = 15;
  bool bf16 = false;
  net::Canon cn;
  net::Shadow sh;
  // caller-owned (bound)
  float *params = nullptr, *grads = nullptr, *exp_avg = nullptr, *exp_avg_sq = nullptr,
        *metrics = nullptr;
  float* metrics_host = nullptr;  // impala_set_metrics_host: the step's metrics also to host memory
  // impala_train_step_rows: while its launches are enqueued, the batch's frames are read from a
  // replay ring through obs_rows (conv12_fwd_s2d, head_step_kernel, lnc3_conv12_bwd)
  bool rows_on = false;
  ObsRows obs_rows{};
  // library-owned
  char* ws = nullptr;
  size_t ws_bytes = 0;
  void* shadow = nullptr;
  float* vecs = nullptr;
  void *act1, *act2, *act3, *y, *h, *dH, *dz, *dact3, *dact2;
  uint32_t* mask1;  // conv1 ReLU bit mask [N][225]
  float *lnstat, *zg, *heads, *dy;  // zg = gelu'(FC pre-activation)
  float *s_w1, *s_b1, *s_w2, *s_b2, *s_w3, *s_b3, *s_ln, *s_fc, *s_bfc, *s_h, *s_bh;
  float *loss_part, *sumsq_part, *adam_sc;
  int64_t* step;
  FusedSync fsync{};  // reduce_adam_kernel's granules, epoch counter and fault word
  bool fused_update = false;  // world_size 1: slab reduction + clip + Adam in one launch
  bool fc_merged = true;      // FC weight + input gradients in one launch (fc_bwd_kernel)
  bool wg23_merged = true;    // conv3 + conv2 weight gradients in one launch (wgrad23_kernel)
  bool c3_tail = true;        // bf16: conv3 + LayerNorm as the tail of the fused conv1/conv2 forward
  bool lc12 = true;           // LayerNorm/conv3 dgrad + conv2 dgrad/conv1 wgrad in one launch
  // the already-final slabs reduced inside the conv wgrad launch (opt-in IMPALA_EARLY_RED=1):
  // bitwise equal, but the merged launch grew by 5.5 us and reduce_grads shrank by only 2 us
  // (0.1214 / 0.1225 vs 0.1195 ms, reduction blocks last / first)
  bool early_red = false;
  // trunk forward + FC forward in one launch with per-producer flags (fwd_chain_kernel,
  // opt-in IMPALA_FWD_CHAIN=1): bitwise equal, but 30.6 us against 22.8 + 5.8 us -- the FC
  // tiles only start on CUs the conv workgroups free, all at the end (step 0.1202 vs 0.1180 ms)
  bool fwd_chain = false;
  unsigned* chain_flags = nullptr;  // [N] one word per conv workgroup
  int fc_splitk = 0;                // fp32 FC forward: 1 = K split over workgroups (in-launch
                                    // combine), 2 = K split over the waves of a workgroup
  int fcsk_pub = 1;                 // its publish form (ops.h fc_fwd_splitk_f32)
  float* fcsk_slab = nullptr;       // [tiles][4 splits][64 x 80] fp32 partials
  unsigned* fcsk_cnt = nullptr;     // [tiles] ticket counters (grow by 4 per launch)
  unsigned chain_epoch = 0;
  Split sp1, sp2, sp3, spfc, sph;
  int n_ln_wg = 0, ln_fpw = 2, n_loss_wg = 0, S_seg = 32, n_red_wg = 0, n_adam_wg = 256;
  // FC weight gradient in one split written straight into the canonical gradient (gemm_wg
  // direct mode, no slab); its workgroups' sums of squares follow the reduction's partials
  bool fc_direct = false;
  int n_fc_wg = 0;
  int n_norm_part = 0;  // clip-norm partials: n_red_wg (+ n_fc_wg)
  RedArgs red{};
  // side stream for the weight-gradient branches (fork/join with events, graph-capturable)
  hipStream_t side = nullptr;
  hipEvent_t ev_fork[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t ev_join = nullptr;
  bool use_side = true;
  // live launch timer: hipEvent pairs around every launch of one kernel id
  int n_cu = 256;
  bool lnc3_fused = true;      // LayerNorm backward + conv3 dgrad in one per-frame kernel
  bool fwd_fused = true;       // conv1 + conv2 forward in one per-frame kernel
  int red_mode = 0;           // slab reductions: 0 all at the end, 1 per branch, 2 side + conv1
  int c1_fpw = 1, c1_wg = 1;  // conv1 wgrad: frames per workgroup, workgroups (= splits)
  int c12f_fpw = 0;           // conv1+conv2 forward frames per workgroup (0: N / CUs)
  float* vt_dbg = nullptr;    // impala_set_debug_vtrace: the step's V-trace outputs
  // live launch timer (impala_timer_*): per kernel id, event pairs handed to
  // hipExtLaunchKernel, which stamps the kernel's own start / end (as rocprofv3 does)
  struct KTimer {
    hipEvent_t* ev = nullptr;
    int cap = 0, n = 0;
    bool armed = false;
  };
  KTimer timers[K_COUNT];
  int timers_armed = 0, timer_last = -1;
  // device step clock (impala_step_clock): stamps[clock_i] by the next step's first kernel
  unsigned long long* clock_buf = nullptr;
  int clock_n = 0, clock_i = 0;
  // hipGraph replay of whole steps: the launch sequence of a step is captured once per batch
  // address set (on a private capture stream) and replayed with one hipGraphLaunch
  struct GraphSlot {
    hipGraphExec_t exec = nullptr;
    int kind = -1;  // G_GRADS, G_UPDATE, G_STEP
    impala_batch key{};
    uint64_t used = 0;
  };
  static constexpr int kGraphSlots = 8;
  GraphSlot graphs[kGraphSlots];
  hipStream_t cap = nullptr;
  bool use_graph = false;
  uint64_t graph_tick = 0;
  // host staging ring (impala_stage*): device batch slots filled by H2D copies on `h2d`;
  // `ready` = the slot's copies are done, `done` = the steps that read it are done
  struct StageSlot {
    char* mem = nullptr;
    impala_batch dev{};
    hipEvent_t ready = nullptr, done = nullptr;
    // impala_stage_rows: the slot's page-locked host block (obs, then the four small fields,
    // impala_stage's layout), allocated at the first row-staging into the slot
    char* host_blk = nullptr;
  };
  static constexpr int kMaxStageSlots = 8;
  StageSlot ring[kMaxStageSlots];
  int n_slots = 0;
  // copy streams: IMPALA_H2D_STREAMS > 1 splits the obs block over several streams (stream 0
  // joins the others and signals `ready`); see impala_stage_init for the measured defaults
  static constexpr int kMaxH2D = 8;
  hipStream_t h2d_s[kMaxH2D] = {};
  hipEvent_t h2d_join[kMaxH2D] = {};
  int n_h2d = 0;
  int h2d_pull_wg = 0;        // > 0: copy everything with h2d_pull_kernel on that many workgroups
  int h2d_pull_threads = 256; // threads per pull workgroup (IMPALA_H2D_THREADS)
  bool h2d_small_pull = true; // SDMA obs: the four small fields in one 1-workgroup pull launch
  hipStream_t h2d = nullptr;  // = h2d_s[0]
  // impala_stage_rows: 0 = collate the rows into the slot's host block with the thread pool,
  // then impala_stage's copies; 1 = one SDMA copy per obs row straight from its memory
  // (IMPALA_STAGE_ROWS=collate|rows; IMPALA_STAGE_THREADS = pool threads).  (The batched copy
  // API, hipMemcpyBatchAsync, is newer than the HIP runtime torch loads.)
  int stage_rows_mode = 0;
  impala_host::HostPool* pool = nullptr;
  impala_host::Stager* stager = nullptr;  // impala_stage_rows_async's thread (lazily started)
  // native data-parallel step (impala_dp_*): the library's own RCCL communicator, so the
  // gradient all-reduces are enqueued with no host round trip and no c10d bookkeeping; the FC +
  // heads bucket is all-reduced on dp_stream while the per-frame backward runs
  ncclComm_t dp_comm = nullptr;
  hipStream_t dp_stream = nullptr;
  hipEvent_t dp_ev[3] = {nullptr, nullptr, nullptr};
  int dp_nranks = 0, dp_rank = -1;
};

namespace {
// persistent grid for gemm_tile: a few workgroups per CU, never more than the tile count
inline int persist_grid(const impala_learner* h, long tiles) {
  const long cap = (long)h->n_cu * 3;
  return (int)(tiles < cap ? tiles : cap);
}

// Every learner kernel is launched through klaunch: hipExtLaunchKernel, with the start / stop
// events of the live timer when kernel id `kid` is armed (the events then carry the kernel's
// own begin / end timestamps, so the timed duration excludes the launch and inter-kernel gap,
// as rocprofv3's kernel trace does).  Steps run without graph replay while a timer is armed.
template <typename... KArgs, typename... Args>
int klaunch(impala_learner* h, int kid, const char* name, void (*kernel)(KArgs...), dim3 grid,
            dim3 block, hipStream_t st, Args... args) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (kid >= 0) {
    auto& t = h->timers[kid];
    if (t.armed && t.n < t.cap) {
      e0 = t.ev[2 * t.n];
      e1 = t.ev[2 * t.n + 1];
      t.n++;
    }
  }
  hipExtLaunchKernelGGL(kernel, grid, block, 0, st, e0, e1, 0, args...);
  CK_LAUNCH(name);
  return 0;
}
}  // namespace

namespace {

// the device step clock's slot for the step being enqueued (nullptr: not armed / full)
unsigned long long* step_stamp(impala_learner* h) {
  return h->clock_buf && h->clock_i < h->clock_n ? h->clock_buf + h->clock_i++ : nullptr;
}

template <typename T>
int launch_forward(impala_learner* h, const uint8_t* obs, int n, hipStream_t st,
                   bool with_heads) {
  using namespace net;
  // K chunk of the LDS-staged tile GEMM: long chunks (few, each a full memory round trip) for
  // bf16; fp32 at most 64 (tools/var_specs/fp32a.py: 32 -> 64 cut fc_fwd 18.2 -> 14.0 us and
  // conv3_fwd 28.3 -> 27.0 us; 128 / 256 lost on conv3_fwd's LDS footprint)
#define BK(kb) (sizeof(T) == 4 ? ((kb) < 64 ? (kb) : 64) : (kb))
  const T* sw = reinterpret_cast<const T*>(h->shadow);
  const Shadow& sh = h->sh;
  const float* vv = h->vecs;
  bool conv3_done = false;
  if (h->fwd_fused) {  // conv1 + conv2 per frame (act1 consumed from LDS)
    const int fpw = h->c12f_fpw > 0 ? h->c12f_fpw : std::max(1, cdiv(n, h->n_cu));
    // at most c3t_fmax<T>() frames per workgroup (bf16 6, fp32 5): conv3 + ReLU + LayerNorm
    // run as the kernel's tail (one launch for the whole conv trunk)
    C3Tail<T> c3{};
    if (h->c3_tail && fpw <= c3t_fmax<T>()) {
      c3.w3 = sw + sh.w3; c3.b3 = vv + Vecs::b3; c3.gam = vv + Vecs::lng; c3.bet = vv + Vecs::lnb;
      c3.act3 = (T*)h->act3; c3.y = (T*)h->y; c3.stats = h->lnstat;
      conv3_done = true;
    }
    // training forward (no heads launch after it): the FC forward joins the launch, each FC
    // tile waiting on flags of the conv workgroups that produce its frames (not under graph
    // capture: the epoch argument changes every launch)
#if IMPALA_AB
    if (sizeof(T) == 2 && conv3_done && !with_heads && h->fwd_chain && !h->use_graph) {
      if (++h->chain_epoch == 0) h->chain_epoch = 1;
      c3.y_sc1 = 1;
      using CC = FwdChainCfg<T>;
      FcFwd<T> fop{n, sw + sh.wfc, vv + Vecs::bfc, (const T*)h->y, h->zg, (T*)h->h};
      const int n_conv = cdiv(n, fpw), n_fc = (HID / CC::FR) * cdiv(n, CC::FC);
      if constexpr (sizeof(T) == 2) {
        if (int r = klaunch(h, K_FWD_CHAIN, "conv123_fwd_fc_fwd", fwd_chain_kernel<T>,
                            dim3(n_conv + n_fc), dim3(512), st, obs, sw + sh.w1, vv + Vecs::b1,
                            sw + sh.w2, vv + Vecs::b2, (T*)h->act1, h->mask1, (T*)h->act2, n, fpw,
                            c3, n_conv, fop, h->chain_flags, h->chain_epoch, h->fsync.fault))
          return r;
      }
      return 0;
    }
#endif
    // the frames from the batch arrays, or (impala_train_step_rows) from a replay ring in place
    auto fwd = [&](const auto& rm) {
      using O = std::decay_t<decltype(rm)>;
      return klaunch(h, conv3_done ? K_CONV123_FWD : K_CONV12_FWD, "conv12_fwd", conv12_fwd_s2d<T, O>,
                     dim3(cdiv(n, fpw)), dim3(c12f_threads<T>()), st, obs, sw + sh.w1,
                     vv + Vecs::b1, sw + sh.w2, vv + Vecs::b2, (T*)h->act1, h->mask1,
                     (T*)h->act2, n, fpw, c3, with_heads ? nullptr : step_stamp(h), rm);
    };
    if (int r = h->rows_on && !with_heads ? fwd(h->obs_rows) : fwd(ObsDirect{})) return r;
  } else {
    if (!with_heads)  // the unfused forward (IMPALA_FWD_FUSED=0): the clock gets a stamp launch
      if (unsigned long long* ss = step_stamp(h))
        if (int r = klaunch(h, -1, "clock_stamp", clock_stamp_kernel, dim3(1), dim3(64), st, ss))
          return r;
    if (int r = klaunch(h, K_CONV1_FWD, "conv1_fwd", conv1_fwd_s2d<T>, dim3(min(n, h->n_cu * 4)),
                        dim3(256), st, obs, sw + sh.w1, vv + Vecs::b1, (T*)h->act1, h->mask1, n))
      return r;
    Conv2Fwd<T> op{n * P2, sw + sh.w2, vv + Vecs::b2, (const T*)h->act1, (T*)h->act2};
    if (int r = klaunch(h, K_CONV2_FWD, "conv2_fwd", gemm_tile<T, 64, 128, BK(64), 1, 4, Conv2Fwd<T>>,
                        dim3(persist_grid(h, cdiv((long)n * P2, 128))), dim3(256), st, op, 1))
      return r;
  }
  if (!conv3_done) {
    Conv3LnFwd<T> op{};
    op.C = n * P3; op.w = sw + sh.w3; op.b = vv + Vecs::b3; op.x = (const T*)h->act2;
    op.out = (T*)h->act3; op.gam = vv + Vecs::lng; op.bet = vv + Vecs::lnb; op.y = (T*)h->y;
    op.stats = h->lnstat;
    op.frames_per_tile = 64 / P3;
    if (int r = klaunch(h, K_CONV3_FWD, "conv3_fwd", gemm_tile<T, 64, 64, BK(96), 2, 2, Conv3LnFwd<T>>,
                        dim3(persist_grid(h, cdiv((long)n * P3, 64))), dim3(256), st, op, 1))
      return r;
  }
#if IMPALA_AB
  if (sizeof(T) == 4 && h->fc_splitk == 2) {
    FcFwd<float> op{n, (const float*)(sw + sh.wfc), vv + Vecs::bfc, (const float*)h->y, h->zg,
                    (float*)h->h};
    const int grid = (HID / fcwk::ROWS) * cdiv(n, fcwk::COLS);
    if (int r = klaunch(h, K_FC_FWD, "fc_fwd_wsplit", fc_fwd_wsplit_f32, dim3(grid), dim3(256), st, op))
      return r;
  } else if (sizeof(T) == 4 && h->fc_splitk == 1) {
    // fp32: 64 x 80 tiles, K split 4 ways, combined by each tile's last split (ops.h)
    FcFwd<float> op{n, (const float*)(sw + sh.wfc), vv + Vecs::bfc, (const float*)h->y, h->zg,
                    (float*)h->h};
    const int grid = (HID / fcsk::ROWS) * cdiv(n, fcsk::COLS) * fcsk::NS;
    auto kern = h->fcsk_pub == 0 ? fc_fwd_splitk_f32<0>
                : h->fcsk_pub == 2 ? fc_fwd_splitk_f32<2> : fc_fwd_splitk_f32<1>;
    if (int r = klaunch(h, K_FC_FWD, "fc_fwd_splitk", kern, dim3(grid), dim3(256), st, op,
                        h->fcsk_slab, h->fcsk_cnt))
      return r;
  } else
#endif
  {
    FcFwd<T> op{n, sw + sh.wfc, vv + Vecs::bfc, (const T*)h->y, h->zg, (T*)h->h};
    // 32 x 32 tiles: 320 workgroups (5.9 vs 6.7 us for 64 x 32, tools/var_specs/fcfwd.py);
    // fp32: two K chunks in registers ahead of the MFMAs (FCF_PF / FCF_KACC)
    constexpr int PF = sizeof(T) == 4 ? FCF_PF : 1, KA = sizeof(T) == 4 ? FCF_KACC : 1;
    constexpr bool KW = sizeof(T) == 4 && FCF_KW;
    constexpr int BR = KW ? FCF_BR : 32, BC = KW ? FCF_BC : 32;
    // KW on FCF_NW waves (8: two per SIMD, K chunk 128 = one k-step per wave per chunk)
    constexpr int NWF = KW ? FCF_NW : 4, FBK = KW && FCF_NW == 8 ? (sizeof(T) == 4 ? 128 : 256) : BK(256);
    if (int r = klaunch(h, K_FC_FWD, "fc_fwd", gemm_tile<T, BR, BC, FBK, 2, NWF / 2, FcFwd<T>, PF, KA, KW>,
                        dim3(persist_grid(h, (long)cdiv(n, BC) * (HID / BR))), dim3(64 * NWF), st, op,
                        HID / BR))
      return r;
  }
  if (with_heads) {  // inference; in training the fused head kernel computes the heads
    HeadsFwd<T> op{n, sw + sh.wh, vv + Vecs::bh, (const T*)h->h, h->heads};
    if (int r = klaunch(h, K_HEADS_FWD, "heads_fwd", gemm_rc<T, 1, 1, HeadsFwd<T>>,
                        dim3(cdiv(n, 64), 1), dim3(256), st, op))
      return r;
  }
  return 0;
}

// slab-reduction segment groups (indices into RedArgs::seg, in the order create() adds them)
enum { RS_CONV1 = 0, RS_CONV2 = 2, RS_CONV3 = 4, RS_LN = 6, RS_FC = 7, RS_END = 11 };

int reduce_segments(impala_learner* h, int s_lo, int s_hi, hipStream_t st, int fin) {
  const int n = h->red.wg_start[s_hi] - h->red.wg_start[s_lo];
  return klaunch(h, K_REDUCE, "reduce_grads", reduce_grads_kernel, dim3(n), dim3(256), st, h->red,
                 s_lo, fin);
}

// part: -1 = the whole backward; 0 = through the conv3 weight gradient, ending with the
// reduction of gradient bucket 1 (conv3 .. heads, canonical [cn.w3, total)); 1 = the rest
// (conv2 weight gradient, conv2 dgrad + conv1 wgrad, bucket 0 = conv1 + conv2, loss metrics).
// Data-parallel replicas all-reduce bucket 1 while part 1 runs.  Three-bucket split: 2 = heads
// step, FC weight gradient and FC dgrad, ending with the reduction of [cn.wfc, total) (FC +
// heads); 3 = LayerNorm backward + conv3 dgrad and the conv3 weight gradient, ending with
// [cn.w3, cn.wfc) (conv3 + LayerNorm); 4 = part 1.  Any split gives bit-identical gradients
// (each reduction workgroup owns a fixed sum-of-squares slot).
template <typename T>
int launch_backward(impala_learner* h, const impala_batch* b, hipStream_t st, int part = -1) {
  using namespace net;
  const int N = h->N, B = h->cfg.batch_size, Tl = h->cfg.rollout_length;
  const T* sw = reinterpret_cast<const T*>(h->shadow);
  const Shadow& sh = h->sh;
  // ---- dgrad chain on `st`; each weight-gradient branch forks onto the side stream as soon
  // as its inputs exist and joins before the slab reduction ----
  // gemm_wg: 32-row m-chunks, several 4-wave groups per workgroup on interleaved chunks (more
  // chunk loads in flight per CU); fp32 keeps one group for its LDS budget.  The bf16 conv
  // weight gradients run 2 groups (56 KB of LDS: two workgroups per CU) rather than 4 (112 KB:
  // one, so the merged launch's 508 workgroups ran in two rounds): 17.1 -> 14.0 us, step 0.1029
  // -> 0.1000 ms (tools/var_specs/bfg.py, profiles/r05bg).  The bf16 FC weight gradient keeps 2
  // (one group: 8.2 -> 8.9 us).
  constexpr int WG4 = sizeof(T) == 2 ? 2 : 1, WG2 = sizeof(T) == 2 ? 2 : 1;
  hipStream_t ss = h->use_side ? h->side : st;
  auto fork = [&](int i) -> int {
    if (!h->use_side) return 0;
    CK(hipEventRecord(h->ev_fork[i], st));
    CK(hipStreamWaitEvent(ss, h->ev_fork[i], 0));
    return 0;
  };
  // FC weight and input gradients in one launch (single stream, slab FC weight gradient)
  const bool fc_merged = h->fc_merged && !h->fc_direct && !h->use_side && h->red_mode != 1;
  // conv3 + conv2 weight gradients in one launch (whole backward only: the data-parallel parts
  // end a gradient bucket between them)
  const bool whole = part == -1 || part == 5 || part == 6;  // the backward after the FC bucket
  const bool wg23 = h->wg23_merged && whole && !h->use_side && h->red_mode == 0;
  // the two per-frame backward chains in one launch (whole backward, same frame runs)
  const bool lc12 = h->lc12 && h->lnc3_fused && h->ln_fpw == h->c1_fpw && whole &&
                    !h->use_side && h->red_mode == 0;
  // with the per-frame backward fused ahead of the merged conv weight gradients, every slab
  // but conv2 / conv3 is final when the latter start: reduce those inside that launch
  // (not for part 5: the fused reduce + Adam reduces every unit itself)
  const bool early = h->early_red && lc12 && wg23 && part != 5;
  if (part == 1 || part == 4) goto part1;
  if (part == 3 || part == 6) goto stage_b;
  // ---- fused head: heads fwd, log-softmax / V-trace / loss, dz, heads weight gradient ----
  {
    HeadArgs ha{};
    ha.h = h->h; ha.zg = h->zg; ha.wh = sw + sh.wh; ha.wht = sw + sh.wht;
    ha.bh = h->vecs + Vecs::bh;
    ha.act = b->actions; ha.rew = b->rewards; ha.disc = b->discounts; ha.mu = b->behaviour_logits;
    ha.B = B; ha.T = Tl; ha.A = h->A; ha.S = h->S_seg; ha.TPW = 64 / h->S_seg;
    ha.lam = h->cfg.vtrace_lambda; ha.crho = h->cfg.clip_rho_threshold;
    ha.cpg = h->cfg.clip_pg_rho_threshold; ha.ent_coef = h->cfg.entropy_coeff;
    ha.vt_mode = h->cfg.vtrace_grad_mode;
    ha.dz = h->dz; ha.partials = h->loss_part; ha.slab_h = h->s_h; ha.slab_bh = h->s_bh;
    ha.heads_out = h->heads;
    ha.vt_dbg = h->cfg.algo == IMPALA_ALGO_PPO ? nullptr : h->vt_dbg;
    // torch.clamp(ratio, 1 - clip, 1 + clip): the bounds are python floats cast to fp32
    ha.clip_lo = (float)(1.0 - (double)h->cfg.ppo_clip);
    ha.clip_hi = (float)(1.0 + (double)h->cfg.ppo_clip);
    const dim3 hg(h->n_loss_wg, head_split<T>());
    if (int r = h->cfg.algo == IMPALA_ALGO_PPO
                    ? klaunch(h, K_HEAD_STEP, "head_step", head_step_kernel<T, true>, hg, dim3(256), st, ha,
                              ObsDirect{})
                    : h->rows_on
                    ? klaunch(h, K_HEAD_STEP, "head_step", head_step_kernel<T, false, ObsRows>, hg, dim3(256),
                              st, ha, h->obs_rows)
                    : klaunch(h, K_HEAD_STEP, "head_step", head_step_kernel<T, false>, hg, dim3(256), st, ha,
                              ObsDirect{}))
      return r;
  }
  if (int r = fork(1)) return r;  // dz ready
  if (fc_merged) {
    FcWgrad<T> ow{};
    ow.M = N; ow.x = (const T*)h->dz; ow.y = (const T*)h->y;
    FcDgrad<T> od{N, sw + sh.wfc, (const T*)h->dz, h->dy};
    using C = FcBwdCfg<T, WG2>;
    const int gx = FLAT / C::WBC, gy = HID / 64, gz = h->spfc.S;
    const int n_rt = FLAT / C::DR, n_dt = n_rt * cdiv(N, C::DC);
    if (int r = klaunch(h, K_FC_BWD, "fc_wgrad_fc_dgrad", fc_bwd_kernel<T, WG2>,
                        dim3(gx * gy * gz + n_dt), dim3(256 * WG2), st, ow, h->s_fc, h->s_bfc,
                        h->spfc.mps, gx, gy, gz, od, n_rt))
      return r;
  } else if (h->fc_direct) {
    FcWgradDirect<T> op{};
    op.M = N; op.x = (const T*)h->dz; op.y = (const T*)h->y;
    op.grads = h->grads; op.wcanon = (long long)h->cn.wfc; op.sumsq = h->sumsq_part + h->n_red_wg;
    constexpr int G = sizeof(T) == 2 ? FCD_G : 1;
    if (int r = klaunch(h, K_FC_WGRAD, "fc_wgrad",
                        gemm_wg<T, FCD_BR, FCD_BC, FCD_WR, FCD_WC, 32, G, FcWgradDirect<T>, FCD_PD>,
                        dim3(FLAT / FCD_BC, HID / FCD_BR, 1), dim3(256 * G), ss, op, nullptr,
                        nullptr, N))
      return r;
  } else {
    FcWgrad<T> op{};
    op.M = N; op.x = (const T*)h->dz; op.y = (const T*)h->y;
    if (int r = klaunch(h, K_FC_WGRAD, "fc_wgrad", gemm_wg<T, 64, 256, 1, 4, 32, WG2, FcWgrad<T>>,
                        dim3(FLAT / 256, HID / 64, h->spfc.S), dim3(256 * WG2), ss, op, h->s_fc,
                        h->s_bfc, h->spfc.mps))
      return r;
  }
  {
    if (h->red_mode == 1)
      if (int r = reduce_segments(h, RS_FC, RS_END, ss, 0)) return r;  // fc + heads slabs
  }
  if (!fc_merged) {
    FcDgrad<T> op{N, sw + sh.wfc, (const T*)h->dz, h->dy};
    if (int r = klaunch(h, K_FC_DGRAD, "fc_dgrad", gemm_tile<T, 64, 64, BK(128), 2, 2, FcDgrad<T>>,
                        dim3(persist_grid(h, (long)cdiv(N, 64) * (FLAT / 64))), dim3(256), st, op,
                        FLAT / 64))
      return r;
  }
  if (part == 2) {  // bucket FC + heads complete
    if (h->use_side) {
      CK(hipEventRecord(h->ev_join, ss));
      CK(hipStreamWaitEvent(st, h->ev_join, 0));
    }
    return reduce_segments(h, RS_FC, RS_END, st, 0);
  }
stage_b:
  if (lc12) {
    auto bwd = [&](const auto& rm) {
      using O = std::decay_t<decltype(rm)>;
      return klaunch(h, K_LNC12_BWD, "ln_conv3_conv2_dgrad_conv1_wgrad", lnc3_conv12_bwd<T, O>,
                     dim3(h->n_ln_wg), dim3(lnc3_threads<T>()), st, (const float*)h->dy,
                     (const T*)h->act3, (const float*)h->lnstat,
                     (const float*)(h->vecs + Vecs::lng), sw + sh.w3, sw + sh.w3t,
                     (const T*)h->act2, (T*)h->dact3, (T*)h->dact2, h->s_ln, b->obs,
                     sw + sh.w2, sw + sh.w2t, (const uint32_t*)h->mask1, h->s_w1, h->s_b1, N,
                     h->ln_fpw, rm);
    };
    if (int r = h->rows_on ? bwd(h->obs_rows) : bwd(ObsDirect{})) return r;
  } else if (h->lnc3_fused) {  // LayerNorm backward + conv3 dgrad per frame
    if (int r = klaunch(h, K_LNC3_BWD, "ln_bwd_conv3_dgrad", lnc3_bwd<T>, dim3(h->n_ln_wg),
                        dim3(lnc3_threads<T>()), st, (const float*)h->dy, (const T*)h->act3,
                        (const float*)h->lnstat, (const float*)(h->vecs + Vecs::lng), sw + sh.w3,
                        sw + sh.w3t, (const T*)h->act2, (T*)h->dact3, (T*)h->dact2, h->s_ln, N,
                        h->ln_fpw))
      return r;
  } else {
    if (int r = klaunch(h, K_LN_BWD, "ln_bwd", ln_bwd_kernel<T>, dim3(h->n_ln_wg), dim3(256), st,
                        (const float*)h->dy, (const T*)h->act3, (const float*)h->lnstat,
                        (const float*)(h->vecs + Vecs::lng), (T*)h->dact3, h->s_ln, N, h->ln_fpw))
      return r;
  }
  if (int r = fork(2)) return r;  // dact3 ready
  if (wg23) {
    Conv3Wgrad<T> o3{};
    o3.M = N * P3; o3.x = (const T*)h->dact3; o3.in = (const T*)h->act2;
    Conv2Wgrad<T> o2{};
    o2.M = N * P2; o2.x = (const T*)h->dact2; o2.in = (const T*)h->act1;
    if (!h->lnc3_fused) {  // dact2 comes from the separate conv3 dgrad
      Conv3Dgrad<T> op{N * P2, sw + sh.w3, (const T*)h->dact3, (const T*)h->act2, (T*)h->dact2};
      if (int r = klaunch(h, K_CONV3_DGRAD, "conv3_dgrad", gemm_tile<T, 64, 128, BK(64), 1, 4, Conv3Dgrad<T>>,
                          dim3(persist_grid(h, cdiv((long)N * P2, 128))), dim3(256), st, op, 1))
        return r;
    }
    const int g3x = K3 / 64, g3z = h->sp3.S, g2x = K2 / Wg2Tile<T>::BC, g2z = h->sp2.S;
#if IMPALA_AB
    if (early) {
      // conv1 + b1 and LayerNorm (+ FC and heads unless part 2 reduced them) units ride along
      const int* ws = h->red.wg_start;
      const int u0 = ws[RS_CONV1], n0 = ws[RS_CONV2] - ws[RS_CONV1];
      const int u1 = ws[RS_LN], n1 = (part == 6 ? ws[RS_FC] : ws[RS_END]) - ws[RS_LN];
      if (int r = klaunch(h, K_WGRAD23, "conv3_wgrad_conv2_wgrad", wgrad23r_kernel<T, WG4>,
                          dim3(g3x * g3z + g2x * g2z + cdiv(n0 + n1, WG4)), dim3(256 * WG4), st,
                          o3, h->s_w3, h->s_b3, h->sp3.mps, g3x, g3z, o2, h->s_w2, h->s_b2,
                          h->sp2.mps, g2x, g2z, h->red, u0, n0, u1, n1))
        return r;
    } else
#endif
    if (int r = klaunch(h, K_WGRAD23, "conv3_wgrad_conv2_wgrad", wgrad23_kernel<T, WG4>,
                               dim3(g3x * g3z + g2x * g2z), dim3(256 * WG4), st, o3, h->s_w3,
                               h->s_b3, h->sp3.mps, g3x, g3z, o2, h->s_w2, h->s_b2, h->sp2.mps,
                               g2x, g2z)) {
      return r;
    }
    goto conv12b;
  }
  {
    Conv3Wgrad<T> op{};
    op.M = N * P3; op.x = (const T*)h->dact3; op.in = (const T*)h->act2;
    // 64 x 64 tiles (9 column tiles x ~28 splits): 4.1 MB of partial slabs instead of 9.4 MB
    // for 64 x 192 tiles x 64 splits, and 9.1 vs 9.8 us (profiles/r02b)
    if (int r = klaunch(h, K_CONV3_WGRAD, "conv3_wgrad", gemm_wg<T, 64, 64, 2, 2, 32, WG4, Conv3Wgrad<T>>,
                        dim3(K3 / 64, 1, h->sp3.S), dim3(256 * WG4), ss, op, h->s_w3, h->s_b3,
                        h->sp3.mps))
      return r;
    if (h->red_mode == 1)
      if (int r = reduce_segments(h, RS_CONV3, RS_FC, ss, 0)) return r;  // conv3 + LayerNorm
  }
  if (!h->lnc3_fused) {
    Conv3Dgrad<T> op{N * P2, sw + sh.w3, (const T*)h->dact3, (const T*)h->act2, (T*)h->dact2};
    if (int r = klaunch(h, K_CONV3_DGRAD, "conv3_dgrad", gemm_tile<T, 64, 128, BK(64), 1, 4, Conv3Dgrad<T>>,
                        dim3(persist_grid(h, cdiv((long)N * P2, 128))), dim3(256), st, op, 1))
      return r;
  }
  if (part == 0 || part == 3) {  // bucket 1 (or conv3 + LayerNorm) complete
    if (h->use_side) {
      CK(hipEventRecord(h->ev_join, ss));
      CK(hipStreamWaitEvent(st, h->ev_join, 0));
    }
    return reduce_segments(h, RS_CONV3, part == 0 ? RS_END : RS_FC, st, 0);
  }
part1:
  if (int r = fork(3)) return r;  // dact2 ready
  {
    Conv2Wgrad<T> op{};
    op.M = N * P2; op.x = (const T*)h->dact2; op.in = (const T*)h->act1;
    if (int r = klaunch(h, K_CONV2_WGRAD, "conv2_wgrad", gemm_wg<T, 64, 128, 1, 4, 32, WG4, Conv2Wgrad<T>>,
                        dim3(K2 / 128, 1, h->sp2.S), dim3(256 * WG4), ss, op, h->s_w2, h->s_b2,
                        h->sp2.mps))
      return r;
    if (h->red_mode == 1) {
      if (int r = reduce_segments(h, RS_CONV2, RS_CONV3, ss, 0)) return r;
    } else if (h->red_mode == 2 && part != 1 && part != 4 && part != 6) {
      // (parts 1 / 4 / 6: conv3 .. heads, or FC + heads, were reduced by an earlier part and
      // may be in an all-reduce right now; the final reduction below covers the rest)
      if (int r = reduce_segments(h, RS_CONV2, RS_END, ss, 0)) return r;
    }
  }
conv12b:
  // conv2 input gradient (ReLU-masked) + conv1 weight gradient, fused per frame
  if (!lc12)
    if (int r = klaunch(h, K_CONV12_BWD, "conv2_dgrad_conv1_wgrad", conv12_bwd_s2d<T>,
                        dim3(h->c1_wg), dim3(256 * c12_groups<T>()), st, b->obs, sw + sh.w2,
                        sw + sh.w2t, (const T*)h->dact2, (const uint32_t*)h->mask1, h->s_w1, h->s_b1, N,
                        h->c1_fpw))
      return r;
  // ---- last slab reduction (conv1) + loss metrics + step += 1; the other branches were
  // reduced on the side stream right after their weight gradients ----
  if (part == 6) {  // the conv + LayerNorm bucket [0, cn.wfc) + loss metrics + step
    if (h->use_side) {
      CK(hipEventRecord(h->ev_join, ss));
      CK(hipStreamWaitEvent(st, h->ev_join, 0));
    }
    return early ? reduce_segments(h, RS_CONV2, RS_LN, st, 1) : reduce_segments(h, RS_CONV1, RS_FC, st, 1);
  }
  if (part == 1 || part == 4) {
    if (h->use_side) {
      CK(hipEventRecord(h->ev_join, ss));
      CK(hipStreamWaitEvent(st, h->ev_join, 0));
    }
    return reduce_segments(h, RS_CONV1, RS_CONV3, st, 1);
  }
  if (h->red_mode == 0) {
    if (h->use_side) {  // join
      CK(hipEventRecord(h->ev_join, ss));
      CK(hipStreamWaitEvent(st, h->ev_join, 0));
    }
    if (part == 5) return 0;  // the fused update kernel reduces the slabs
    if (early) {  // conv1, LayerNorm, FC and heads were reduced beside the conv weight gradients
      if (int r = reduce_segments(h, RS_CONV2, RS_LN, st, 1)) return r;
    } else if (int r = reduce_segments(h, RS_CONV1, RS_END, st, 1)) {
      return r;
    }
  } else {
    if (int r = reduce_segments(h, RS_CONV1, RS_CONV2, st, 1)) return r;
    if (h->use_side) {  // join
      CK(hipEventRecord(h->ev_join, ss));
      CK(hipStreamWaitEvent(st, h->ev_join, 0));
    }
  }
  return 0;
}

template <typename T>
int launch_adam(impala_learner* h, hipStream_t st) {
  AdamArgs aa{};
  aa.params = h->params; aa.grads = h->grads; aa.m = h->exp_avg; aa.v = h->exp_avg_sq;
  aa.metrics = h->metrics; aa.sumsq_part = h->sumsq_part; aa.n_part = h->n_norm_part;
  aa.metrics_host = h->metrics_host;
  aa.step = h->step;
  aa.sc = h->adam_sc; aa.b1 = dec(h->cfg.adam_beta1); aa.b2 = dec(h->cfg.adam_beta2);
  aa.eps = h->cfg.adam_eps; aa.max_norm = h->cfg.max_grad_norm;
  aa.inv_world = 1.f / (float)h->cfg.world_size;
  aa.sp = ShadowPtrs{h->shadow, h->vecs, h->A};
  aa.cn = h->cn; aa.sh = h->sh;
  // HID blocks for the FC weight rows, then the other parameters (adam_kernel)
  const long rest = (long)h->cn.total - (long)(h->cn.bfc - h->cn.wfc);
  return klaunch(h, K_ADAM, "adam", adam_kernel<T>, dim3(net::HID + cdiv(rest, 256)),
                 dim3(256), st, aa);
}

#if IMPALA_AB
// slab reduction + clip + Adam in one launch (world_size 1; backward run with part 5)
template <typename T>
int launch_reduce_adam(impala_learner* h, hipStream_t st) {
  AdamArgs aa{};
  aa.params = h->params; aa.grads = h->grads; aa.m = h->exp_avg; aa.v = h->exp_avg_sq;
  aa.metrics = h->metrics; aa.sumsq_part = h->sumsq_part; aa.n_part = h->n_norm_part;
  aa.step = h->step;
  aa.sc = h->adam_sc; aa.b1 = dec(h->cfg.adam_beta1); aa.b2 = dec(h->cfg.adam_beta2);
  aa.eps = h->cfg.adam_eps; aa.max_norm = h->cfg.max_grad_norm;
  aa.inv_world = 1.f / (float)h->cfg.world_size;
  aa.sp = ShadowPtrs{h->shadow, h->vecs, h->A};
  aa.cn = h->cn; aa.sh = h->sh;
  return klaunch(h, K_REDUCE_ADAM, "reduce_grads_adam", reduce_adam_kernel<T>,
                 dim3(cdiv(h->n_red_wg, FU_MAX_UNITS)),
                 dim3(256), st, h->red, aa, h->fsync);
}
#endif  // IMPALA_AB

template <typename T>
int launch_pack(impala_learner* h, hipStream_t st) {
  pack_params_kernel<T><<<cdiv((long)h->cn.total, 256), 256, 0, st>>>(h->params, ShadowPtrs{h->shadow, h->vecs, h->A},
                                                     h->cn, h->sh);
  CK_LAUNCH("pack_params");
  return 0;
}

void drop_graphs(impala_learner* h) {
  for (auto& g : h->graphs) {
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    g = impala_learner::GraphSlot{};
  }
}

// The staging rings' copy streams, shared by every handle on a device that asks for the same
// number: a process's streams share GPU_MAX_HW_QUEUES (4) hardware queues, and each handle's own
// pair of copy streams took a share of them (a second handle's staging ran at 0.42 instead of
// 0.30 ms per step beside the first's, profiles/r06w).  Reference-counted; the last handle's
// release destroys them.
struct SharedH2D {
  int device = -1, n = 0, refs = 0;
  hipStream_t s[impala_learner::kMaxH2D] = {};
};
std::mutex g_h2d_mu;
SharedH2D g_h2d[16];

int acquire_h2d(impala_learner* h, int n) {
  std::lock_guard<std::mutex> lk(g_h2d_mu);
  SharedH2D* e = nullptr;
  for (auto& x : g_h2d)
    if (x.refs > 0 && x.device == h->device && x.n == n) e = &x;
  if (!e) {
    for (auto& x : g_h2d)
      if (x.refs == 0) {
        e = &x;
        break;
      }
    if (!e) return fail(IMPALA_E_STATE, "impala_stage_init: too many staging stream sets");
    e->device = h->device;
    e->n = 0;
    for (int i = 0; i < n; ++i) {
      if (hipStreamCreateWithFlags(&e->s[i], hipStreamNonBlocking) != hipSuccess) {
        for (int j = 0; j < i; ++j) (void)hipStreamDestroy(e->s[j]);
        return fail(IMPALA_E_STATE, "impala_stage_init: hipStreamCreate failed");
      }
    }
    e->n = n;
  }
  ++e->refs;
  for (int i = 0; i < n; ++i) h->h2d_s[i] = e->s[i];
  return 0;
}

void release_h2d(impala_learner* h) {
  if (!h->n_h2d) return;
  std::lock_guard<std::mutex> lk(g_h2d_mu);
  for (auto& x : g_h2d)
    if (x.refs > 0 && x.device == h->device && x.n == h->n_h2d && x.s[0] == h->h2d_s[0]) {
      if (--x.refs == 0) {
        for (int i = 0; i < x.n; ++i) (void)hipStreamDestroy(x.s[i]);
        x = SharedH2D{};
      }
      break;
    }
}

void free_ring(impala_learner* h) {
  if (h->stager) {  // no staging job may still be writing into the ring
    std::string m;
    (void)h->stager->wait(-1, m);
  }
  for (int i = 0; i < h->n_h2d; ++i) (void)hipStreamSynchronize(h->h2d_s[i]);
  for (auto& s : h->ring) {
    if (s.done) (void)hipEventSynchronize(s.done);
    if (s.ready) (void)hipEventDestroy(s.ready);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.mem) (void)hipFree(s.mem);
    if (s.host_blk) (void)hipHostFree(s.host_blk);
    s = impala_learner::StageSlot{};
  }
  h->n_slots = 0;
}

int check_bound(impala_learner* h, bool train = true) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (!h->params) return fail(IMPALA_E_STATE, "impala_bind_state() not called");
  if (train && (!h->grads || !h->exp_avg || !h->exp_avg_sq || !h->metrics))
    return fail(IMPALA_E_STATE, "training needs grads, exp_avg, exp_avg_sq and metrics bound");
  return 0;
}

int check_batch(const impala_batch* b, bool ppo = false) {
  if (!b || !b->obs || !b->actions || !b->rewards || (!ppo && !b->discounts) ||
      !b->behaviour_logits)
    return fail(IMPALA_E_INVALID, "null batch pointer");
  if (((uintptr_t)b->obs & 15) != 0) return fail(IMPALA_E_INVALID, "obs must be 16-byte aligned");
  return 0;
}

}  // namespace

extern "C" {

int impala_abi_version(void) { return IMPALA_ABI_VERSION; }
const char* impala_last_error(void) { return g_err.c_str(); }

int impala_config_default(impala_config* c) {
  if (!c) return fail(IMPALA_E_INVALID, "null cfg");
  c->batch_size = 8;
  c->rollout_length = 20;
  c->num_actions = 15;
  c->dtype = IMPALA_DTYPE_F32;
  c->lr = 1e-4f;
  c->adam_beta1 = 0.9f;
  c->adam_beta2 = 0.999f;
  c->adam_eps = 1e-5f;
  c->max_grad_norm = 0.5f;
  c->entropy_coeff = 0.01f;
  c->vtrace_lambda = 1.f;
  c->clip_rho_threshold = 1.f;
  c->clip_pg_rho_threshold = 1.f;
  c->world_size = 1;
  c->algo = IMPALA_ALGO_IMPALA;
  c->ppo_clip = 0.1f;
  c->vtrace_grad_mode = IMPALA_VTRACE_SG_ADVANTAGE;
  return 0;
}

size_t impala_param_count(int num_actions) { return net::canon(num_actions).total; }

int impala_create(const impala_config* cfg, int device, impala_learner** out) {
  using namespace net;
  if (!cfg || !out) return fail(IMPALA_E_INVALID, "null argument");
  *out = nullptr;
  if (cfg->batch_size < 1) return fail(IMPALA_E_INVALID, "batch_size must be >= 1");
  if (cfg->algo != IMPALA_ALGO_IMPALA && cfg->algo != IMPALA_ALGO_PPO)
    return fail(IMPALA_E_INVALID, "unknown algo");
  if (cfg->algo == IMPALA_ALGO_PPO && cfg->rollout_length != 1)
    return fail(IMPALA_E_UNSUPPORTED, "PPO handles take flat transitions: rollout_length must be 1");
  if (cfg->algo == IMPALA_ALGO_IMPALA && (cfg->rollout_length < 2 || cfg->rollout_length > 64))
    return fail(IMPALA_E_UNSUPPORTED, "rollout_length must be in [2, 64]");
  if (!(cfg->ppo_clip >= 0.f && cfg->ppo_clip < 1.f))
    return fail(IMPALA_E_INVALID, "ppo_clip must be in [0, 1)");
  if (cfg->num_actions < 1 || cfg->num_actions > MAX_A)
    return fail(IMPALA_E_UNSUPPORTED, "num_actions must be in [1, 15]");
  if (cfg->vtrace_grad_mode < IMPALA_VTRACE_SG_ADVANTAGE || cfg->vtrace_grad_mode > IMPALA_VTRACE_SG_NONE)
    return fail(IMPALA_E_INVALID, "unknown vtrace_grad_mode");
  if (cfg->dtype != IMPALA_DTYPE_F32 && cfg->dtype != IMPALA_DTYPE_BF16)
    return fail(IMPALA_E_INVALID, "unknown dtype");
  if (cfg->world_size < 1) return fail(IMPALA_E_INVALID, "world_size must be >= 1");
#if !IMPALA_AB
  // the measured-slower alternatives are compiled into A/B builds only (common.h IMPALA_AB)
  for (const char* v : {"IMPALA_FC_SPLITK", "IMPALA_FWD_CHAIN", "IMPALA_FUSED_UPDATE",
                        "IMPALA_EARLY_RED"}) {
    // the split-K FC forward is an fp32-only variant: bf16 handles ignore the switch, as the
    // A/B build does
    if (cfg->dtype != IMPALA_DTYPE_F32 && std::string(v) == "IMPALA_FC_SPLITK") continue;
    const char* e = std::getenv(v);
    if (e && e[0] && e[0] != '0')
      return fail(IMPALA_E_UNSUPPORTED, std::string(v) + " selects an A/B variant this library "
                                        "was built without (python -m impala_amd.build --ab)");
  }
#endif
  CK(hipSetDevice(device));
  impala_learner* h = new (std::nothrow) impala_learner();
  if (!h) return fail(IMPALA_E_INVALID, "out of host memory");
  h->cfg = *cfg;
  h->device = device;
  h->A = cfg->num_actions;
  h->bf16 = cfg->dtype == IMPALA_DTYPE_BF16;
  h->N = cfg->batch_size * cfg->rollout_length;
  {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cu > 0)
      h->n_cu = cu;
  }
  h->cn = canon(h->A);
  h->sh = shadow();
  const int N = h->N;
  const size_t es = h->bf16 ? 2 : 4;
  h->S_seg = next_pow2(cfg->rollout_length);
  h->n_loss_wg = cdiv(cfg->batch_size, 64 / h->S_seg);  // fused head: 64/S trajectories per WG
  if (const char* lf = std::getenv("IMPALA_LNC3_FUSED")) h->lnc3_fused = lf[0] != '0';
  if (h->lnc3_fused) {  // frames per workgroup of the fused kernel (one slab each)
    h->ln_fpw = std::max(1, cdiv(N, h->n_cu));
    h->n_ln_wg = cdiv(N, h->ln_fpw);
  } else {
    h->n_ln_wg = cdiv(N, 4 * h->ln_fpw);
  }

  // upper bound on the reduce workgroups (each segment: count/4 float4 columns, >= 16 per WG)
  h->n_red_wg = 11 + (OC1 * K1 + OC1 + OC2 * K2 + OC2 + OC3 * K3 + OC3 + 2 * FLAT + HID * FLAT +
                      HID + HEADS * HID + HEADS) / 4 / 16;
  h->sph.S = h->n_loss_wg;  // heads weight-gradient partials: one slab per head workgroup
  // FC weight-gradient splits: 96 workgroups for bf16; fp32 128 (8 splits: fc_bwd 20.3 us and
  // the reduction 7.55 against 20.7 / 7.75 for 256 workgroups, 27.8 us for 64;
  // tools/var_specs/{fc32b,spfc32}.py)
  int fc_wg = h->bf16 ? 96 : 128;
  if (const char* e = std::getenv("IMPALA_FC_WG")) fc_wg = std::max(16, std::atoi(e));
  h->spfc = plan_split(N, (FLAT / 256) * (HID / 64), fc_wg);
  // one-split FC weight gradient written straight into the canonical gradient (opt-in,
  // IMPALA_FC_DIRECT=1, up to 8192 frames): it drops the 6.3 MB FC slab and 256 reduction
  // workgroups, but the one-split GEMM is latency-bound on its per-CU load concurrency and the
  // step measured 0.1340-0.1368 ms in every tile shape against 0.1325-0.1330 ms for the split
  // slab (profiles/r02d/fc_direct_variants.txt)
  h->fc_direct = false;
  if (const char* e = std::getenv("IMPALA_FC_DIRECT")) h->fc_direct = N <= 8192 && e[0] == '1';
  h->n_fc_wg = (FLAT / FCD_BC) * (HID / FCD_BR);
  // the conv weight gradients' m splits: ~256 workgroups each (IMPALA_WG3_TARGET /
  // IMPALA_WG2_TARGET override the count for A/B runs; more splits, more slab bytes to reduce)
  int wg3 = 256, wg2 = 256;
  if (const char* e = std::getenv("IMPALA_WG3_TARGET")) wg3 = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("IMPALA_WG2_TARGET")) wg2 = std::max(1, std::atoi(e));
  h->sp3 = plan_split((long)N * P3, K3 / 64, wg3);
  h->sp2 = plan_split((long)N * P2, K2 / 128, wg2);
  h->c1_fpw = std::max(1, cdiv(N, h->n_cu));
  if (const char* e = std::getenv("IMPALA_C1_FPW")) h->c1_fpw = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("IMPALA_C12F_FPW")) h->c12f_fpw = std::max(0, std::atoi(e));
  h->c1_wg = cdiv(N, h->c1_fpw);
  h->sp1.S = h->c1_wg;  // slab splits of conv1 (one per workgroup)

  // ---- one workspace allocation, 256-byte aligned carve ----
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t o_shadow = take(h->sh.total * es);
  const size_t o_vecs = take(Vecs::total * 4);
  const size_t o_act1 = take((size_t)N * P1 * OC1 * es);
  const size_t o_act2 = take((size_t)N * P2 * OC2 * es);
  const size_t o_act3 = take((size_t)N * FLAT * es);
  const size_t o_y = take((size_t)N * YLD * es);
  const size_t o_h = take((size_t)N * HID * es);
  const size_t o_dH = take((size_t)N * HPAD * es);
  const size_t o_dz = take((size_t)N * HID * es);
  const size_t o_dact3 = take((size_t)N * FLAT * es);
  const size_t o_dact2 = take((size_t)N * P2 * OC2 * es);
  const size_t o_mask1 = take((size_t)N * P1 * 4);
  const size_t o_lnstat = take((size_t)N * 2 * 4);
  const size_t o_z = take((size_t)N * HID * 4);
  const size_t o_heads = take((size_t)N * HEADS * 4);
  const size_t o_dy = take((size_t)N * FLAT * 4);
  const size_t o_sw1 = take((size_t)h->sp1.S * OC1 * K1 * 4);
  const size_t o_sb1 = take((size_t)h->sp1.S * OC1 * 4);
  const size_t o_sw2 = take((size_t)h->sp2.S * OC2 * K2 * 4);
  const size_t o_sb2 = take((size_t)h->sp2.S * OC2 * 4);
  const size_t o_sw3 = take((size_t)h->sp3.S * OC3 * K3 * 4);
  const size_t o_sb3 = take((size_t)h->sp3.S * OC3 * 4);
  const size_t o_sln = take((size_t)h->n_ln_wg * 2 * FLAT * 4);
  const size_t o_sfc = take((size_t)h->spfc.S * HID * FLAT * 4);
  const size_t o_sbfc = take((size_t)h->spfc.S * HID * 4);
  const size_t o_sh = take((size_t)h->sph.S * HEADS * HID * 4);
  const size_t o_sbh = take((size_t)h->sph.S * HEADS * 4);
  const size_t o_lpart = take((size_t)h->n_loss_wg * 8 * 4);
  const size_t o_spart = take((size_t)(h->n_red_wg + 3) / 4 * 16);  // zero tail: float4 reads
  const size_t o_adsc = take(2 * 4);
  const size_t o_step = take(8);
  const size_t o_gran = take((size_t)h->n_red_wg * 8);  // fused update granules (upper bound)
  const size_t o_fsync = take(16);                       // epoch counter, fault word
  const size_t o_chain = take((size_t)N * 4);            // forward-chain producer flags
  if (const char* e = std::getenv("IMPALA_FC_SPLITK")) h->fc_splitk = es == 4 ? std::atoi(e) : 0;
  const size_t fcsk_tiles = h->fc_splitk == 1 ? (size_t)(HID / fcsk::ROWS) * cdiv(N, fcsk::COLS) : 0;
  const size_t o_fcsk = take(fcsk_tiles * fcsk::NS * fcsk::PART * 4);  // opt-in split-K partials
  const size_t o_fcskc = take(fcsk_tiles * 4);
  h->ws_bytes = off;
  hipError_t e = hipMalloc(&h->ws, off);
  if (e != hipSuccess) {
    delete h;
    return fail((int)e, std::string("hipMalloc workspace: ") + hipGetErrorString(e));
  }
  e = hipMemset(h->ws, 0, off);
  if (e != hipSuccess) {
    (void)hipFree(h->ws);
    delete h;
    return fail((int)e, std::string("hipMemset workspace: ") + hipGetErrorString(e));
  }
  char* w = h->ws;
  h->shadow = w + o_shadow;
  h->vecs = (float*)(w + o_vecs);
  h->act1 = w + o_act1; h->act2 = w + o_act2; h->act3 = w + o_act3; h->y = w + o_y;
  h->h = w + o_h; h->dH = w + o_dH; h->dz = w + o_dz; h->dact3 = w + o_dact3;
  h->dact2 = w + o_dact2; h->mask1 = (uint32_t*)(w + o_mask1);
  h->lnstat = (float*)(w + o_lnstat); h->zg = (float*)(w + o_z); h->heads = (float*)(w + o_heads);
  h->dy = (float*)(w + o_dy);
  h->s_w1 = (float*)(w + o_sw1); h->s_b1 = (float*)(w + o_sb1);
  h->s_w2 = (float*)(w + o_sw2); h->s_b2 = (float*)(w + o_sb2);
  h->s_w3 = (float*)(w + o_sw3); h->s_b3 = (float*)(w + o_sb3);
  h->s_ln = (float*)(w + o_sln); h->s_fc = (float*)(w + o_sfc); h->s_bfc = (float*)(w + o_sbfc);
  h->s_h = (float*)(w + o_sh); h->s_bh = (float*)(w + o_sbh);
  h->loss_part = (float*)(w + o_lpart); h->sumsq_part = (float*)(w + o_spart);
  h->adam_sc = (float*)(w + o_adsc);
  h->step = (int64_t*)(w + o_step);
  h->fsync.gran = (unsigned long long*)(w + o_gran);
  h->fsync.epoch_ctr = (unsigned*)(w + o_fsync);
  h->fsync.fault = (unsigned*)(w + o_fsync + 4);
  h->chain_flags = (unsigned*)(w + o_chain);
  h->fcsk_slab = (float*)(w + o_fcsk);
  h->fcsk_cnt = (unsigned*)(w + o_fcskc);
  if (const char* e = std::getenv("IMPALA_FCSK_PUB")) h->fcsk_pub = std::atoi(e);
  if (const char* rm = std::getenv("IMPALA_RED_MODE")) h->red_mode = std::atoi(rm);
  if (const char* ff = std::getenv("IMPALA_FWD_FUSED")) h->fwd_fused = ff[0] != '0';
  if (const char* e = std::getenv("IMPALA_FC_MERGED")) h->fc_merged = e[0] != '0';
  if (const char* e = std::getenv("IMPALA_WG23_MERGED")) h->wg23_merged = e[0] != '0';
  if (const char* e = std::getenv("IMPALA_C3_TAIL")) h->c3_tail = e[0] != '0';
  if (const char* e = std::getenv("IMPALA_LC12")) h->lc12 = e[0] != '0';
  if (const char* e = std::getenv("IMPALA_EARLY_RED")) h->early_red = e[0] == '1';
  if (const char* e = std::getenv("IMPALA_FWD_CHAIN")) h->fwd_chain = e[0] == '1';
  // hipGraph replay of whole steps (opt-in): it cuts the host enqueue cost of a step ~3x, but
  // on MI355X / ROCm 7 the replayed step ran slower on the device than direct launches
  // (174 vs 165 us), so direct launches are the default
  if (const char* g = std::getenv("IMPALA_GRAPH")) h->use_graph = g[0] == '1';
  // the capture stream exists only for graph replay: every stream a process creates takes a
  // share of its GPU_MAX_HW_QUEUES hardware queues (profiles/r06w)
  if (h->use_graph && hipStreamCreateWithFlags(&h->cap, hipStreamNonBlocking) != hipSuccess) {
    impala_destroy(h);
    return fail(IMPALA_E_STATE, "hipStreamCreate (capture stream) failed");
  }
  // The weight-gradient branches may run on a side stream (IMPALA_SIDE_STREAM=1).  Measured on
  // MI355X the kernels do not overlap usefully and the fork / join costs more than it hides
  // (DESIGN.md §7), so one stream is the default.
  const char* side = std::getenv("IMPALA_SIDE_STREAM");
  if (!side || side[0] != '1') {
    h->use_side = false;
  } else if (hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking) != hipSuccess) {
    h->use_side = false;
    h->side = nullptr;
  } else {
    for (int i = 0; i < 4; ++i)
      if (hipEventCreateWithFlags(&h->ev_fork[i], hipEventDisableTiming) != hipSuccess)
        h->use_side = false;
    if (hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess)
      h->use_side = false;
  }
  {
    RedArgs& ra = h->red;
    int ns = 0;
    // split loads per thread the split-group count aims for (IMPALA_RED_LPT): 16 -> 10.3 us,
    // 8 -> 10.7, 4 -> 11.2, 2 -> 11.6 (rocprof, B=64 T=20 bf16, profiles/r01k)
    int lpt = 16;
    if (const char* e = std::getenv("IMPALA_RED_LPT")) lpt = std::max(1, std::atoi(e));
    auto add = [&](const float* slab, int S, int count, int kind, long long canon) {
      int sg = 1;
      while (sg < 16 && sg * lpt < S) sg <<= 1;  // ~lpt+ loads per thread, <= 16 groups
      ra.seg[ns] = RedSeg{slab, S, count, kind, canon, sg};
      ra.wg_start[ns + 1] = ra.wg_start[ns] + cdiv(count / 4, 256 / sg);
      ++ns;
    };
    ra.wg_start[0] = 0;
    add(h->s_w1, h->sp1.S, OC1 * K1, RK_CONV1, (long long)h->cn.w1);
    add(h->s_b1, h->sp1.S, OC1, RK_ID, (long long)h->cn.b1);
    add(h->s_w2, h->sp2.S, OC2 * K2, RK_CONV2, (long long)h->cn.w2);
    add(h->s_b2, h->sp2.S, OC2, RK_ID, (long long)h->cn.b2);
    add(h->s_w3, h->sp3.S, OC3 * K3, RK_CONV3, (long long)h->cn.w3);
    add(h->s_b3, h->sp3.S, OC3, RK_ID, (long long)h->cn.b3);
    add(h->s_ln, h->n_ln_wg, 2 * FLAT, RK_LN, (long long)h->cn.lng);
    // (direct FC: empty segments, so the segment indices stay fixed)
    add(h->s_fc, h->spfc.S, h->fc_direct ? 0 : HID * FLAT, RK_FC, (long long)h->cn.wfc);
    add(h->s_bfc, h->spfc.S, h->fc_direct ? 0 : HID, RK_ID, (long long)h->cn.bfc);
    add(h->s_h, h->sph.S, HEADS * HID, RK_HEADS_W, 0);
    add(h->s_bh, h->sph.S, HEADS, RK_HEADS_B, 0);
    h->n_red_wg = ra.wg_start[ns];
    h->n_norm_part = h->n_red_wg + (h->fc_direct ? h->n_fc_wg : 0);
    if (ns != RS_END) {
      impala_destroy(h);
      return fail(IMPALA_E_STATE, "reduce segment table out of sync");
    }
    ra.nseg = ns;
    ra.cn = h->cn;
    ra.sumsq_part = h->sumsq_part;
    ra.loss_part = h->loss_part;
    ra.n_loss_part = h->n_loss_wg;
    ra.B = cfg->batch_size;
    ra.T = cfg->rollout_length;
    ra.A = h->A;
    ra.ent_coef = cfg->entropy_coeff;
    ra.algo = cfg->algo;
    ra.step = h->step;
    ra.lr = dec(cfg->lr); ra.b1 = dec(cfg->adam_beta1); ra.b2 = dec(cfg->adam_beta2);
    ra.adam_sc = h->adam_sc;
  }
  // fused slab reduction + clip + Adam (reduce_adam_kernel, IMPALA_FUSED_UPDATE=1): world_size
  // 1, the single-stream end-of-backward reduction, and every reduction unit on a resident
  // workgroup.  Opt-in: bitwise equal to reduce_grads + adam but slower on MI355X (20 vs
  // 10.3 + 6.0 us at B=64 T=20 bf16; the all-gather of the norm partials alone takes ~4.5 us
  // after the last unit publishes, more than the kernel boundary it removes: DESIGN.md §7)
  h->fsync.n_units = h->n_red_wg;
  h->fsync.n_part = h->n_norm_part;
  h->fsync.part = h->sumsq_part;
  if (const char* e = std::getenv("IMPALA_FUSED_UPDATE")) h->fused_update = e[0] == '1';
  // (it updates exactly the elements it reduces, so the direct FC gradient is off with it)
  if (h->fused_update && h->fc_direct) h->fused_update = false;
  if (cfg->world_size != 1 || h->red_mode != 0 || h->n_red_wg > 3 * FU_MAX_UNITS * h->n_cu)
    h->fused_update = false;
  *out = h;
  return 0;
}

extern "C++" {
namespace {
// RCCL entry points, resolved by dlopen on first use: the library has no link-time RCCL
// dependency, and inside a torch process the loader hands back torch's already-loaded copy
// (same SONAME), so the handle's communicator and torch's live in one RCCL instance.
struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommCount) comm_count = nullptr;
  std::string err;
};
const RcclApi& rccl() {
  static const RcclApi api = [] {
    RcclApi a;
    void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!lib) lib = dlopen("librccl.so.1", RTLD_NOW);
    if (!lib) lib = dlopen("librccl.so", RTLD_NOW);
    if (!lib) {
      const char* e = dlerror();
      a.err = std::string("dlopen librccl: ") + (e ? e : "not found");
      return a;
    }
    a.get_unique_id = (decltype(a.get_unique_id))dlsym(lib, "ncclGetUniqueId");
    a.comm_init_rank = (decltype(a.comm_init_rank))dlsym(lib, "ncclCommInitRank");
    a.all_reduce = (decltype(a.all_reduce))dlsym(lib, "ncclAllReduce");
    a.comm_destroy = (decltype(a.comm_destroy))dlsym(lib, "ncclCommDestroy");
    a.error_string = (decltype(a.error_string))dlsym(lib, "ncclGetErrorString");
    a.comm_count = (decltype(a.comm_count))dlsym(lib, "ncclCommCount");
    if (!a.get_unique_id || !a.comm_init_rank || !a.all_reduce || !a.comm_destroy ||
        !a.error_string || !a.comm_count)
      a.err = "librccl lacks an expected entry point";
    return a;
  }();
  return api;
}
int rccl_fail(const char* what, ncclResult_t r) {
  return fail(IMPALA_E_RCCL, std::string(what) + ": " + rccl().error_string(r));
}
void dp_release(impala_learner* h) {
  if (h->dp_comm) (void)rccl().comm_destroy(h->dp_comm);
  h->dp_comm = nullptr;
  if (h->dp_stream) (void)hipStreamDestroy(h->dp_stream);
  h->dp_stream = nullptr;
  for (auto& e : h->dp_ev)
    if (e) { (void)hipEventDestroy(e); e = nullptr; }
  h->dp_nranks = 0;
  h->dp_rank = -1;
}
}  // namespace
}  // extern "C++"

int impala_destroy(impala_learner* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();  // replays may still be in flight on the caller's streams
  drop_graphs(h);
  free_ring(h);
  release_h2d(h);  // (the shared copy streams; the join events are the handle's)
  for (int i = 0; i < h->n_h2d; ++i)
    if (h->h2d_join[i]) (void)hipEventDestroy(h->h2d_join[i]);
  for (auto& t : h->timers) {
    for (int i = 0; i < 2 * t.cap; ++i) (void)hipEventDestroy(t.ev[i]);
    delete[] t.ev;
  }
  if (h->cap) (void)hipStreamDestroy(h->cap);
  for (int i = 0; i < 4; ++i)
    if (h->ev_fork[i]) (void)hipEventDestroy(h->ev_fork[i]);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->side) {
    (void)hipStreamSynchronize(h->side);
    (void)hipStreamDestroy(h->side);
  }
  dp_release(h);
  delete h->stager;  // (free_ring above already waited for its jobs)
  delete h->pool;
  if (h->ws) (void)hipFree(h->ws);
  delete h;
  return 0;
}

int impala_bind_state(impala_learner* h, float* params, float* grads, float* exp_avg,
                      float* exp_avg_sq, float* metrics, void* stream) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (!params) return fail(IMPALA_E_INVALID, "null params pointer");
  h->params = params; h->grads = grads; h->exp_avg = exp_avg; h->exp_avg_sq = exp_avg_sq;
  h->metrics = metrics;
  drop_graphs(h);  // captured launches hold the previous state pointers
  h->red.grads = grads;
  h->red.metrics = metrics;
  return impala_refresh_weights(h, stream);
}

int impala_set_metrics(impala_learner* h, float* metrics) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (!metrics) return fail(IMPALA_E_INVALID, "null metrics pointer");
  if (h->metrics != metrics) {
    h->metrics = metrics;
    h->red.metrics = metrics;
    if (h->use_graph) drop_graphs(h);  // captured launches hold the previous pointer
  }
  return 0;
}

int impala_set_metrics_host(impala_learner* h, float* host) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (host) {
    if (h->fused_update)  // the A/B fused reduce + Adam launch does not write it
      return fail(IMPALA_E_UNSUPPORTED, "impala_set_metrics_host: not with IMPALA_FUSED_UPDATE");
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, host) != hipSuccess || at.type != hipMemoryTypeHost) {
      (void)hipGetLastError();
      return fail(IMPALA_E_INVALID, "impala_set_metrics_host: not page-locked host memory");
    }
    if (((uintptr_t)host & 3) != 0) return fail(IMPALA_E_INVALID, "impala_set_metrics_host: misaligned");
  }
  if (h->metrics_host != host) {
    h->metrics_host = host;
    if (h->use_graph) drop_graphs(h);  // captured launches hold the previous pointer
  }
  return 0;
}

int impala_set_debug_vtrace(impala_learner* h, float* out) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (h->vt_dbg != out) drop_graphs(h);  // captured launches hold the previous pointer
  h->vt_dbg = out;
  return 0;
}

int impala_refresh_weights(impala_learner* h, void* stream) {
  if (int r = check_bound(h, false)) return r;
  CK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  return h->bf16 ? launch_pack<__bf16>(h, st) : launch_pack<float>(h, st);
}

int impala_set_step(impala_learner* h, int64_t step, void* stream) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (step < 0) return fail(IMPALA_E_INVALID, "negative step");
  CK(hipSetDevice(h->device));
  static thread_local int64_t host_step;
  host_step = step;
  CK(hipMemcpyAsync(h->step, &host_step, 8, hipMemcpyHostToDevice, (hipStream_t)stream));
  CK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

int impala_forward(impala_learner* h, const uint8_t* obs, int n, float* logits, float* values,
                   void* stream) {
  if (int r = check_bound(h, false)) return r;
  if (!obs || !logits || !values) return fail(IMPALA_E_INVALID, "null pointer");
  if (n < 1 || n > h->N) return fail(IMPALA_E_INVALID, "n must be in [1, B*T]");
  if (((uintptr_t)obs & 15) != 0) return fail(IMPALA_E_INVALID, "obs must be 16-byte aligned");
  CK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  int r = h->bf16 ? launch_forward<__bf16>(h, obs, n, st, true)
                  : launch_forward<float>(h, obs, n, st, true);
  if (r) return r;
  split_heads_kernel<<<cdiv((long)n * net::HEADS, 256), 256, 0, st>>>(h->heads, n, h->A, logits,
                                                                       values);
  CK_LAUNCH("split_heads");
  return 0;
}

int impala_act(impala_learner* h, const uint8_t* obs, int n, const uint8_t* deterministic,
               int deterministic_all, uint64_t seed, uint64_t counter, int64_t* actions,
               float* logits, float* values, void* stream) {
  if (int r = check_bound(h, false)) return r;
  if (!obs || !actions || !logits || !values) return fail(IMPALA_E_INVALID, "null pointer");
  if (n < 1 || n > h->N) return fail(IMPALA_E_INVALID, "n must be in [1, B*T]");
  if (((uintptr_t)obs & 15) != 0) return fail(IMPALA_E_INVALID, "obs must be 16-byte aligned");
  CK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  int r = h->bf16 ? launch_forward<__bf16>(h, obs, n, st, true)
                  : launch_forward<float>(h, obs, n, st, true);
  if (r) return r;
  act_heads_kernel<<<cdiv(n, 256), 256, 0, st>>>(h->heads, n, h->A, deterministic,
                                                 deterministic_all, seed, counter, actions,
                                                 logits, values);
  CK_LAUNCH("act_heads");
  return 0;
}

extern "C++" {
namespace {
int enqueue_grads(impala_learner* h, const impala_batch* b, hipStream_t st, int part = -1) {
  if (part == -1 || part == 0 || part == 2 || part == 5) {  // (parts 1, 3, 4, 6 continue a backward)
    int r = h->bf16 ? launch_forward<__bf16>(h, b->obs, h->N, st, false)
                    : launch_forward<float>(h, b->obs, h->N, st, false);
    if (r) return r;
  }
  return h->bf16 ? launch_backward<__bf16>(h, b, st, part) : launch_backward<float>(h, b, st, part);
}

int enqueue_update(impala_learner* h, hipStream_t st) {
  if (h->cfg.world_size > 1) {
    if (int r = klaunch(h, K_SUMSQ, "sumsq", sumsq_kernel, dim3(h->n_norm_part), dim3(256), st,
                        (const float*)h->grads, (size_t)h->cn.total, h->sumsq_part))
      return r;
  }
  return h->bf16 ? launch_adam<__bf16>(h, st) : launch_adam<float>(h, st);
}

bool same_batch(const impala_batch& a, const impala_batch& b) {
  return a.obs == b.obs && a.actions == b.actions && a.rewards == b.rewards &&
         a.discounts == b.discounts && a.behaviour_logits == b.behaviour_logits;
}

// Run `body` (which enqueues a step's launches on the stream it is given) through the graph
// cache: replay a graph captured for the same kind and batch addresses, or capture one on the
// private capture stream, instantiate it and launch it on `st`.  With the live timer armed
// (its events must be recorded per launch) or IMPALA_GRAPH=0 the launches go straight to `st`.
template <class Body>
int run_graphed(impala_learner* h, int kind, const impala_batch* b, hipStream_t st, Body&& body) {
  if (!h->use_graph || h->timers_armed > 0 || h->clock_buf) return body(st);
  const impala_batch key = b ? *b : impala_batch{};
  for (auto& g : h->graphs)
    if (g.exec && g.kind == kind && same_batch(g.key, key)) {
      g.used = ++h->graph_tick;
      CK(hipGraphLaunch(g.exec, st));
      return 0;
    }
  CK(hipStreamBeginCapture(h->cap, hipStreamCaptureModeThreadLocal));
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
  *slot = impala_learner::GraphSlot{exec, kind, key, ++h->graph_tick};
  CK(hipGraphLaunch(exec, st));
  return 0;
}
enum { G_GRADS = 0, G_UPDATE = 1, G_STEP = 2, G_GRADS0 = 3 };  // G_GRADS0 + part (0..4)
}  // namespace
}  // extern "C++"

int impala_compute_grads(impala_learner* h, const impala_batch* b, void* stream) {
  if (int r = check_bound(h)) return r;
  if (int r = check_batch(b, h->cfg.algo == IMPALA_ALGO_PPO)) return r;
  CK(hipSetDevice(h->device));
  return run_graphed(h, G_GRADS, b, (hipStream_t)stream,
                     [&](hipStream_t s) { return enqueue_grads(h, b, s); });
}

int impala_compute_grads_part(impala_learner* h, const impala_batch* b, int part, void* stream) {
  if (part < 0 || part > 6 || part == 5) return fail(IMPALA_E_INVALID, "part must be 0..4 or 6");
  if (int r = check_bound(h)) return r;
  if (int r = check_batch(b, h->cfg.algo == IMPALA_ALGO_PPO)) return r;
  CK(hipSetDevice(h->device));
  return run_graphed(h, G_GRADS0 + part, b, (hipStream_t)stream,
                     [&](hipStream_t s) { return enqueue_grads(h, b, s, part); });
}

size_t impala_grad_bucket_offset(const impala_learner* h) { return h ? h->cn.w3 : 0; }
size_t impala_grad_bucket_offset_fc(const impala_learner* h) { return h ? h->cn.wfc : 0; }

int impala_apply_update(impala_learner* h, void* stream) {
  if (int r = check_bound(h)) return r;
  CK(hipSetDevice(h->device));
  return run_graphed(h, G_UPDATE, nullptr, (hipStream_t)stream,
                     [&](hipStream_t s) { return enqueue_update(h, s); });
}

int impala_dp_unique_id(void* out) {
  if (!out) return fail(IMPALA_E_INVALID, "null unique-id buffer");
  const RcclApi& api = rccl();
  if (!api.err.empty()) return fail(IMPALA_E_RCCL, api.err);
  ncclUniqueId id;
  if (ncclResult_t r = api.get_unique_id(&id)) return rccl_fail("ncclGetUniqueId", r);
  static_assert(sizeof(ncclUniqueId) == IMPALA_DP_ID_BYTES, "unique id size");
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

int impala_dp_init(impala_learner* h, const void* unique_id, int nranks, int rank) {
  if (!h || !unique_id) return fail(IMPALA_E_INVALID, "null argument");
  if (nranks != h->cfg.world_size || rank < 0 || rank >= nranks)
    return fail(IMPALA_E_INVALID, "nranks must equal the handle's world_size and 0 <= rank < nranks");
  const RcclApi& api = rccl();
  if (!api.err.empty()) return fail(IMPALA_E_RCCL, api.err);
  CK(hipSetDevice(h->device));
  dp_release(h);
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  // collective over the nranks processes (each blocks until all have joined)
  if (ncclResult_t r = api.comm_init_rank(&h->dp_comm, nranks, id, rank)) {
    h->dp_comm = nullptr;
    return rccl_fail("ncclCommInitRank", r);
  }
  // the rest cannot leave a half-initialised handle: any failure releases the communicator
  // (impala_dp_train_step then reports that impala_dp_init has not run)
  hipError_t e = hipStreamCreateWithFlags(&h->dp_stream, hipStreamNonBlocking);
  for (auto& ev : h->dp_ev)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    dp_release(h);
    return fail((int)e, std::string("impala_dp_init: ") + hipGetErrorString(e));
  }
  int count = 0;
  if (ncclResult_t r = api.comm_count(h->dp_comm, &count)) {
    dp_release(h);
    return rccl_fail("ncclCommCount", r);
  }
  if (count != nranks) {
    dp_release(h);
    return fail(IMPALA_E_RCCL, "ncclCommCount disagrees with nranks");
  }
  h->dp_nranks = count;
  h->dp_rank = rank;
  return 0;
}

int impala_dp_nranks(const impala_learner* h, int* nranks) {
  if (!h || !nranks) return fail(IMPALA_E_INVALID, "null argument");
  *nranks = 0;
  if (!h->dp_comm) return 0;
  const RcclApi& api = rccl();
  if (!api.err.empty()) return fail(IMPALA_E_RCCL, api.err);
  if (ncclResult_t r = api.comm_count(h->dp_comm, nranks)) return rccl_fail("ncclCommCount", r);
  return 0;
}

int impala_dp_train_step(impala_learner* h, const impala_batch* b, int buckets, void* stream) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (!h->dp_comm || !h->dp_stream || !h->dp_ev[2])
    return fail(IMPALA_E_STATE, "impala_dp_init has not run on this handle");
  if (buckets != 1 && buckets != 2) return fail(IMPALA_E_INVALID, "buckets must be 1 or 2");
  if (int r = check_bound(h)) return r;
  if (int r = check_batch(b, h->cfg.algo == IMPALA_ALGO_PPO)) return r;
  CK(hipSetDevice(h->device));
  const hipStream_t st = (hipStream_t)stream;
  const RcclApi& api = rccl();
  float* g = h->grads;
  const size_t n = (size_t)h->cn.total, off_fc = (size_t)h->cn.wfc;
  if (buckets == 1) {  // the whole backward, one all-reduce on the compute stream, the update
    if (int r = enqueue_grads(h, b, st)) return r;
    if (ncclResult_t r = api.all_reduce(g, g, n, ncclFloat32, ncclSum, h->dp_comm, st))
      return rccl_fail("ncclAllReduce", r);
    return enqueue_update(h, st);
  }
  // two buckets: part 2 (forward, heads step, FC gradients) leaves grads[off_fc ..] final; its
  // all-reduce runs on dp_stream while part 6 (the per-frame backward, the conv weight
  // gradients) runs on `st`; then grads[.. off_fc] follow on dp_stream and `st` waits for both
  if (int r = enqueue_grads(h, b, st, 2)) return r;
  CK(hipEventRecord(h->dp_ev[0], st));
  CK(hipStreamWaitEvent(h->dp_stream, h->dp_ev[0], 0));
  if (ncclResult_t r = api.all_reduce(g + off_fc, g + off_fc, n - off_fc, ncclFloat32, ncclSum,
                                      h->dp_comm, h->dp_stream))
    return rccl_fail("ncclAllReduce (FC + heads bucket)", r);
  if (int r = enqueue_grads(h, b, st, 6)) return r;
  CK(hipEventRecord(h->dp_ev[1], st));
  CK(hipStreamWaitEvent(h->dp_stream, h->dp_ev[1], 0));
  if (ncclResult_t r = api.all_reduce(g, g, off_fc, ncclFloat32, ncclSum, h->dp_comm, h->dp_stream))
    return rccl_fail("ncclAllReduce (conv + LayerNorm bucket)", r);
  CK(hipEventRecord(h->dp_ev[2], h->dp_stream));
  CK(hipStreamWaitEvent(st, h->dp_ev[2], 0));
  return enqueue_update(h, st);
}

int impala_ppo_train_step(impala_learner* h, const impala_ppo_batch* pb, void* stream) {
  if (!h || !pb) return fail(IMPALA_E_INVALID, "null argument");
  if (h->cfg.algo != IMPALA_ALGO_PPO) return fail(IMPALA_E_STATE, "not a PPO handle");
  const impala_batch b{pb->obs, pb->actions, pb->targets, nullptr, pb->behaviour_logits};
  return impala_train_step(h, &b, stream);
}

int impala_train_step(impala_learner* h, const impala_batch* b, void* stream) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (h->cfg.world_size != 1)
    return fail(IMPALA_E_STATE, "world_size > 1: use compute_grads + all-reduce + apply_update");
  if (int r = check_bound(h)) return r;
  if (int r = check_batch(b, h->cfg.algo == IMPALA_ALGO_PPO)) return r;
  CK(hipSetDevice(h->device));
  return run_graphed(h, G_STEP, b, (hipStream_t)stream, [&](hipStream_t s) {
#if IMPALA_AB
    if (h->fused_update) {
      if (int r = enqueue_grads(h, b, s, 5)) return r;
      return h->bf16 ? launch_reduce_adam<__bf16>(h, s) : launch_reduce_adam<float>(h, s);
    }
#endif
    if (int r = enqueue_grads(h, b, s)) return r;
    return enqueue_update(h, s);
  });
}

int impala_train_step_rows(impala_learner* h, const impala_batch* ring, const int64_t* rows, int n,
                           int64_t capacity, void* stream) {
  if (!h || !ring || !rows) return fail(IMPALA_E_INVALID, "null argument");
  if (h->cfg.world_size != 1 || h->cfg.algo != IMPALA_ALGO_IMPALA)
    return fail(IMPALA_E_UNSUPPORTED, "impala_train_step_rows: IMPALA handles of world_size 1");
  // only the default launches read the batch through the row map: the fused forward
  // (conv12_fwd_s2d), the fused head and the fused per-frame backward (lnc3_conv12_bwd)
  const bool default_path = h->fwd_fused && h->lc12 && h->lnc3_fused && h->ln_fpw == h->c1_fpw &&
                            !h->use_side && h->red_mode == 0 && !h->fused_update && !h->fwd_chain;
  if (!default_path)
    return fail(IMPALA_E_UNSUPPORTED, "impala_train_step_rows: not on the default kernel path");
  if (n != h->cfg.batch_size || n > kObsRowsMax)
    return fail(IMPALA_E_INVALID, "impala_train_step_rows: n must equal batch_size (at most 256)");
  if (capacity < 1 || capacity > INT32_MAX / h->cfg.rollout_length)
    return fail(IMPALA_E_INVALID, "impala_train_step_rows: bad capacity");
  for (int i = 0; i < n; ++i)
    if (rows[i] < 0 || rows[i] >= capacity)
      return fail(IMPALA_E_INVALID, "impala_train_step_rows: row index out of range");
  if (int r = check_bound(h)) return r;
  if (int r = check_batch(ring)) return r;
  CK(hipSetDevice(h->device));
  h->obs_rows.T = h->cfg.rollout_length;
  for (int i = 0; i < n; ++i) h->obs_rows.rows[i] = (int)rows[i];
  h->rows_on = true;
  // direct launches: the rows change every step, a captured graph would hold the first ones
  int r = enqueue_grads(h, ring, (hipStream_t)stream);
  if (r == 0) r = enqueue_update(h, (hipStream_t)stream);
  h->rows_on = false;
  return r;
}

namespace {
int gather_launch(const void* const* src, void* const* dst, const size_t* row_bytes, int nfields,
                  const int64_t* idx, const int64_t* host_idx, int n, void* stream) {
  if (nfields < 1 || nfields > 8 || n < 0 || !src || !dst || !row_bytes ||
      (n > 0 && !idx && !host_idx))
    return fail(IMPALA_E_INVALID, "bad gather arguments");
  if (n == 0) return 0;
  GatherArgs ga{};
  int units = 0;
  for (int f = 0; f < nfields; ++f) {
    if (!src[f] || !dst[f] || row_bytes[f] % 4 != 0 || row_bytes[f] == 0)
      return fail(IMPALA_E_INVALID, "gather: null field or row size not a positive multiple of 4");
    ga.src[f] = (const char*)src[f];
    ga.dst[f] = (char*)dst[f];
    ga.row_bytes[f] = (long long)row_bytes[f];
    ga.pieces[f] = (int)((row_bytes[f] + GATHER_PIECE - 1) / GATHER_PIECE);
    ga.unit0[f] = units;
    units += ga.pieces[f] * n;
  }
  ga.unit0[nfields] = units;
  ga.nfields = nfields;
  ga.idx = idx;
  ga.n = n;
  if (!idx)
    for (int i = 0; i < n; ++i) ga.hidx[i] = (int)host_idx[i];
  gather_rows_kernel<<<dim3(units), 256, 0, (hipStream_t)stream>>>(ga);
  CK_LAUNCH("gather_rows");
  return 0;
}
}  // namespace

int impala_gather_rows(const void* const* src, void* const* dst, const size_t* row_bytes,
                       int nfields, const int64_t* idx, int n, void* stream) {
  if (n > 0 && !idx) return fail(IMPALA_E_INVALID, "bad gather arguments");
  return gather_launch(src, dst, row_bytes, nfields, idx, nullptr, n, stream);
}

int impala_gather_rows_hidx(const void* const* src, void* const* dst, const size_t* row_bytes,
                            int nfields, const int64_t* host_idx, int n, void* stream) {
  if (n > 0 && !host_idx) return fail(IMPALA_E_INVALID, "bad gather arguments");
  for (int i = 0; i < n; ++i)
    if (host_idx[i] < 0 || host_idx[i] > INT32_MAX)
      return fail(IMPALA_E_INVALID, "gather: host index out of range");
  // GATHER_HIDX rows per launch, their indices in the launch's arguments
  for (int i0 = 0; i0 < n; i0 += GATHER_HIDX) {
    const int m = std::min(GATHER_HIDX, n - i0);
    void* d[8];
    for (int f = 0; f < nfields && f < 8; ++f)
      d[f] = dst && dst[f] ? (char*)dst[f] + (size_t)i0 * row_bytes[f] : nullptr;
    if (int r = gather_launch(src, dst ? d : nullptr, row_bytes, nfields, nullptr, host_idx + i0, m,
                              stream))
      return r;
  }
  return 0;
}

// Prime the copy path at init: the learner's staging loop (ImpalaLearner._stage_host) for
// IMPALA_STAGE_PRIME rounds (default 24, 0 = off) in each of two shapes on a page-locked scratch batch, with a
// 250 us spin kernel on a private stream standing in for each step.  An H2D hipMemcpyAsync is
// given an SDMA engine by the runtime at issue time (hsa_amd_memory_get_preferred_copy_engine /
// copy_engine_status, then hsa_amd_memory_async_copy_on_engine), and the first copy given an
// engine creates that engine's queue inside the call: a 6-9 ms host stall before the copy is
// submitted (HIP + HSA API traces, profiles/r05d; hsa_queue_create alone takes 6-6.5 ms here).
// Which engines a loop gets depends on what is in flight and waiting when it issues (copies
// queued behind the previous step's events), so rounds of copies with nothing to wait for did
// not reach them (r05c, r05e); in the driver's 20-step host-staged pass one such stall landed
// in the timed steps (0.67 ms per step against a 0.30 ms median, profiles/r05a).
int prime_copy_path(impala_learner* h) {
  int rounds = 24;
  if (const char* e = std::getenv("IMPALA_STAGE_PRIME")) rounds = std::max(0, std::atoi(e));
  if (rounds == 0 || h->n_slots < 2) return 0;
  const size_t N = (size_t)h->N;
  const size_t sz[5] = {N * 3 * 64 * 64, N * 8, N * 4, N * 4, N * (size_t)h->A * 4};
  size_t total = 0;
  for (size_t b : sz) total += (b + 255) & ~(size_t)255;
  char* scratch = nullptr;
  CK(hipHostMalloc((void**)&scratch, total, hipHostMallocDefault));
  std::memset(scratch, 0, total);
  impala_batch hb{};
  {
    size_t o = 0;
    const void* p[5];
    for (int f = 0; f < 5; ++f) {
      p[f] = scratch + o;
      o += (sz[f] + 255) & ~(size_t)255;
    }
    hb = impala_batch{(const uint8_t*)p[0], (const int64_t*)p[1], (const float*)p[2],
                      (const float*)p[3], (const float*)p[4]};
  }
  hipStream_t cs = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
  int r = e == hipSuccess ? impala_stage(h, &hb, 0) : (int)e;
  for (int k = 0; k < rounds && r == 0 && e == hipSuccess; ++k) {
    const int s = k & 1;
    e = hipEventSynchronize(h->ring[1 - s].ready);             // stage_wait(1 - s)
    if (e == hipSuccess) r = impala_stage(h, &hb, 1 - s);      // stage(1 - s)
    if (r == 0 && e == hipSuccess) e = hipStreamWaitEvent(cs, h->ring[s].ready, 0);  // slot_batch(s)
    if (r == 0 && e == hipSuccess) {
      stage_prime_spin_kernel<<<1, 64, 0, cs>>>(25000);      // the "step" (250 us)
      e = hipGetLastError();
    }
    if (r == 0 && e == hipSuccess) e = hipEventRecord(h->ring[s].done, cs);  // slot_release(s)
  }
  // ... then the same rounds over every slot with the host running ahead, as a loop that reads
  // its metrics only every k steps does (DistributedAgent sync_every > 1): the host waits only
  // for a slot's previous copy (the collate's wait before it rewrites the slot's host block), so
  // every copy is queued behind the event of a step still two slots back.  Without this phase
  // that loop met one 7 ms queue-creation stall in its first dozen steps (profiles/r06y).
  for (int k = 0; k < rounds && r == 0 && e == hipSuccess; ++k) {
    const int s = k % h->n_slots;
    e = hipEventSynchronize(h->ring[s].ready);
    if (e == hipSuccess) r = impala_stage(h, &hb, s);
    if (r == 0 && e == hipSuccess) e = hipStreamWaitEvent(cs, h->ring[s].ready, 0);
    if (r == 0 && e == hipSuccess) {
      stage_prime_spin_kernel<<<1, 64, 0, cs>>>(25000);
      e = hipGetLastError();
    }
    if (r == 0 && e == hipSuccess) e = hipEventRecord(h->ring[s].done, cs);
  }
  if (cs) {
    const hipError_t es = hipStreamSynchronize(cs);
    if (e == hipSuccess) e = es;
  }
  for (int i = 0; i < h->n_h2d; ++i) {
    const hipError_t es = hipStreamSynchronize(h->h2d_s[i]);
    if (e == hipSuccess) e = es;
  }
  // leave the ring as stage_init's allocation loop does: both events recorded (complete) on
  // h2d, none referring to work of the private stream about to be destroyed
  for (int i = 0; i < h->n_slots && e == hipSuccess; ++i) {
    e = hipEventRecord(h->ring[i].ready, h->h2d);
    if (e == hipSuccess) e = hipEventRecord(h->ring[i].done, h->h2d);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(h->h2d);
  if (cs) (void)hipStreamDestroy(cs);
  (void)hipHostFree(scratch);
  if (r) return r;
  if (e != hipSuccess)
    return fail((int)e, std::string("impala_stage_init (copy-path priming): ") + hipGetErrorString(e));
  return 0;
}

int impala_stage_init(impala_learner* h, int nslots) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (nslots < 1 || nslots > impala_learner::kMaxStageSlots)
    return fail(IMPALA_E_INVALID, "nslots must be in [1, 8]");
  CK(hipSetDevice(h->device));
  free_ring(h);
  if (!h->n_h2d) {
    // Default: hipMemcpyAsync (SDMA) of obs split over 2 streams, the four small fields in one
    // small pull launch.  Beside the fp32 step (profiles/r04hs: H2D bandwidth A/B) SDMA on
    // 1 / 2 / 4 streams kept 41-43 / 46.4 / 43.9 GB/s, while the pull kernel (8 x 256 threads,
    // 45-48 GB/s alone and the round-1 default) fell to 36 GB/s and slowed the trunk forward it
    // shares CUs with from 63 to 190-210 us (rocprofv3 kernel trace, r04hs).
    // IMPALA_H2D_KERNEL=<workgroups> copies everything with the pull kernel instead.
    // Data-parallel handles (world_size > 1) never use the pull kernel unless asked: whether
    // every device of a node maps a rank's page-locked buffers is not something this library
    // checks.
    h->h2d_pull_wg = 0;
    if (const char* e = std::getenv("IMPALA_H2D_KERNEL")) h->h2d_pull_wg = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("IMPALA_H2D_THREADS"))
      h->h2d_pull_threads = std::max(64, std::min(1024, std::atoi(e) / 64 * 64));
    h->h2d_small_pull = h->cfg.world_size == 1;
    if (const char* e = std::getenv("IMPALA_H2D_SMALL_PULL")) h->h2d_small_pull = e[0] == '1';
    if (const char* e = std::getenv("IMPALA_STAGE_ROWS"))
      h->stage_rows_mode = std::strcmp(e, "rows") == 0 ? 1 : 0;
    int n = h->h2d_pull_wg > 0 ? 1 : 2;
    if (const char* e = std::getenv("IMPALA_H2D_STREAMS")) n = std::atoi(e);
    n = std::max(1, std::min(n, (int)impala_learner::kMaxH2D));
    if (int r = acquire_h2d(h, n)) return r;
    h->n_h2d = n;
    for (int i = 0; i < n; ++i) CK(hipEventCreateWithFlags(&h->h2d_join[i], hipEventDisableTiming));
    h->h2d = h->h2d_s[0];
  }
  const size_t N = (size_t)h->N;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t o_obs = take(N * 3 * 64 * 64), o_act = take(N * 8), o_rew = take(N * 4),
               o_disc = take(N * 4), o_mu = take(N * (size_t)h->A * 4);
  for (int i = 0; i < nslots; ++i) {
    auto& s = h->ring[i];
    hipError_t e = hipMalloc(&s.mem, off);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    // both events start recorded (complete), so the first stage / slot_batch never waits
    if (e == hipSuccess) e = hipEventRecord(s.ready, h->h2d);
    if (e == hipSuccess) e = hipEventRecord(s.done, h->h2d);
    if (e != hipSuccess) {
      free_ring(h);
      return fail((int)e, std::string("impala_stage_init: ") + hipGetErrorString(e));
    }
    s.dev = impala_batch{(const uint8_t*)(s.mem + o_obs), (const int64_t*)(s.mem + o_act),
                         (const float*)(s.mem + o_rew), (const float*)(s.mem + o_disc),
                         (const float*)(s.mem + o_mu)};
  }
  h->n_slots = nslots;
  if (h->h2d_pull_wg == 0) {
    if (int r = prime_copy_path(h)) {
      free_ring(h);
      return r;
    }
  }
  return 0;
}

namespace {
// Where the staging threads run (IMPALA_STAGE_PIN): "gpu" (default) the CPUs of the NUMA node
// the device's PCIe link hangs off, so the page-locked blocks they first touch and fill sit
// next to the DMA engines that read them; "caller" the calling thread's node; "0" anywhere.
std::vector<int> stage_cpus(const impala_learner* h) {
  const char* pin = std::getenv("IMPALA_STAGE_PIN");
  if (pin && pin[0] == '0') return {};
  if (pin && std::strcmp(pin, "caller") == 0) return impala_host::local_node_cpus();
  char bus[64] = {};
  int node = -1;
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), h->device) == hipSuccess) {
    for (char* c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
    const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    if (FILE* f = std::fopen(path.c_str(), "r")) {
      if (std::fscanf(f, "%d", &node) != 1) node = -1;
      std::fclose(f);
    }
  } else {
    (void)hipGetLastError();
  }
  return impala_host::local_node_cpus(node);  // (node -1: the caller's)
}

// the staging jobs of `slot` (every slot when < 0) queued by impala_stage_rows_async have run;
// a failed one's status is returned here
int wait_staged(impala_learner* h, int slot) {
  if (!h->stager) return 0;
  std::string m;
  if (int r = h->stager->wait(slot, m)) return fail(r, "impala_stage_rows_async: " + m);
  return 0;
}
}  // namespace

namespace {
int stage_now(impala_learner* h, const impala_batch* b, int slot);
}  // namespace

int impala_stage(impala_learner* h, const impala_batch* b, int slot) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (slot < 0 || slot >= h->n_slots)
    return fail(IMPALA_E_INVALID, "slot out of range (impala_stage_init not called?)");
  if (int r = wait_staged(h, -1)) return r;  // one staging at a time per handle
  return stage_now(h, b, slot);
}

namespace {
// impala_stage's copies (also run by the staging thread's jobs, which must not wait on
// themselves)
int stage_now(impala_learner* h, const impala_batch* b, int slot) {
  const bool ppo = h->cfg.algo == IMPALA_ALGO_PPO;
  if (!b || !b->obs || !b->actions || !b->rewards || (!ppo && !b->discounts) ||
      !b->behaviour_logits)
    return fail(IMPALA_E_INVALID, "null batch pointer");
  CK(hipSetDevice(h->device));
  auto& s = h->ring[slot];
  const size_t N = (size_t)h->N;
  const int ns = h->n_h2d;
  for (int i = 0; i < ns; ++i)  // the steps that read the slot have run
    CK(hipStreamWaitEvent(h->h2d_s[i], s.done, 0));
  // the pull kernel reads page-locked, device-mapped host fields (hipHostGetDevicePointer);
  // anything else takes hipMemcpyAsync
  const void* hsrc[5] = {b->obs, b->actions, b->rewards, b->discounts, b->behaviour_logits};
  const void* msrc[5] = {};
  bool mapped = h->h2d_pull_wg > 0 || h->h2d_small_pull;
  for (int f = 0; f < 5 && mapped; ++f) {
    if (!hsrc[f]) continue;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, const_cast<void*>(hsrc[f]), 0) != hipSuccess || !dp ||
        (((uintptr_t)dp) & 15) != 0) {
      (void)hipGetLastError();
      mapped = false;
    }
    msrc[f] = dp;
  }
  void* dst[5] = {(void*)s.dev.obs, (void*)s.dev.actions, (void*)s.dev.rewards,
                  (void*)s.dev.discounts, (void*)s.dev.behaviour_logits};
  const size_t bytes[5] = {N * 3 * 64 * 64, N * 8, N * 4, N * 4, N * (size_t)h->A * 4};
  auto pull = [&](int f_lo, int wgs, int threads) -> int {
    PullArgs pa{};
    for (int f = f_lo; f < 5; ++f) {
      if (!msrc[f]) continue;
      pa.src[pa.nf] = (const char*)msrc[f];
      pa.dst[pa.nf] = (char*)dst[f];
      pa.bytes[pa.nf] = (long long)bytes[f];
      ++pa.nf;
    }
    h2d_pull_kernel<<<wgs, threads, 0, h->h2d>>>(pa);
    CK_LAUNCH("h2d_pull");
    return 0;
  };
  if (mapped && h->h2d_pull_wg > 0) {
    if (int r = pull(0, h->h2d_pull_wg, h->h2d_pull_threads)) return r;
  } else {
    // the small fields first on stream 0 (one pull launch, or four copies), then obs in ns
    // contiguous chunks, one per copy stream
    if (mapped && h->h2d_small_pull) {
      // 8 workgroups, one per XCD: ~100 KB at PCIe latency (one workgroup took 37-42 us,
      // delaying the obs chunk behind it on the stream; rocprofv3 trace, r04hs3)
      if (int r = pull(1, 8, 256)) return r;
    } else {
      CK(hipMemcpyAsync(dst[1], b->actions, bytes[1], hipMemcpyDefault, h->h2d));
      CK(hipMemcpyAsync(dst[2], b->rewards, bytes[2], hipMemcpyDefault, h->h2d));
      if (b->discounts) CK(hipMemcpyAsync(dst[3], b->discounts, bytes[3], hipMemcpyDefault, h->h2d));
      CK(hipMemcpyAsync(dst[4], b->behaviour_logits, bytes[4], hipMemcpyDefault, h->h2d));
    }
    const size_t ob = bytes[0], chunk = (ob / ns + 4095) & ~(size_t)4095;
    for (int i = 0; i < ns; ++i) {
      const size_t o0 = std::min(ob, (size_t)i * chunk), o1 = std::min(ob, o0 + chunk);
      if (o1 > o0)
        CK(hipMemcpyAsync((char*)s.dev.obs + o0, b->obs + o0, o1 - o0, hipMemcpyDefault, h->h2d_s[i]));
    }
  }
  for (int i = 1; i < ns; ++i) {
    CK(hipEventRecord(h->h2d_join[i], h->h2d_s[i]));
    CK(hipStreamWaitEvent(h->h2d, h->h2d_join[i], 0));
  }
  CK(hipEventRecord(s.ready, h->h2d));
  return 0;
}
}  // namespace

// Row staging (impala_stage_rows): the batch is B trajectories scattered in host memory (the
// replay's rows), not one collated host batch.  Default (collate): the host's thread pool
// copies the rows into the slot's page-locked block -- obs, then the four small fields, in
// impala_stage's layout -- and impala_stage's copies follow (obs over the SDMA streams, the
// small fields in one pull launch).  One thread's memcpy moves the 15.7 MB of a C2 batch in
// ~1 ms, over three times the PCIe copy it feeds; the pool's threads share it.  The rows modes
// instead copy each obs row by SDMA straight from its own memory (runs of adjacent rows merged)
// and collate only the small fields.
namespace {
int check_rows(impala_learner* h, const impala_rows* rows, int n, int slot) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (slot < 0 || slot >= h->n_slots)
    return fail(IMPALA_E_INVALID, "slot out of range (impala_stage_init not called?)");
  const bool ppo = h->cfg.algo == IMPALA_ALGO_PPO;
  if (!rows || n != h->cfg.batch_size)
    return fail(IMPALA_E_INVALID, "impala_stage_rows: n must equal the handle's batch_size");
  if (!rows->obs || !rows->actions || !rows->rewards || (!ppo && !rows->discounts) ||
      !rows->behaviour_logits)
    return fail(IMPALA_E_INVALID, "impala_stage_rows: null row array");
  for (int b = 0; b < n; ++b)
    if (!rows->obs[b] || !rows->actions[b] || !rows->rewards[b] ||
        (!ppo && !rows->discounts[b]) || !rows->behaviour_logits[b])
      return fail(IMPALA_E_INVALID, "impala_stage_rows: null row pointer");
  return 0;
}
int stage_rows_now(impala_learner* h, const impala_rows* rows, int n, int slot);
}  // namespace

int impala_stage_rows(impala_learner* h, const impala_rows* rows, int n, int slot) {
  if (int r = check_rows(h, rows, n, slot)) return r;
  if (int r = wait_staged(h, -1)) return r;  // one staging at a time per handle
  return stage_rows_now(h, rows, n, slot);
}

int impala_stage_rows_async(impala_learner* h, const impala_rows* rows, int n, int slot) {
  if (int r = check_rows(h, rows, n, slot)) return r;
  if (int r = wait_staged(h, slot)) return r;  // the slot's previous job
  if (!h->stager) {
    h->stager = new (std::nothrow) impala_host::Stager(stage_cpus(h));
    if (!h->stager) return fail(IMPALA_E_STATE, "impala_stage_rows_async: staging thread");
  }
  // the job owns copies of the five pointer arrays; the rows themselves stay the caller's
  auto p = std::make_shared<std::vector<const void*>>();
  p->reserve(5 * (size_t)n);
  const void* const* f[5] = {rows->obs, rows->actions, rows->rewards, rows->discounts,
                             rows->behaviour_logits};
  for (int k = 0; k < 5; ++k)
    for (int b = 0; b < n; ++b) p->push_back(f[k] ? f[k][b] : nullptr);
  h->stager->submit(slot, [h, p, n, slot](std::string& msg) {
    const void* const* d = p->data();
    const impala_rows r{d, d + n, d + 2 * n, d[3 * n] ? d + 3 * n : nullptr, d + 4 * n};
    const int st = stage_rows_now(h, &r, n, slot);
    if (st) msg = impala_last_error();
    return st;
  });
  return 0;
}

namespace {
int stage_rows_now(impala_learner* h, const impala_rows* rows, int n, int slot) {
  const bool ppo = h->cfg.algo == IMPALA_ALGO_PPO;
  CK(hipSetDevice(h->device));
  auto& s = h->ring[slot];
  const size_t T = (size_t)h->cfg.rollout_length, N = (size_t)h->N, A = (size_t)h->A;
  const size_t rb[5] = {T * 3 * 64 * 64, T * 8, T * 4, T * 4, T * A * 4};
  // host block layout: obs | actions | rewards | discounts | behaviour logits (256-B aligned)
  size_t off[6];
  off[0] = 0;
  for (int f = 0; f < 5; ++f) off[f + 1] = off[f] + ((N * rb[f] / T + 255) & ~(size_t)255);
  if (!s.host_blk) {
    void* p = nullptr;
    // IMPALA_STAGE_HOSTMEM=1: mapped + portable (the round-6 first form); default flags
    // otherwise (as torch's page-locked tensors, which impala_stage copies from)
    const char* hm = std::getenv("IMPALA_STAGE_HOSTMEM");
    const unsigned flags = hm && hm[0] == '1' ? (hipHostMallocMapped | hipHostMallocPortable)
                                              : hipHostMallocDefault;
    CK(hipHostMalloc(&p, off[5], flags));
    s.host_blk = (char*)p;
  }
  // the slot's previous copies (out of its host block too) have finished before it is rewritten
  CK(hipEventSynchronize(s.ready));
  const void* const* src[5] = {rows->obs, rows->actions, rows->rewards, rows->discounts,
                               rows->behaviour_logits};
  char* hb = s.host_blk;
  const bool collate = h->stage_rows_mode == 0;
  // host copies: obs rows in 64 KB pieces (collate mode), each small field as one task
  constexpr size_t kPiece = 65536;
  const int per_row = collate ? (int)((rb[0] + kPiece - 1) / kPiece) : 0;
  const int n_obs_tasks = per_row * n;
  auto task = [&](int i) {
    if (i < n_obs_tasks) {
      const int b = i / per_row;
      const size_t o = (size_t)(i - b * per_row) * kPiece, len = std::min(kPiece, rb[0] - o);
      impala_host::copy_stream(hb + (size_t)b * rb[0] + o, (const char*)src[0][b] + o, len);
      return;
    }
    const int f = 1 + (i - n_obs_tasks);
    if (f == 3 && ppo) return;
    for (int b = 0; b < n; ++b) std::memcpy(hb + off[f] + (size_t)b * rb[f], src[f][b], rb[f]);
  };
  const int ntasks = n_obs_tasks + 4;
  if (collate && !h->pool) {
    int nt = 7;
    if (const char* e = std::getenv("IMPALA_STAGE_THREADS")) nt = std::max(0, std::atoi(e) - 1);
    h->pool = new (std::nothrow) impala_host::HostPool(nt, stage_cpus(h));
    if (!h->pool) return fail(IMPALA_E_STATE, "impala_stage_rows: thread pool");
  }
  if (h->pool && collate) {
    h->pool->run(ntasks, task);
  } else {
    for (int i = 0; i < ntasks; ++i) task(i);
  }
  if (collate) {
    const impala_batch hbat{(const uint8_t*)(hb + off[0]), (const int64_t*)(hb + off[1]),
                            (const float*)(hb + off[2]),
                            ppo ? nullptr : (const float*)(hb + off[3]), (const float*)(hb + off[4])};
    return stage_now(h, &hbat, slot);
  }
  const int ns = h->n_h2d;
  for (int i = 0; i < ns; ++i)  // the steps that read the slot have run
    CK(hipStreamWaitEvent(h->h2d_s[i], s.done, 0));
  void* dst[5] = {(void*)s.dev.obs, (void*)s.dev.actions, (void*)s.dev.rewards,
                  (void*)s.dev.discounts, (void*)s.dev.behaviour_logits};
  void* hb_dev = nullptr;
  if (hipHostGetDevicePointer(&hb_dev, hb, 0) != hipSuccess || (((uintptr_t)hb_dev) & 15) != 0) {
    (void)hipGetLastError();
    hb_dev = nullptr;
  }
  if (hb_dev && (h->h2d_small_pull || h->h2d_pull_wg > 0)) {
    PullArgs pa{};
    for (int f = 1; f < 5; ++f) {
      if (f == 3 && ppo) continue;
      pa.src[pa.nf] = (const char*)hb_dev + off[f];
      pa.dst[pa.nf] = (char*)dst[f];
      pa.bytes[pa.nf] = (long long)(N * rb[f] / T);
      ++pa.nf;
    }
    h2d_pull_kernel<<<8, 256, 0, h->h2d>>>(pa);
    CK_LAUNCH("h2d_pull");
  } else {
    for (int f = 1; f < 5; ++f)
      if (!(f == 3 && ppo))
        CK(hipMemcpyAsync(dst[f], hb + off[f], N * rb[f] / T, hipMemcpyDefault, h->h2d));
  }
  // obs rows: runs of adjacent source rows become one copy, dealt round-robin over the streams
  const char* const* ob = reinterpret_cast<const char* const*>(rows->obs);
  int k = 0;
  for (int b = 0; b < n;) {
    int e = b + 1;
    while (e < n && ob[e] == ob[e - 1] + rb[0]) ++e;
    char* d = (char*)dst[0] + (size_t)b * rb[0];
    const size_t len = (size_t)(e - b) * rb[0];
    CK(hipMemcpyAsync(d, ob[b], len, hipMemcpyDefault, h->h2d_s[k++ % ns]));
    b = e;
  }
  for (int i = 1; i < ns; ++i) {
    CK(hipEventRecord(h->h2d_join[i], h->h2d_s[i]));
    CK(hipStreamWaitEvent(h->h2d, h->h2d_join[i], 0));
  }
  CK(hipEventRecord(s.ready, h->h2d));
  return 0;
}
}  // namespace

int impala_stage_wait(impala_learner* h, int slot) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (slot < 0 || slot >= h->n_slots) return fail(IMPALA_E_INVALID, "slot out of range");
  if (int r = wait_staged(h, slot)) return r;
  CK(hipEventSynchronize(h->ring[slot].ready));
  return 0;
}

int impala_slot_batch(impala_learner* h, int slot, void* stream, impala_batch* out) {
  if (!h || !out) return fail(IMPALA_E_INVALID, "null argument");
  if (slot < 0 || slot >= h->n_slots) return fail(IMPALA_E_INVALID, "slot out of range");
  if (int r = wait_staged(h, slot)) return r;  // its copies are enqueued (ready recorded)
  CK(hipSetDevice(h->device));
  CK(hipStreamWaitEvent((hipStream_t)stream, h->ring[slot].ready, 0));
  *out = h->ring[slot].dev;
  return 0;
}

int impala_slot_release(impala_learner* h, int slot, void* stream) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (slot < 0 || slot >= h->n_slots) return fail(IMPALA_E_INVALID, "slot out of range");
  CK(hipSetDevice(h->device));
  CK(hipEventRecord(h->ring[slot].done, (hipStream_t)stream));
  return 0;
}

int impala_kernel_count(void) { return K_COUNT; }
const char* impala_kernel_name(int kernel_id) {
  return (kernel_id >= 0 && kernel_id < K_COUNT) ? kKernelNames[kernel_id] : "";
}

int impala_timer_start(impala_learner* h, int kernel_id, int max_launches) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (kernel_id < -1 || kernel_id >= K_COUNT || max_launches < 0)
    return fail(IMPALA_E_INVALID, "bad kernel id / capacity");
  CK(hipSetDevice(h->device));
  if (kernel_id < 0) {  // disarm every timer
    for (auto& t : h->timers) t.armed = false;
    h->timers_armed = 0;
    return 0;
  }
  auto& t = h->timers[kernel_id];
  if (max_launches > t.cap) {
    for (int i = 0; i < 2 * t.cap; ++i) (void)hipEventDestroy(t.ev[i]);
    delete[] t.ev;
    t.ev = new hipEvent_t[2 * max_launches]();
    t.cap = 0;
    for (int i = 0; i < 2 * max_launches; ++i) CK(hipEventCreate(&t.ev[i]));
    t.cap = max_launches;
  }
  if (!t.armed) h->timers_armed++;
  t.armed = true;
  t.n = 0;
  h->timer_last = kernel_id;
  return 0;
}

int impala_timer_read_kernel(impala_learner* h, int kernel_id, float* total_ms, int* launches) {
  if (!h || !total_ms || !launches) return fail(IMPALA_E_INVALID, "null argument");
  if (kernel_id < 0 || kernel_id >= K_COUNT) return fail(IMPALA_E_INVALID, "bad kernel id");
  CK(hipSetDevice(h->device));
  auto& t = h->timers[kernel_id];
  float tot = 0.f;
  for (int i = 0; i < t.n; ++i) {
    CK(hipEventSynchronize(t.ev[2 * i + 1]));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, t.ev[2 * i], t.ev[2 * i + 1]));
    tot += ms;
  }
  *total_ms = tot;
  *launches = t.n;
  if (t.armed) h->timers_armed--;
  t.armed = false;
  t.n = 0;
  return 0;
}

int impala_step_clock(impala_learner* h, unsigned long long* stamps, int n) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (n < 0 || (n > 0 && !stamps)) return fail(IMPALA_E_INVALID, "bad step clock buffer / count");
  if (n > 0 && h->fwd_chain)  // the A/B forward-chain launch takes no stamp
    return fail(IMPALA_E_UNSUPPORTED, "the step clock does not stamp the IMPALA_FWD_CHAIN forward");
  h->clock_buf = n > 0 ? stamps : nullptr;
  h->clock_n = n;
  h->clock_i = 0;
  return 0;
}

int impala_step_clock_end(impala_learner* h, void* stream, int* steps) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (!h->clock_buf) return fail(IMPALA_E_STATE, "step clock not armed");
  CK(hipSetDevice(h->device));
  unsigned long long* out = h->clock_buf + h->clock_i;
  if (steps) *steps = h->clock_i;
  h->clock_buf = nullptr;
  h->clock_n = h->clock_i = 0;
  if (int r = klaunch(h, -1, "clock_stamp", clock_stamp_kernel, dim3(1), dim3(64),
                      (hipStream_t)stream, out))
    return r;
  return 0;
}

int impala_timer_read(impala_learner* h, float* total_ms, int* launches) {
  if (!h) return fail(IMPALA_E_INVALID, "null handle");
  if (h->timer_last < 0) {
    if (!total_ms || !launches) return fail(IMPALA_E_INVALID, "null argument");
    *total_ms = 0.f;
    *launches = 0;
    return 0;
  }
  return impala_timer_read_kernel(h, h->timer_last, total_ms, launches);
}

int impala_vtrace(const float* v_tm1, const float* v_t, const float* r_t, const float* discount_t,
                  const float* rho_tm1, int B, int L, float lambda_, float clip_rho_threshold,
                  float clip_pg_rho_threshold, float* pg_advantage, float* td_error,
                  float* q_estimate, void* stream) {
  if (B < 1 || L < 1 || L > 64) return fail(IMPALA_E_INVALID, "need B >= 1 and 1 <= L <= 64");
  if (!v_tm1 || !v_t || !r_t || !discount_t || !rho_tm1 || !pg_advantage || !td_error ||
      !q_estimate)
    return fail(IMPALA_E_INVALID, "null pointer");
  const int S = next_pow2(L);
  const int wgs = cdiv(B, 4 * (64 / S));
  vtrace_kernel<<<wgs, 256, 0, (hipStream_t)stream>>>(v_tm1, v_t, r_t, discount_t, rho_tm1, B, L, S,
                                                      lambda_, clip_rho_threshold,
                                                      clip_pg_rho_threshold, pg_advantage,
                                                      td_error, q_estimate);
  CK_LAUNCH("vtrace");
  return 0;
}

int impala_loss_head(const float* logits, const float* values, const int64_t* actions,
                     const float* rewards, const float* discounts, const float* behaviour_logits,
                     int B, int T, int A, float entropy_coeff, float lambda_, float clip_rho,
                     float clip_pg_rho, int vtrace_grad_mode, float* dlogits, float* dvalues,
                     float* metrics6, float* adv, float* err, float* q, float* rho, void* stream) {
  if (B < 1 || T < 2 || T > 64 || A < 1 || A > net::MAX_A)
    return fail(IMPALA_E_INVALID, "need B >= 1, 2 <= T <= 64, 1 <= A <= 15");
  if (vtrace_grad_mode < IMPALA_VTRACE_SG_ADVANTAGE || vtrace_grad_mode > IMPALA_VTRACE_SG_NONE)
    return fail(IMPALA_E_INVALID, "unknown vtrace_grad_mode");
  if (!logits || !values || !actions || !rewards || !discounts || !behaviour_logits || !dlogits ||
      !dvalues || !metrics6)
    return fail(IMPALA_E_INVALID, "null pointer");
  const bool dbg = adv && err && q;
  hipStream_t st = (hipStream_t)stream;
  const int S = next_pow2(T);
  const int wgs = cdiv(B, 4 * (64 / S));
  float* part = nullptr;
  CK(hipMallocAsync((void**)&part, (size_t)wgs * 8 * 4, st));
  LossArgs la{};
  la.logits = logits; la.lg_ld = A; la.values = values; la.v_ld = 1;
  la.act = actions; la.rew = rewards; la.disc = discounts; la.mu = behaviour_logits;
  la.B = B; la.T = T; la.A = A; la.S = S; la.vt_mode = vtrace_grad_mode;
  la.lam = lambda_; la.crho = clip_rho; la.cpg = clip_pg_rho; la.ent_coef = entropy_coeff;
  la.partials = part;
  la.dbg_adv = dbg ? adv : nullptr; la.dbg_err = dbg ? err : nullptr; la.dbg_q = dbg ? q : nullptr;
  la.dbg_rho = rho;
  loss_head_kernel<float><<<wgs, 256, 0, st>>>(la, dlogits, A, dvalues, 1, 0);
  CK_LAUNCH("loss_head");
  finalize_loss_kernel<<<1, 64, 0, st>>>(part, wgs, B, T, entropy_coeff, metrics6);
  CK_LAUNCH("finalize_loss");
  CK(hipFreeAsync(part, st));
  return 0;
}

int impala_ppo_loss_head(const float* logits, const float* values, const int64_t* actions,
                         const float* targets, const float* behaviour_logits, int N, int A,
                         float entropy_coeff, float clip_coeff, float* dlogits, float* dvalues,
                         float* metrics7, void* stream) {
  if (N < 1 || A < 1 || A > net::MAX_A) return fail(IMPALA_E_INVALID, "need N >= 1, 1 <= A <= 15");
  if (!logits || !values || !actions || !targets || !behaviour_logits || !dlogits || !dvalues ||
      !metrics7)
    return fail(IMPALA_E_INVALID, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int wgs = cdiv(N, 256);
  float *part = nullptr, *m9 = nullptr;
  CK(hipMallocAsync((void**)&part, (size_t)wgs * 8 * 4, st));
  CK(hipMallocAsync((void**)&m9, IMPALA_NUM_METRICS * 4, st));
  ppo_loss_head_kernel<<<wgs, 256, 0, st>>>(logits, values, actions, targets, behaviour_logits, N,
                                            A, entropy_coeff, (float)(1.0 - (double)clip_coeff),
                                            (float)(1.0 + (double)clip_coeff), dlogits, dvalues,
                                            part);
  CK_LAUNCH("ppo_loss_head");
  finalize_ppo_kernel<<<1, 64, 0, st>>>(part, wgs, N, entropy_coeff, m9);
  CK_LAUNCH("finalize_ppo");
  CK(hipMemcpyAsync(metrics7, m9, 6 * 4, hipMemcpyDeviceToDevice, st));
  CK(hipMemcpyAsync(metrics7 + 6, m9 + IMPALA_M_TARGET, 4, hipMemcpyDeviceToDevice, st));
  CK(hipFreeAsync(part, st));
  CK(hipFreeAsync(m9, st));
  return 0;
}

}  // extern "C"
