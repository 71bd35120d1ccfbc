/* impala_hip.h — C-ABI of the MI355X-native IMPALA learner (libimpala_hip.so).
 *
 * Drop-in boundary for the reference's learner path.  Every entry point replaces a piece of
 * the reference's PyTorch learner (paths relative to the d3sm0/impala repository):
 *
 *   impala_train_step      agents/impala/learning.py:140-177  ImpalaLearner._train_step
 *                          (forward, Categorical log-prob / ratio, batched V-trace, pg/value/
 *                          entropy loss, backward, clip_grad_norm_(0.5), Adam.step)
 *   impala_compute_grads   learning.py:141-170 (zero_grad .. loss.backward + metrics)
 *   impala_ppo_train_step  agents/ppo/learning.py:131-143  PPOLearner._train_step
 *                          (losses.py:131-155 ppo_loss, backward, clip, Adam)
 *   impala_apply_update    learning.py:172-176 (clip_grad_norm_ + optimizer.step), after the
 *                          caller's gradient all-reduce in the data-parallel learner
 *   impala_forward         models/distributed_models.py:17-19 AtariPPOModel.forward
 *   impala_act             models/distributed_models.py:21-32 AtariPPOModel.act (forward +
 *                          argmax / softmax-multinomial action)
 *   impala_vtrace          rlego.vtrace_td_error_and_advantage as called through
 *                          learning.py:15-26,150-153 (returns pg_advantage, td_error, q)
 *   impala_loss_head       learning.py:144-170 given network outputs (loss, metrics, d/dlogits,
 *                          d/dvalues)
 *   impala_bind_state      the optimizer/parameter ownership of agents/impala/builder.py:42-59
 *
 * Conventions: plain pointers and sizes, no torch types.  All tensor pointers are DEVICE
 * pointers on the learner's device; `stream` is a hipStream_t passed as void* (NULL = the
 * legacy default stream).  Every call returns 0 on success or a non-zero status (a hipError_t
 * value, or IMPALA_E_* below); impala_last_error() describes the last failure of the calling
 * thread.  Calls are asynchronous on `stream` (no host synchronisation inside), except
 * impala_create / impala_destroy.  No exceptions or aborts cross the ABI.
 *
 * Layouts (batch-major, as agents/impala/learning.py:142-145):
 *   obs               uint8  [B][T][3][64][64]
 *   actions           int64  [B][T]
 *   rewards, discounts float [B][T]
 *   behaviour_logits  float  [B][T][A]
 * Parameters: one flat fp32 buffer in torch state_dict order of AtariPPOModel
 * (model.body.body.{0,2,4}.{weight,bias}, model.projection.{0,1}.{weight,bias},
 *  model.actor.{weight,bias}, model.critic.{weight,bias}); grads / Adam moments alike.
 */
#ifndef IMPALA_HIP_H_
#define IMPALA_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IMPALA_ABI_VERSION 3

#define IMPALA_OK 0
#define IMPALA_E_INVALID 1001   /* bad argument / shape */
#define IMPALA_E_STATE 1002     /* state not bound / wrong call order */
#define IMPALA_E_UNSUPPORTED 1003
#define IMPALA_E_RCCL 1004      /* RCCL missing or a collective call failed */

#define IMPALA_DTYPE_F32 0      /* fp32 operands, f32 MFMA (parity mode) */
#define IMPALA_DTYPE_BF16 1     /* bf16 operands, fp32 accumulate / master weights */

/* metric slots written to the bound metrics buffer (names as learning.py:161-174) */
#define IMPALA_M_LOSS 0
#define IMPALA_M_ENTROPY 1
#define IMPALA_M_TD 2
#define IMPALA_M_PG 3
#define IMPALA_M_KL 4
#define IMPALA_M_RATIO 5
#define IMPALA_M_GRAD_NORM 6
#define IMPALA_M_STEP 7
#define IMPALA_M_TARGET 8       /* PPO only: train/target (losses.py:150) */
#define IMPALA_NUM_METRICS 9

#define IMPALA_ALGO_IMPALA 0    /* V-trace actor-critic (agents/impala/learning.py:140-177) */
#define IMPALA_ALGO_PPO 1       /* PPO clipped surrogate (agents/ppo/learning.py:131-143) */

/* V-trace gradient semantics.  learning.py:148-155 detaches neither rho nor
 * the advantage it multiplies into pg_loss; which V-trace quantities are constants is decided
 * inside the third-party rlego.vtrace_td_error_and_advantage (absent, unpinned).  Forward values
 * do not depend on the mode.
 *   SG_ADVANTAGE targets and pg advantages constant (default): SURVEY.md §8(c)'s restatement,
 *                the IMPALA paper's estimator
 *   SG_TARGETS   rlax vtrace_td_error_and_advantage(stop_target_gradients=True) taken literally
 *                with the reference's un-detached advantage: extra terms through
 *                min(clip_pg_rho, rho), v_tm1 and the bootstrap v_t[-1]
 *   SG_NONE      stop_target_gradients=False: gradients through the whole V-trace scan */
#define IMPALA_VTRACE_SG_ADVANTAGE 0
#define IMPALA_VTRACE_SG_TARGETS 1
#define IMPALA_VTRACE_SG_NONE 2

typedef struct impala_learner impala_learner;

typedef struct {
  int batch_size;              /* B per replica (conf/agent/impala.yaml batch_size)          */
  int rollout_length;          /* T (conf/agent/impala.yaml rollout_length), 2..64           */
  int num_actions;             /* A (procgen 15), 1..15                                      */
  int dtype;                   /* IMPALA_DTYPE_*                                             */
  float lr, adam_beta1, adam_beta2, adam_eps;   /* builder.py:43-44: lr 1e-4, eps 1e-5     */
  float max_grad_norm;         /* learning.py:93: 0.5                                        */
  float entropy_coeff;         /* learning.py:94: 0.01                                       */
  float vtrace_lambda;         /* rlego default 1.0                                          */
  float clip_rho_threshold;    /* rlego default 1.0                                          */
  float clip_pg_rho_threshold; /* rlego default 1.0                                          */
  int world_size;              /* data-parallel replicas (gradient average divisor)          */
  int algo;                    /* IMPALA_ALGO_*; PPO needs rollout_length 1 (flat transitions) */
  float ppo_clip;              /* losses.py:131 clip_coeff 0.1                               */
  int vtrace_grad_mode;        /* IMPALA_VTRACE_SG_*, default IMPALA_VTRACE_SG_ADVANTAGE      */
} impala_config;

typedef struct {
  const uint8_t* obs;
  const int64_t* actions;
  const float* rewards;
  const float* discounts;
  const float* behaviour_logits;
} impala_batch;

/* PPO transitions (agents/ppo/learning.py:132): obs [N][3][64][64], actions [N], value
 * targets [N], behaviour (reference-policy) logits [N][A]; N = batch_size. */
typedef struct {
  const uint8_t* obs;
  const int64_t* actions;
  const float* targets;
  const float* behaviour_logits;
} impala_ppo_batch;

int impala_abi_version(void);
const char* impala_last_error(void);
int impala_config_default(impala_config* cfg);
/* number of fp32 parameters of AtariPPOModel for `num_actions` (344,496 for A = 15) */
size_t impala_param_count(int num_actions);

int impala_create(const impala_config* cfg, int device, impala_learner** out);
int impala_destroy(impala_learner* h);

/* Bind caller-owned device buffers (each impala_param_count() floats; metrics
 * IMPALA_NUM_METRICS floats).
 * Only `params` is required for impala_forward (inference-only handles); the training calls
 * need all five.
 * The library reads/writes them in place: params and Adam moments are updated by
 * impala_apply_update, grads hold the post-clip gradient afterwards (as p.grad does). */
int impala_bind_state(impala_learner* h, float* params, float* grads, float* exp_avg,
                      float* exp_avg_sq, float* metrics, void* stream);
/* Point the following steps' metrics (IMPALA_NUM_METRICS floats, every slot written by each
 * step) at another caller-owned device buffer, host-side only: a learner hands every step a
 * fresh vector -- the values it returns (agents/impala/learning.py:161-174) -- instead of
 * copying the bound one after the step (a device copy of 36 bytes costs ~5 us of the stream). */
int impala_set_metrics(impala_learner* h, float* metrics);
/* Also write each following step's metrics vector to `host` (16 floats of page-locked host
 * memory, e.g. hipHostMalloc / torch pin_memory; NULL stops it): the step's last kernel stores
 * the IMPALA_NUM_METRICS values there, then sets the 32-bit word host[15] to 1 after a system
 * fence.  A caller that zeroes host[15] before enqueueing the step reads `float(v)` of every
 * metric (agents/distributed_agent.py:29-31) from host memory as soon as it sees the word (or
 * after an event recorded behind the step), with no device-to-host copy enqueued.  Not with the
 * A/B fused update. */
int impala_set_metrics_host(impala_learner* h, float* host);
/* Re-derive the kernel-layout weights after the caller changed `params` (load_state_dict). */
int impala_refresh_weights(impala_learner* h, void* stream);
/* Adam step counter (torch state['step']); for checkpoint resume. */
int impala_set_step(impala_learner* h, int64_t step, void* stream);

/* Debug export of the step's own V-trace (IMPALA handles): when `out` is non-NULL, every
 * following training step writes the pg_advantage, td_error and q_estimate it computed inside
 * the fused head ([3][B][T-1], learning.py:150-153) and the importance ratio rho ([B][T],
 * learning.py:148), then the values v the scan ran on ([B][T], learning.py:146) to `out`
 * (3*B*(T-1) + 2*B*T floats, device memory).  NULL disables it. */
int impala_set_debug_vtrace(impala_learner* h, float* out);

/* Policy/value forward of n frames (n <= B*T): logits [n][A], values [n]. */
int impala_forward(impala_learner* h, const uint8_t* obs, int n, float* logits, float* values,
                   void* stream);

/* Actor inference (models/distributed_models.py:21-32 AtariPPOModel.act) for n frames: the
 * forward, then per frame logits [n][A], value [n] and the action [n] -- argmax of the logits
 * where deterministic[f] != 0 (deterministic may be NULL: deterministic_all applies to every
 * frame), else a sample of softmax(logits) drawn from a counter-based uniform keyed by
 * (seed, counter, f); pass a fresh counter per call. */
int impala_act(impala_learner* h, const uint8_t* obs, int n, const uint8_t* deterministic,
               int deterministic_all, uint64_t seed, uint64_t counter, int64_t* actions,
               float* logits, float* values, void* stream);

/* Full learner update for one batch (world_size must be 1). */
int impala_train_step(impala_learner* h, const impala_batch* batch, void* stream);
/* PPOLearner._train_step (agents/ppo/learning.py:131-143) on an IMPALA_ALGO_PPO handle:
 * forward, ppo_loss, backward, clip_grad_norm_, Adam; metrics slots 0-8 (slot 8 = target).
 * The data-parallel calls (impala_compute_grads*, impala_apply_update) take the same batch
 * as an impala_batch with rewards = targets and discounts unused. */
int impala_ppo_train_step(impala_learner* h, const impala_ppo_batch* batch, void* stream);
/* Data-parallel split: gradients of the local batch into `grads` (local mean) ... */
int impala_compute_grads(impala_learner* h, const impala_batch* batch, void* stream);
/* ... caller all-reduces (sums) `grads` across replicas ... then: average (1/world_size),
 * global-norm clip and Adam. */
int impala_apply_update(impala_learner* h, void* stream);
/* The same gradients in two parts, so the all-reduce of the first bucket overlaps the rest of
 * the backward (SURVEY.md §8(e) "2 buckets").  part 0: forward and backward through the conv3
 * weight gradient; on return (stream order) grads[impala_grad_bucket_offset(h) ..] -- conv3,
 * LayerNorm, FC and heads -- are final.  part 1 (same batch): the conv2 weight gradient and
 * conv2 dgrad + conv1 wgrad; then grads[0 .. offset) -- conv1, conv2 -- and the metrics are
 * final.  part 0 then part 1 give bit-identical grads to impala_compute_grads. */
int impala_compute_grads_part(impala_learner* h, const impala_batch* batch, int part, void* stream);
size_t impala_grad_bucket_offset(const impala_learner* h);
/* Three buckets, for a longer all-reduce window: part 2 (forward, heads step, FC weight
 * gradient, FC dgrad) leaves grads[impala_grad_bucket_offset_fc(h) ..] -- FC and heads, 1.07 MB
 * of the 1.38 MB -- final; part 3 (same batch: LayerNorm backward, conv3 dgrad and weight
 * gradient) finalises [impala_grad_bucket_offset(h), impala_grad_bucket_offset_fc(h)); part 4
 * = part 1.  Parts 2, 3, 4 give bit-identical grads to impala_compute_grads.
 * Two buckets with the fused per-frame backward: part 2, then part 6 (same batch: the fused
 * LayerNorm / conv3 / conv2 input gradients + conv1 weight gradient, the conv3 + conv2 weight
 * gradients) finalises [0, impala_grad_bucket_offset_fc(h)) and the metrics.  Parts 2, 6 give
 * bit-identical grads to impala_compute_grads. */
size_t impala_grad_bucket_offset_fc(const impala_learner* h);

/* Native data-parallel step (SURVEY.md §8(b) impala_create(..., rccl_comm), §8(e)): the handle
 * owns an RCCL communicator over the world_size replicas (one process per GPU), so the whole
 * data-parallel step -- learning.py:141-176 on the local shard, the gradient all-reduce over
 * xGMI, clip and Adam on the summed gradient -- is enqueued by one call with no host round trip.
 * impala_dp_unique_id: one rank creates the 128-byte communicator id (ncclGetUniqueId) and the
 * caller hands it to every rank (torch.distributed.broadcast); impala_dp_init (collective: every
 * rank calls it, nranks = the handle's world_size) creates the communicator.  RCCL is loaded at
 * run time (librccl.so.1; inside torch the already-loaded copy). */
#define IMPALA_DP_ID_BYTES 128
int impala_dp_unique_id(void* out);
int impala_dp_init(impala_learner* h, const void* unique_id, int nranks, int rank);
/* *nranks = the rank count of the handle's RCCL communicator (ncclCommCount), 0 before
 * impala_dp_init: the bench records it so a multi-GPU result shows RCCL saw every rank. */
int impala_dp_nranks(const impala_learner* h, int* nranks);
/* buckets 1: the whole backward, then one in-place ncclAllReduce(sum) of the flat gradient on
 * `stream`, then the update.  buckets 2: part 2 (forward, heads step, FC gradients), whose FC +
 * heads gradient (1.07 MB) is all-reduced on the handle's side stream while part 6 (the
 * per-frame backward, the conv weight gradients) runs on `stream`; then the conv + LayerNorm
 * bucket; `stream` waits for both before the update.  Both give bit-identical parameters. */
int impala_dp_train_step(impala_learner* h, const impala_batch* batch, int buckets, void* stream);

/* Replay gather (agents/impala/builder.py:30-36 UniformSampler.sample + learning.py:121-123
 * collate/H2D, done in HBM): for each field f < nfields (<= 8), copy row idx[i] of src[f] to
 * row i of dst[f], rows of row_bytes[f] bytes (multiple of 4); idx is a device int64 [n]. */
int impala_gather_rows(const void* const* src, void* const* dst, const size_t* row_bytes,
                       int nfields, const int64_t* idx, int n, void* stream);
/* The same gather with the row indices in HOST memory, read during the call and passed in the
 * launches' own arguments (256 rows per launch): no index upload, so nothing but the gather
 * itself is enqueued on `stream` (DeviceReplayBuffer.sample). */
int impala_gather_rows_hidx(const void* const* src, void* const* dst, const size_t* row_bytes,
                            int nfields, const int64_t* host_idx, int n, void* stream);

/* The full learner step (impala_train_step) on B trajectories read IN PLACE from a replay ring
 * (agents/impala/builder.py:30-36 replay + learning.py:121-123,142 sample / collate / .to):
 * `ring` holds the ring's five arrays -- obs u8 [capacity][T][3][64][64], actions i64
 * [capacity][T], rewards / discounts f32 [capacity][T], behaviour logits f32 [capacity][T][A]
 * (device memory) -- and rows[0..n) (host memory, n == batch_size <= 256, each in
 * [0, capacity)) the sampled slots: trajectory b of the step is slot rows[b].  No gather is
 * enqueued; the forward, the fused head and the per-frame backward read the ring's rows
 * through a row map in their launch arguments.  Bitwise equal to impala_train_step on the
 * gathered batch.  IMPALA_E_UNSUPPORTED when the handle does not run the default fused
 * kernels (A/B knobs), world_size > 1 or PPO: gather, then impala_train_step. */
int impala_train_step_rows(impala_learner* h, const impala_batch* ring, const int64_t* rows, int n,
                           int64_t capacity, void* stream);

/* Host staging ring (SURVEY.md §8(b) impala_stage; replaces the 5·B pageable `.to(device)`
 * copies of learning.py:121-123).  The handle owns `nslots` device batch slots of B*T frames
 * and a non-blocking H2D stream:
 *   impala_stage_init     allocate the ring (1..8 slots; re-init frees the old ring) and, for the
 *                         SDMA copy path, prime it: the staging loop runs 24 rounds on a scratch
 *                         page-locked batch, so the runtime's one-time SDMA-queue creations
 *                         (6-9 ms host stalls inside hipMemcpyAsync) fall here and not into the
 *                         first steps; ~50 ms (IMPALA_STAGE_PRIME=<rounds>, 0 = off)
 *   impala_stage          enqueue the H2D copies of one host batch (page-locked memory makes
 *                         them asynchronous; discounts may be NULL on PPO handles) into `slot`,
 *                         ordered after the last impala_slot_release of that slot
 *   impala_stage_wait     block the host until the copies into `slot` have finished (the host
 *                         batch may then be overwritten)
 *   impala_slot_batch     make `stream` wait for the slot's copies; *out = its device views,
 *                         to pass to impala_train_step / impala_compute_grads*
 *   impala_slot_release   record on `stream` that the steps reading the slot are enqueued
 * With two slots, staging batch k+1 overlaps the step on batch k.  The copies are SDMA
 * (hipMemcpyAsync) of obs over 2 streams, plus one small pull-kernel launch for the other
 * four fields when they are page-locked and device-mapped (IMPALA_H2D_STREAMS,
 * IMPALA_H2D_SMALL_PULL, IMPALA_H2D_KERNEL select other paths).  Call
 * impala_stage_wait on a slot before restaging it, as a producer refilling its host buffers
 * must: a host that stages without ever waiting runs ahead and the runtime stalls the copies. */
int impala_stage_init(impala_learner* h, int nslots);
int impala_stage(impala_learner* h, const impala_batch* host, int slot);
/* Row staging: the same as impala_stage for a batch the caller has NOT collated -- the list of
 * B trajectories that replay_buffer.sample(B) returns (agents/impala/learning.py:121-123,142;
 * rlmeta CircularBuffer rows).  rows->obs[b] .. rows->behaviour_logits[b] point at trajectory
 * b's T-row fields in host memory (obs T*3*64*64 bytes, actions T int64, rewards / discounts T
 * floats, behaviour_logits T*A floats; discounts may be NULL on PPO handles); n must equal the
 * batch size.  Each obs row is copied by SDMA straight from its own memory into the slot (rows
 * in page-locked memory -- e.g. a pinned replay arena -- make the copies asynchronous;
 * adjacent rows are merged into one copy); the small fields are collated by the host into a
 * page-locked block of the slot (the call waits for the slot's previous copies first). */
typedef struct {
  const void* const* obs;
  const void* const* actions;
  const void* const* rewards;
  const void* const* discounts;
  const void* const* behaviour_logits;
} impala_rows;
int impala_stage_rows(impala_learner* h, const impala_rows* rows, int n, int slot);
/* The same staging run by the handle's staging thread: returns once the row pointers are
 * copied, before the host collate; the rows must stay unchanged until impala_stage_wait(slot).
 * impala_slot_batch / impala_stage_wait on the slot (and every other staging call) first wait
 * for its job, and report the job's failure if it failed.  The host's collate of step k+1 then
 * runs beside the caller's enqueue of step k (ImpalaLearner's prefetch). */
int impala_stage_rows_async(impala_learner* h, const impala_rows* rows, int n, int slot);
int impala_stage_wait(impala_learner* h, int slot);
int impala_slot_batch(impala_learner* h, int slot, void* stream, impala_batch* out);
int impala_slot_release(impala_learner* h, int slot, void* stream);

/* Live launch timer (bench / roofline): arm kernel `kernel_id` (see impala_kernel_name) for its
 * next `max_launches` launches; each is launched with hipExtLaunchKernel and a start / stop
 * event pair, which the runtime stamps with the kernel's own begin / end (the duration
 * rocprofv3's kernel trace reports, without the launch gap).  Several kernels may be armed at
 * once; kernel_id -1 disarms all.  impala_timer_read_kernel() synchronises on a kernel's events,
 * returns the summed duration and launch count, and disarms it; impala_timer_read() does the
 * same for the kernel armed last. */
int impala_kernel_count(void);
const char* impala_kernel_name(int kernel_id);
int impala_timer_start(impala_learner* h, int kernel_id, int max_launches);
int impala_timer_read(impala_learner* h, float* total_ms, int* launches);
int impala_timer_read_kernel(impala_learner* h, int kernel_id, float* total_ms, int* launches);

/* Device step clock (bench): the first kernel of each of the next `n` learner steps (train,
 * data-parallel and PPO steps; not impala_act) stamps the device's constant 100 MHz clock
 * (s_memrealtime) as its first workgroup starts, into stamps[0 .. n-1] (a device buffer of
 * n + 1 uint64).  impala_step_clock_end enqueues one 1-thread kernel on `stream` that stamps
 * the slot after the last stamped step (stamps[*steps], *steps = the steps stamped, <= n)
 * once that step has finished, and disarms.  Step i took stamps[i+1] - stamps[i]
 * ticks of 10 ns.  Unlike a timing event per step, nothing is enqueued between the steps (an
 * event or marker per step costs the fp32 step ~1.4 %, tools/region_order.py).  Steps run
 * without graph replay while the clock is armed.  n = 0 disarms without stamping. */
int impala_step_clock(impala_learner* h, unsigned long long* stamps, int n);
int impala_step_clock_end(impala_learner* h, void* stream, int* steps);

/* Standalone batched V-trace, [B][L] row-major, L <= 64 (test / reuse entry point). */
int impala_vtrace(const float* v_tm1, const float* v_t, const float* r_t, const float* discount_t,
                  const float* rho_tm1, int B, int L, float lambda_, float clip_rho_threshold,
                  float clip_pg_rho_threshold, float* pg_advantage, float* td_error,
                  float* q_estimate, void* stream);

/* Standalone fused loss head given network outputs: logits [B][T][A], values [B][T].
 * Writes dlogits [B][T][A], dvalues [B][T] (under vtrace_grad_mode, IMPALA_VTRACE_SG_*),
 * metrics[6] (loss, entropy, td, pg, kl, ratio), and optionally (nullable) adv/err/q [B][T-1],
 * rho [B][T]. */
int impala_loss_head(const float* logits, const float* values, const int64_t* actions,
                     const float* rewards, const float* discounts, const float* behaviour_logits,
                     int B, int T, int A, float entropy_coeff, float lambda_, float clip_rho,
                     float clip_pg_rho, int vtrace_grad_mode, float* dlogits, float* dvalues,
                     float* metrics6, float* adv, float* err, float* q, float* rho, void* stream);

/* Standalone PPO loss head (losses.py:131-155) given outputs: logits [N][A], values [N].
 * Writes dlogits [N][A], dvalues [N] and metrics7 (loss, entropy, td, pg, kl, ratio, target). */
int impala_ppo_loss_head(const float* logits, const float* values, const int64_t* actions,
                         const float* targets, const float* behaviour_logits, int N, int A,
                         float entropy_coeff, float clip_coeff, float* dlogits, float* dvalues,
                         float* metrics7, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* IMPALA_HIP_H_ */
