/* sac_hip.h — C-ABI of the MI355X-native SAC learner (in libimpala_hip.so).
 *
 * SURVEY.md §8(f) row 4 / BASELINE config 5.  Every entry point replaces a piece of the
 * reference's PyTorch SAC learner (paths relative to the d3sm0/impala repository):
 *
 *   sac_train_step   agents/sac/learning.py:146-193  SACLearner.train_step after the replay
 *                    sample: _train_critic (:195-211, critic_loss :233-248), _train_actor
 *                    (:213-223, actor_loss :251-257), _train_alpha (:225-230, alpha_loss
 *                    :260-265) and the Polyak updates of the target critic / target actor
 *                    (:174-180); optimizers as agents/sac/builder.py:42-47
 *   sac_act          models/sac_model.py:190-200  SoftActor.act (actor inference)
 *   sac_policy       models/sac_model.py:202-203 + :19-29  SoftActor.policy / to_action
 *   sac_sample       rlmeta UniformSampler.sample + ReplayBuffer gather as built by
 *                    agents/sac/builder.py:30-36, done in HBM (indices, probabilities, rows)
 *
 * Networks (models/sac_model.py): actor = ActorBody (Linear(D,256)-ReLU-Linear(256,256)-ReLU,
 * :92-109) + ContionusHead (fc_mean, fc_logstd with tanh rescale to [-5, 2], :125-139); critic =
 * two SoftQNetwork (Linear(D+K,256)-ReLU-Linear(256,256)-ReLU-Linear(256,1), :75-89).
 *
 * Parameters are flat fp32 buffers in torch `parameters()` order:
 *   actor  : actor.body.body.0.{weight,bias}, actor.body.body.2.{weight,bias},
 *            actor.head.fc_mean.{weight,bias}, actor.head.fc_logstd.{weight,bias}
 *   critic : critic.q1.body.{0,2,4}.{weight,bias}, critic.q2.body.{0,2,4}.{weight,bias}
 * (SoftCritic.critic; the target critic has the same layout, the target actor the actor's).
 *
 * Conventions as impala_hip.h: plain device pointers, `stream` = hipStream_t as void*,
 * 0 = success else a hipError_t or IMPALA_E_* code with impala_last_error() describing it.
 */
#ifndef SAC_HIP_H_
#define SAC_HIP_H_

#include <stddef.h>
#include <stdint.h>

#include "impala_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* metric slots (names as agents/sac/learning.py:243-265 and :206,:220) */
#define SAC_M_QF1_LOSS 0
#define SAC_M_QF2_LOSS 1
#define SAC_M_QF1 2
#define SAC_M_QF2 3
#define SAC_M_QF_LOSS 4
#define SAC_M_CRITIC_GRAD_NORM 5
#define SAC_M_ACTOR_LOSS 6
#define SAC_M_ACTOR_STD 7
#define SAC_M_ACTOR_GRAD_NORM 8
#define SAC_M_ALPHA_LOSS 9
#define SAC_M_ALPHA 10
#define SAC_M_STEP 11
#define SAC_NUM_METRICS 12

#define SAC_HIDDEN 256        /* models/sac_model.py: every hidden layer is 256 wide */
#define SAC_MAX_ACT 16

typedef struct sac_learner sac_learner;

typedef struct {
  int obs_dim;          /* D = prod(observation_space.shape)                       */
  int act_dim;          /* K = prod(action_space.shape), 1..16                     */
  int batch_size;       /* N (conf/agent/sac.yaml batch_size 256)                  */
  int dtype;            /* IMPALA_DTYPE_F32 (parity) / IMPALA_DTYPE_BF16 (perf)    */
  float critic_lr;      /* sac.yaml optimizer.critic_lr 0.003                      */
  float actor_lr;       /* sac.yaml optimizer.actor_lr 0.0003                      */
  float adam_beta1, adam_beta2, adam_eps;  /* torch defaults; eps sac.yaml 1e-5   */
  float max_grad_norm;  /* learning.py:99 default 40 (<= 0: no clipping, None)    */
  float tau;            /* learning.py:102 0.005                                   */
  float gamma;          /* learning.py:233 critic_loss gamma 0.99                  */
  int tune_alpha;       /* sac.yaml tune_alpha true                                */
  float target_entropy; /* sac_model.py:163 -prod(action_space)                   */
  float prio_exponent;  /* learning.py:198 probabilities.pow(-0.4)                */
  uint64_t seed;        /* device Normal noise for rsample() when the batch has none */
} sac_config;

/* One sampled batch (learning.py:147-148 after map_nested(squeeze)).  s, s1 [N][D],
 * a [N][K], r [N] fp32, done [N] uint8 (bool), probabilities [N] fp32 (NULL: all equal).
 * noise: NULL, or [3][N][K] standard-normal draws replacing the three Normal.rsample() calls
 * in call order (target actor on s1, actor on s, actor on s for alpha); NULL draws them on
 * the device (counter-based, seeded by cfg.seed and the step).  priorities: NULL or [N]
 * output, |y - min(q1, q2)| (critic_loss next_priorities). */
typedef struct {
  const float* s;
  const float* a;
  const float* r;
  const float* s1;
  const uint8_t* done;
  const float* probabilities;
  const float* noise;
  float* priorities;
} sac_batch;

/* Caller-owned device state (flat fp32): actor params / grads / Adam moments / target actor,
 * critic likewise with its target, log_alpha[4] = {value, grad, exp_avg, exp_avg_sq}, and
 * metrics[SAC_NUM_METRICS]. */
typedef struct {
  float *actor, *actor_grad, *actor_m, *actor_v, *target_actor;
  float *critic, *critic_grad, *critic_m, *critic_v, *target_critic;
  float* log_alpha;
  float* metrics;
} sac_state;

int sac_config_default(sac_config* cfg);
size_t sac_actor_param_count(int obs_dim, int act_dim);
size_t sac_critic_param_count(int obs_dim, int act_dim);

int sac_create(const sac_config* cfg, int device, sac_learner** out);
int sac_destroy(sac_learner* h);
int sac_bind_state(sac_learner* h, const sac_state* st, void* stream);
/* re-derive kernel-layout weights after the caller changed any bound parameter buffer */
int sac_refresh_weights(sac_learner* h, void* stream);
/* Adam step counters (torch state['step']): critic params, actor params, log_alpha */
int sac_set_steps(sac_learner* h, int64_t critic_step, int64_t actor_step, int64_t alpha_step,
                  void* stream);

int sac_train_step(sac_learner* h, const sac_batch* batch, void* stream);

/* SoftActor.act: action = tanh(mu + std * noise * noise_scale) * action_scale + action_bias
 * for n <= batch_size observations obs [n][D]; noise [n][K] (NULL = zero noise). */
int sac_act(sac_learner* h, const float* obs, int n, const float* noise, float noise_scale,
            float action_scale, float action_bias, float* action, void* stream);
/* SoftActor.forward / policy (sac_model.py:115-122,202-203; to_action with rsample = mean +
 * noise * std, noise NULL = 0): mean [n][K], log_std [n][K], action [n][K], log_prob [n],
 * std [n][K] (any output may be NULL). */
int sac_policy(sac_learner* h, const float* obs, int n, const float* noise, float* mean,
               float* log_std, float* action, float* log_prob, float* std_out, void* stream);
/* SoftCritic.forward / target (sac_model.py:170-175): q1, q2 [n] of the critic (target = 0)
 * or of the target critic (target = 1) at obs [n][D], act [n][K]. */
int sac_q_forward(sac_learner* h, const float* obs, const float* act, int n, int target,
                  float* q1, float* q2, void* stream);

/* Live launch timer (bench / roofline): the step is a fixed chain of launches ("phases",
 * sac_phase_name); arm an event pair around each of the next `max_launches` launches of one
 * phase on the stream it runs on (steps run without graph replay while armed);
 * sac_timer_read synchronises and returns the summed duration. */
int sac_phase_count(void);
const char* sac_phase_name(int phase);
int sac_timer_start(sac_learner* h, int phase, int max_launches);
int sac_timer_read(sac_learner* h, float* total_ms, int* launches);

/* Uniform replay sampling in HBM (UniformSampler over keys [0, size); without replacement
 * when n <= size, as impala_amd.replay.ReplayBuffer): idx [n] int64 drawn from a counter-based
 * generator (seed, counter), probabilities [n] = 1/size, then row idx[i] of each of up to 8
 * fields src[f] (rows of row_bytes[f] bytes, any size) copied to row i of dst[f]. */
int sac_sample(uint64_t seed, uint64_t counter, int64_t size, int n, int64_t* idx,
               float* probabilities, const void* const* src, void* const* dst,
               const size_t* row_bytes, int nfields, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SAC_HIP_H_ */
