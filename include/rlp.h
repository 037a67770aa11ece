/*
 * rlp.h — C-ABI of the MI355X (gfx950) batched env-step + PPO2 rollout library (librlp.so).
 *
 * This is the drop-in boundary for the reference's on-policy hot path
 * (HKPolyU-UAV/ReinforcementLearningPlatform). Every entry point replaces one
 * piece of per-env Python/numpy/torch-CPU code; the reference interface it replaces is cited
 * (path:line, relative to the reference root) next to each declaration.
 *
 * Conventions
 *  - All array pointers are DEVICE pointers (e.g. torch.Tensor.data_ptr() on cuda), unless a
 *    parameter is documented as host memory. Param structs are host memory and are passed to the
 *    kernels by value.
 *  - Physics state is float64, struct-of-arrays: state[d * n + i] is component d of env i.
 *    Observations / actions are float32, env-major: obs[i * S + s].
 *    Rollout buffers are time-major: buf[(t * n + i) * S + s]  (== RolloutBuffer rows, T*n of them).
 *  - Every call is stream-ordered on `stream` (a hipStream_t; NULL = the legacy default stream)
 *    and never synchronises the host unless documented.
 *  - Return value: RLP_OK (0) on success; RLP_EINVAL / RLP_EUNSUPPORTED on bad arguments;
 *    -(int)hipError_t for a HIP launch error. Nothing throws or aborts across the ABI.
 *    rlp_last_error_string() returns a thread-local description of the last failure.
 *  - The library allocates no device memory. Callers own every buffer; calls that need scratch
 *    take a caller-owned workspace sized by a *_workspace_* query and return RLP_EINVAL when it is
 *    too small (checked on the host before any launch).
 */
#ifndef RLP_H_
#define RLP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *rlp_stream_t; /* hipStream_t */

#define RLP_OK 0
#define RLP_EINVAL (-1000)
#define RLP_EUNSUPPORTED (-1001)
#define RLP_ENOMEM (-1002)  /* unused since ABI version 2 (no library allocations); kept reserved */

#define RLP_ABI_VERSION 3  /* 2: caller-owned rollout / mlp_forward workspaces (round 5);
                              3: per-call mlp_precision of rlp_mfma_forward / rlp_value_fixup,
                                 rlp_selftest_gemm_guard, rlp_reward_norm_statistics /
                                 rlp_reward_norm_apply / rlp_gae_normalized (round 6) */

/* ------------------------------------------------------------------------------------------ */
/* Environment kinds. Each kind is one specific reference env copy (copies diverge). */
/* ------------------------------------------------------------------------------------------ */
enum rlp_env_kind {
    /* environment/CartPole/CartPole.py (== demonstration/PPO2/PPO2-4-CartPole/CartPole.py;
       DPPO2 copy differs only in the reset law, expressed through the params). */
    RLP_ENV_CARTPOLE = 1,
    /* demonstration/PPO2/PPO2-4-CartPoleAngleOnly/cartpole_angleonly.py */
    RLP_ENV_CARTPOLE_ANGLEONLY = 2,
    /* environment/SecondOrderIntegration/SecondOrderIntegration.py (+ DPPO2/DDPG copy via params) */
    RLP_ENV_SOI = 3,
    /* environment/UGV/UGVForward.py (+ PPO2/DPPO2 copies via params) */
    RLP_ENV_UGV_FORWARD = 4,
    /* environment/UGV/UGVBidirectional.py (+ PPO2 copy via params) */
    RLP_ENV_UGV_BIDIRECTIONAL = 5,
    /* environment/UavRobust/UavHoverOuterLoop.py: 6-DoF rigid body (uav.py) + FNTSMC attitude
       loop (FNTSMC.py) driven by an RL virtual-acceleration command. */
    RLP_ENV_UAV_HOVER_OUTER_LOOP = 6,
    /* environment/UGVForwardObstacleAvoidance/UGVForwardObstacleAvoidance.py: unicycle + 37-beam
       fake lidar against up to 15 circular obstacles per env (map.py generate_circle_obs_training). */
    RLP_ENV_UGV_OBSTACLE_AVOIDANCE = 7,
};

/* Physics-state dimension D, observation dim S and action dim A per kind (also queryable). */
#define RLP_CARTPOLE_D 5  /* theta, dtheta, x, dx, time */
#define RLP_ANGLEONLY_D 5 /* theta, dtheta, x, dx, time */
#define RLP_SOI_D 7       /* x, y, vx, vy, time, target_x, target_y */
#define RLP_UGV_D 8       /* x, y, vel, phi, omega, time, target_x, target_y */
#define RLP_UAV_D 22      /* x y z vx vy vz phi theta psi p q r | time | pos_ref[3] | s1[3] | att_ref[3] */
#define RLP_UGVOA_NOBS 15   /* obstacle slots per env: obsNum 10 (env dir, PPO2 demo) or 15 (DPPO2 demo,
                               DPPO2-4-UGVForwardObstacleAvoidance/UGVForwardObstacleAvoidance.py:543) */
#define RLP_UGVOA_NLASER 37 /* beams: int(2 * laserRange / laserStep) + 1 = 180/5 + 1 */
#define RLP_UGVOA_D (8 + 3 * RLP_UGVOA_NOBS) /* x y vel phi omega time tx ty | (cx cy r) x NOBS */

/* CartPole.py:27-46 (physical constants), :187-217 get_reward literals, :273-274 reset law. */
typedef struct rlp_cartpole_params {
    double theta_max;   /* deg2rad(45) */
    double dtheta_max;  /* deg2rad(90) */
    double x_max;       /* 1.5 */
    double dx_max;      /* 3 */
    double static_gain; /* 2.0 */
    double M, m, g, ell, kf;
    double fm;       /* 8: action range [-fm, fm] */
    double dt;       /* 0.02 */
    double time_max; /* 5 */
    double reset_theta_lo, reset_theta_hi; /* theta0 ~ U(lo, hi) */
    double reset_x_lo, reset_x_hi;         /* x0 ~ U(lo, hi) */
    double Q_x, Q_dx, Q_theta, Q_omega, R; /* get_reward :192-196 */
    int32_t n_sub_div; /* h = dt / n_sub_div, `while time < tt` (CartPole.py:242-252) */
    int32_t reserved;
} rlp_cartpole_params;

/* Two copies (variant):
 * RLP_ANGLEONLY_PPO2_COPY  demonstration/PPO2/PPO2-4-CartPoleAngleOnly/cartpole_angleonly.py:27-41
 *   (== the DPPO2 copy): one RK4 step of h = dt = 0.02 (:218-229), fm 5, timeMax 5, flags
 *   1 angle / 3 time / 4 success (later overrides), reward -Q_theta th^2 ... (:170-195);
 * RLP_ANGLEONLY_ENV_FILE  environment/CartPole/CartPoleAngleOnly.py:36-39: dt 0.01 in 10 RK4
 *   sub-steps of h = dt/10 under the fp64 `while time < tt` loop (:231-244, 10 or 11 by step
 *   index), fm 8, timeMax 6, flags 1 angle (wins) else 3 time, no success flag (:144-166), and the
 *   angle-increment reward (:168-208: -2 / 0 / +2 as |theta| grows / holds / shrinks in degrees,
 *   +5 inside 0.5 deg, -100 on flag 1, +500 on flag 3). Reset :245-279 / :266-300 alike. */
#define RLP_ANGLEONLY_PPO2_COPY 0
#define RLP_ANGLEONLY_ENV_FILE 1
typedef struct rlp_angleonly_params {
    double theta_max;   /* deg2rad(45) */
    double static_gain; /* 2.0 */
    double norm_dtheta; /* norm_4_boundless_state = 4 */
    double M, m, g, ell, kf;
    double fm;       /* 5 (env file: 8) */
    double dt;       /* 0.02 (env file: 0.01) */
    double time_max; /* 5 (env file: 6) */
    double reset_theta_lo, reset_theta_hi;
    double Q_theta, Q_omega, R; /* 10, 0, 0 (PPO2 copy's reward) */
    int32_t variant;            /* RLP_ANGLEONLY_PPO2_COPY | RLP_ANGLEONLY_ENV_FILE */
    int32_t n_sub_div;          /* env file: 10 (rk44 :232) */
} rlp_angleonly_params;

/* SecondOrderIntegration.py:13-60, reward :251-284, reset :328-352. */
typedef struct rlp_soi_params {
    double map_size[2]; /* 5, 5 */
    double k;           /* 0.15 linear drag */
    double mass;        /* 1.0 */
    double dt;          /* 0.02 (one RK4 step: the `while` loop runs exactly once) */
    double time_max;    /* 5.0 */
    double v_max;       /* 3 (obs normaliser) */
    double f_max;       /* 3: action range [-f_max, f_max]^2 */
    double admissible_error; /* 0 */
    double obs_gain;    /* 1 for the env file; 2 (static_gain) in the DPPO2/DDPG copies */
    double reset_margin; /* 0.1: pos ~ U(0+m, map-m) */
    double Q_pos, Q_vel, Q_acc; /* 1, 0.1, 0.05 (DPPO2/DDPG copies: 1, 0, 0) */
    int32_t success_enabled;    /* 1: flag 3 on success (env file); 0 in the DPPO2/DDPG copies */
    int32_t reserved;
} rlp_soi_params;

/* UGVForward.py / UGVBidirectional.py:34-63, reward :263-279, reset :334-362. */
typedef struct rlp_ugv_params {
    double map_size[2]; /* 5, 5 */
    double dt;          /* 0.02 */
    double time_max;    /* 10 (DPPO2 UGVForward copy: 5) */
    double kf, kt;      /* 0.1, 0.1 */
    double v_max;       /* 3 */
    double omega_max;   /* 2*pi */
    double a_linear_max;  /* 3 */
    double a_angular_max; /* 2*pi */
    double static_gain;   /* 1 */
    double reset_margin;  /* 0.5 */
    double Q_pos, Q_vel, Q_phi, Q_omega; /* 2, 0 (PPO2/DPPO2 copies: 0.1), 2, 1 */
    int32_t phi_gate_abs; /* u_phi active if |e| > 0.1 (PPO2 Bidirectional copy) vs e > 0.1 */
    int32_t reserved;
} rlp_ugv_params;

/* uav.py:12-31 uav_param; FNTSMC.py:4-15 fntsmc_param (attitude loop);
   UavHoverOuterLoop.py:33-43 limits, :93-110 reward. Values of
   demonstration/PPO/PPO-4-UavHoverOuterLoop/train.py:24-56. */
typedef struct rlp_uav_hover_params {
    double m, g;
    double J[3];
    double kr, kt;
    double dt, time_max;
    double pos0[3], vel0[3], angle0[3], pqr0[3];
    double pos_zone[3][2];
    double att_zone[3][2];
    double att_k1[3], att_k2[3], att_alpha[3], att_beta[3], att_gamma[3], att_lmd[3];
    double att_saturation[3];
    double att_ctrl_dt;
    double static_gain;
    double e_pos_max[3], e_pos_min[3];
    double vel_max[3], vel_min[3];
    double dot_att_min[3], dot_att_max[3];
    double u_min, u_max;
    double target_offset; /* generate_random_point(offset=1.0) */
    double Qx, Qv, R;     /* 1, 0.1, 0.02 */
} rlp_uav_hover_params;

/* UGVForwardObstacleAvoidance.py:12-104 (constants), get_fake_laser :274-397, get_state :399-411,
   is_Terminal :433-450, get_reward :452-469, ode/rk44 :471-502, reset :520-557 with
   map.py:152-174 generate_circle_obs_training(5, 5, 4 r_vehicle, 4 r_vehicle, 0.2, 0.5, n_obs).
   shaped = 1 selects the PPO2/DPPO2 demo copies (demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/
   UGVForwardObstacleAvoidance.py): dt 0.05, success ignores omega (:421-427), the r1..r4 shaped
   reward (:449-473) and rk44's gate on the pre-step velocity (:488-500). */
typedef struct rlp_ugv_oa_params {
    double map_size[2];   /* 5, 5 */
    double dt, time_max;  /* 0.1, 15 */
    double kf, kt;        /* 0.1, 0.1 */
    double v_max, e_phi_max, omega_max;   /* 3, pi, 2 pi */
    double a_linear_max, a_angular_max;   /* 3, 2 pi */
    double r_vehicle;     /* 0.15 */
    double laser_dis, laser_blind, laser_range; /* 2, 0, deg2rad(90) */
    double static_gain;   /* 1 */
    double Q_pos, Q_vel, Q_phi, Q_omega;  /* 2, 0, 2, 1 */
    double safety_dis_obs, safety_dis_st; /* 4 r_vehicle, 4 r_vehicle */
    double r_min, r_max;  /* 0.2, 0.5 */
    double st_margin;     /* 0.3: start/target ~ U(margin, map - margin) */
    int32_t n_obs;        /* obstacles placed by reset, <= RLP_UGVOA_NOBS; unused slots are parked
                             outside the map, where they can neither collide nor be seen */
    int32_t max_tries;    /* rejection-sampling bound per draw (an unplaceable obstacle is parked) */
    int32_t shaped;       /* 0: env-dir copy, 1: PPO2/DPPO2 demo copy */
    int32_t reserved;
} rlp_ugv_oa_params;

/* Dimensions of a kind. Returns RLP_EINVAL for an unknown kind. Host-only, no device work. */
int rlp_env_dims(int kind, int *D, int *S, int *A);

/* rl_base.reset(random) — e.g. CartPole.py:266-295, UavHoverOuterLoop.py:152-214.
 * For every env i with (mask == NULL || mask[i] != 0):
 *   init_state != NULL : state[:, i] = init_state[:, i]            (f64, [D][n], teacher forcing)
 *   init_state == NULL : reset law with a counter-based Philox4x32-10 stream keyed by
 *                        (seed, counter, env_id0 + i): bit-identical on every rank/GPU.
 * Hidden controller state that the reference carries across resets (UAV s1 / att_ref,
 * UavHoverOuterLoop.py:152-208) is carried here too. */
int rlp_env_reset(int kind, const void *params, double *state, int n, const uint8_t *mask,
                  const double *init_state, uint64_t seed, uint64_t counter, uint64_t env_id0,
                  rlp_stream_t stream);

/* rl_base.get_state() (e.g. CartPole.py:145-153): obs[i*S+s] (f32). */
int rlp_env_observe(int kind, const void *params, const double *state, int n, float *obs,
                    rlp_stream_t stream);

/* rl_base.step_update(action) (CartPole.py:257-264; SecondOrderIntegration.py:316-326;
 * UGVForward.py:322-332; UavHoverOuterLoop.py:115-150), one env per lane, f64 physics.
 * action [n][A] f32 (the dtype choose_action hands to step_update). Outputs:
 *   obs_cur  [n][S] f32  current_state before the step (nullable)
 *   obs_next [n][S] f32  next_state
 *   reward   [n]    f64  env.reward
 *   flag     [n]    i32  terminal_flag
 *   done     [n]    u8   is_terminal                                                    */
int rlp_env_step(int kind, const void *params, double *state, int n, const float *action,
                 float *obs_cur, float *obs_next, double *reward, int32_t *flag, uint8_t *done,
                 rlp_stream_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Policy / value networks: Linear(+tanh) stacks defined by the demo drivers                   */
/* (demonstration/PPO2/PPO2-4-CartPole/train.py:39-125: fc1/fc2/mean_layer, fc1/fc2/fc3).      */
/* ------------------------------------------------------------------------------------------ */
#define RLP_MLP_MAX_LAYERS 8
enum rlp_act { RLP_ACT_NONE = 0, RLP_ACT_TANH = 1, RLP_ACT_RELU = 2 };

typedef struct rlp_mlp_desc {
    int32_t n_layers;                    /* number of Linear layers */
    int32_t dims[RLP_MLP_MAX_LAYERS + 1]; /* dims[0] = in, dims[l+1] = out of layer l */
    int32_t act[RLP_MLP_MAX_LAYERS];     /* activation after layer l */
} rlp_mlp_desc;

/* Plain parameter layout: for each layer l: W_l row-major [out][in] then b_l [out]
 * (== torch.cat([p.flatten() for p in module.parameters()]) for Linear stacks). */
int64_t rlp_mlp_param_count(const rlp_mlp_desc *desc);

/* Batched forward y[n][out] = MLP(x[n][in]) (nn.Sequential / driver forward()), fp32, MFMA
 * (v_mfma_f32_16x16x4_f32) for every layer; rows with mask[i]==0 are skipped (mask nullable).
 * Unmasked batches of >= 2048 rows run on the tiled GEMM, one launch per layer — or, for the
 * DDPG / SAC actors' shape (three layers, relu, relu, tanh / none, <= 64 inputs, hidden widths
 * multiples of 32 up to 256, <= 8 outputs), all three layers in one fused launch. The per-layer
 * path keeps two hidden activations in `workspace` (device, rlp_mlp_forward_workspace_bytes(desc,
 * n) bytes; 0 — and workspace nullable — for every other path). */
int64_t rlp_mlp_forward_workspace_bytes(const rlp_mlp_desc *desc, int n);
int rlp_mlp_forward(const rlp_mlp_desc *desc, const float *params, const float *x, float *y, int n,
                    const uint8_t *mask, void *workspace, int64_t workspace_bytes,
                    rlp_stream_t stream);

/* Size (floats) and packing of the MFMA-fragment layout used by rlp_rollout for a
 * [S -> H -> H -> A] tanh network (H in {64,128,256}). Returns RLP_EUNSUPPORTED otherwise. */
int64_t rlp_mfma_packed_count(const rlp_mlp_desc *desc);
int rlp_mfma_pack(const rlp_mlp_desc *desc, const float *params, float *packed, rlp_stream_t stream);

/* SAC squashed-Gaussian policy head: SACActor.forward (utils/classes.py:464-486, and the demo
 * drivers' copy with a per-dim log_std clamp, demonstration/SAC/SAC-4-UGVForward/train.py:68-88)
 * after the trunk, plus SAC.choose_action's clamp (Soft_Actor_Critic.py:63-67). Per row i, dim j:
 *   ls = clamp(head[i][A + j], ls_lo[j], ls_hi[j]);  std = exp(ls)
 *   u  = deterministic ? head[i][j] : head[i][j] + std * eps        (Normal.rsample)
 *   log_pi[i] = sum_j Normal(mean, std).log_prob(u) - sum_j 2 (log 2 - u - softplus(-2 u))
 *   action = tanh(u) * gain[j] + off[j], then clamped to [a_min, a_max] when a_min != NULL.
 * head: [n][2A] device (mean | log_std, i.e. the two Linear heads concatenated); eps from
 * `noise` [n][A] when non-NULL, else Philox normals keyed (seed, counter, env_id0 + i) as in
 * rlp_policy_sample. ls_lo, ls_hi, gain, off, a_min, a_max: HOST arrays of A floats (a_min, a_max
 * nullable together); log_pi nullable. fp32 throughout, as torch. */
int rlp_sac_sample(const float *head, int n, int A, const float *ls_lo, const float *ls_hi,
                   const float *gain, const float *off, const float *a_min, const float *a_max,
                   int deterministic, const float *noise, uint64_t seed, uint64_t counter,
                   uint64_t env_id0, float *action, float *log_pi, rlp_stream_t stream);

/* Proximal_Policy_Optimization2.choose_action (Proximal_Policy_Optimization2.py:69-76):
 *   a = clamp(mean + std*eps, a_min, a_max);  logp = Normal(mean, std).log_prob(a)  (per dim)
 * eps from `noise` [n][A] if non-NULL, else Philox normals keyed (seed, counter, env_id0+i).
 * std, a_min, a_max: HOST arrays of A floats. */
int rlp_policy_sample(const float *mean, int n, int A, const float *std, const float *a_min,
                      const float *a_max, const float *noise, uint64_t seed, uint64_t counter,
                      uint64_t env_id0, float *action, float *logp, rlp_stream_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Fused batched rollout (demonstration/PPO2/PPO2-4-CartPole/train.py:184-217 for n envs):    */
/* T x { auto-reset, actor forward + Gaussian sample, critic V(s), env step, buffer append }  */
/* ------------------------------------------------------------------------------------------ */
enum rlp_success_rule {
    RLP_SUCCESS_DONE_AND_FLAG_NE = 0, /* done && flag != F  (PPO2 drivers, train.py:199-205) */
    RLP_SUCCESS_FLAG_NE = 1,          /* flag != F, also on non-terminal steps (DPPO2 CartPole,
                                         DPPO2-4-CartPole/Distributed_PPO2.py:138) */
    RLP_SUCCESS_FLAG_EQ = 2,          /* flag == F  (PPO-4-UavHoverOuterLoop/train.py:217) */
};

typedef struct rlp_rollout_bufs {
    float *obs;        /* [T][n][S] s_t                                     (RolloutBuffer.s)   */
    float *obs_next;   /* [T][n][S] s'_t                                    (RolloutBuffer.s_)  */
    float *action;     /* [T][n][A]                                         (RolloutBuffer.a)   */
    float *logp;       /* [T][n][A]                                         (RolloutBuffer.a_lp)*/
    float *reward;     /* [T][n]   raw env.reward (normalised later)        (RolloutBuffer.r)   */
    float *value;      /* [T][n]   V(s_t)                                                        */
    float *value_next; /* [T][n]   V(s'_t) where !done (== V(s_{t+1})); done rows are left to
                                   rlp_value_fixup (critic on s'_t where the GAE needs it)       */
    uint8_t *done;     /* [T][n]                                            (RolloutBuffer.done)*/
    uint8_t *success;  /* [T][n]                                            (RolloutBuffer.success)*/
    int8_t *flag;      /* [T][n]   terminal_flag                                                 */
} rlp_rollout_bufs;

typedef struct rlp_rollout_cfg {
    int32_t T;            /* steps per env in this segment */
    int32_t n;            /* envs on this device */
    uint64_t seed;        /* Philox key */
    uint64_t step0;       /* global step counter of the first step (Philox counter) */
    uint64_t env_id0;     /* global id of env 0 on this device (rank * n) */
    int32_t success_rule; /* enum rlp_success_rule */
    int32_t success_flag; /* F */
    float std[4];         /* actor.std per action dim (host values) */
    float a_min[4], a_max[4];
    /* per-call kernel selection; 0 = the library-wide default set by rlp_set_mlp_precision /
     * rlp_set_rollout_physics / rlp_set_rollout_sub, else value + 1 (mlp_precision: 1 RLP_MLP_FP32,
     * 2 RLP_MLP_F16X3; physics: 1 register-resident, 2 shared, 4 one 8-wave block per CU, 6 one
     * 4-wave block per CU, 8 auto — the knob's -1; 3, 5, 7 RLP_EINVAL); sub: 0 default, 1, 2, 4 */
    int32_t mlp_precision, physics, sub;
    /* 0: actor / critic are rlp_mfma_pack buffers of [S -> 256 -> 256 -> A] tanh nets (the fused
     * kernels); 1: plain parameters (rlp_mlp_param_count floats, torch order) of any Linear stack
     * whose actor ends in tanh (the PPO2-SOI demo's 4-128-64-32-2 / 4-64-64-1): per step
     * rlp_mlp_forward's kernels + one sample / env-step / append kernel, same draws and buffers */
    int32_t net_layout;
    /* device scratch of the multi-launch paths (net_layout 1, RLP_ENV_UGV_OBSTACLE_AVOIDANCE):
     * rlp_rollout_workspace_bytes(...) bytes, nullable when that is 0 (the fused kernels) */
    void *workspace;
    int64_t workspace_bytes;
} rlp_rollout_cfg;

/* state: [D][n] f64 in/out, carried across segments. need_reset: [n] u8 in/out (1 = env is
 * terminal / fresh and resets, with the reset law, before its next step; the reference driver's
 * `if env.is_terminal: env.reset(random=True)`, train.py:187-191). actor/critic: MFMA-packed
 * (rlp_mfma_pack). Supported kinds: RLP_ENV_CARTPOLE, RLP_ENV_CARTPOLE_ANGLEONLY,
 * RLP_ENV_UGV_FORWARD, RLP_ENV_UGV_BIDIRECTIONAL, RLP_ENV_SOI, RLP_ENV_UAV_HOVER_OUTER_LOOP
 * with actor [S->H->H->A] (tanh, tanh, tanh*gain+off) and critic [S->H->H->1]. */
int rlp_rollout(int kind, const void *env_params, double *state, uint8_t *need_reset,
                const rlp_mlp_desc *actor_desc, const float *actor_packed,
                const rlp_mlp_desc *critic_desc, const float *critic_packed,
                const rlp_rollout_cfg *cfg, const rlp_rollout_bufs *bufs, rlp_stream_t stream);
/* bytes of cfg->workspace that rlp_rollout needs for this kind, nets and cfg (T, n, net_layout):
 * 0 for the fused kernels; RLP_EINVAL on bad arguments. Host-only. */
int64_t rlp_rollout_workspace_bytes(int kind, const rlp_mlp_desc *actor_desc,
                                    const rlp_mlp_desc *critic_desc, const rlp_rollout_cfg *cfg);

/* Batched forward of an MFMA-packed [S->H->H->A] net (H = 256): y[rows][A] (last-layer act
 * applied). Proximal_Policy_Optimization2.evaluate (:63-67) / critic(s) in learn() (:91-92).
 * mlp_precision (per call, as rlp_rollout_cfg.mlp_precision): 0 = the library-wide default
 * (rlp_set_mlp_precision), 1 = RLP_MLP_FP32 (exact f32 MFMA), 2 = RLP_MLP_F16X3 (the rollout's
 * split hidden layer). Concurrent callers pass 1 or 2 and never depend on the global. */
int rlp_mfma_forward(const rlp_mlp_desc *desc, const float *packed, const float *x, float *y,
                     int64_t rows, int mlp_precision, rlp_stream_t stream);

/* Bootstrap values the rollout kernel cannot provide: value_next[i] = critic(obs_next[i]) for
 * rows with done[i] && !success[i] (e.g. CartPole time-outs); every other row is either written by
 * rlp_rollout (V(s'_t) == V(s_{t+1})) or multiplied by (1 - success) = 0 in the GAE (:93).
 * mlp_precision: as rlp_mfma_forward. */
int rlp_value_fixup(const rlp_mlp_desc *critic_desc, const float *critic_packed,
                    const float *obs_next, const uint8_t *done, const uint8_t *success,
                    float *value_next, int64_t rows, int mlp_precision, rlp_stream_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Learn-side scans (Proximal_Policy_Optimization2.learn, :84-100; utils/classes.py:626-656)   */
/* ------------------------------------------------------------------------------------------ */

/* Normalization(shape=1) over the rollout's reward stream (utils/classes.py:647-656):
 * time step t's n rewards are merged into the running statistics in env order (Welford when
 * n == 1, reproducing the reference exactly including the first-call std = x quirk; Chan's
 * parallel merge otherwise), then every reward of step t is normalised with the statistics
 * after that merge. rms: device f64[4] = {count, mean, S, std}, in/out across segments.
 * work: device f64[rlp_reward_norm_workspace(T, n)] scratch. reward_out may alias reward_in.
 * rlp_reward_norm_statistics, then the elementwise normalisation. */
int64_t rlp_reward_norm_workspace(int T, int n);
int rlp_reward_norm(const float *reward_in, int T, int n, double *rms, double *work,
                    float *reward_out, rlp_stream_t stream);

/* The statistics half of rlp_reward_norm (one rank): chunk statistics, per-step merges and the
 * running recurrence (rms updated; step t's (mean_t, std_t) kept in `work` for
 * rlp_gae_normalized). The rewards themselves are not written: rlp_gae_normalized normalises
 * them as it loads them. */
int rlp_reward_norm_statistics(const float *reward_in, int T, int n, double *rms, double *work,
                               rlp_stream_t stream);
/* The normalised rewards themselves, from the statistics a preceding rlp_reward_norm_statistics
 * (or rlp_reward_norm / rlp_reward_norm_finish) left in `work` (for callers that keep them). */
int rlp_reward_norm_apply(const float *reward_in, int T, int n, const double *work,
                          float *reward_out, rlp_stream_t stream);

/* rlp_reward_norm in two stages, for one running normaliser shared by `world` ranks of n envs
 * each (the Welford/Chan merge across ranks):
 *   rlp_reward_norm_stats  writes this rank's chunk statistics, the first
 *                          rlp_reward_norm_parts(T, n) doubles of `work`;
 *   (the caller all-gathers those doubles of every rank into `parts`, rank-major)
 *   rlp_reward_norm_finish merges, per time step, all world * chunks in global env order, runs
 *                          the running-statistics recurrence with world * n rewards per step and
 *                          normalises this rank's rewards.
 * Every rank then holds the same rms, and the result equals one rank of world * n envs bit for
 * bit when n is a multiple of 4096. world = 1 with parts = work is rlp_reward_norm. */
int64_t rlp_reward_norm_parts(int T, int n);
int rlp_reward_norm_stats(const float *reward_in, int T, int n, double *work, rlp_stream_t stream);
int rlp_reward_norm_finish(const float *reward_in, int T, int n, int world, const double *parts,
                           double *rms, double *work, float *reward_out, rlp_stream_t stream);

/* GAE(lambda) backward scan per env (Proximal_Policy_Optimization2.py:93-98), fp32 in the
 * reference's exact operation order (bit-identical to the NumPy-2 loop):
 *   delta = (r + ((float)gamma * (1 - success)) * v_next) - v
 *   gae   = delta + ((float)(gamma*lambda) * gae) * (1 - done)
 *   adv = gae; v_target = adv + v
 * All arrays [T][n]. adv_stats (device f64, nullable; at least 3 * rlp_adv_stats_parts(n) + 2):
 * overwritten with one (count, mean, M2) partial per 256-env block, f64, computed without atomics
 * (per-lane shifted sums, a fixed-order Chan combine): run-to-run deterministic. */
int rlp_adv_stats_parts(int n);
int rlp_gae(const float *reward, const float *value, const float *value_next, const uint8_t *done,
            const uint8_t *success, double gamma, double lambda, int T, int n, float *adv,
            float *v_target, double *adv_stats, rlp_stream_t stream);

/* rlp_reward_norm + rlp_gae without the normalised-reward array: reward_raw is the rollout's
 * reward and reward_work the `work` of a preceding rlp_reward_norm_statistics over it; each
 * reward is normalised as it is loaded, with the same expression as rlp_reward_norm, so adv /
 * v_target / the partials are bit-identical to rlp_reward_norm followed by rlp_gae. */
int rlp_gae_normalized(const float *reward_raw, const double *reward_work, const float *value,
                       const float *value_next, const uint8_t *done, const uint8_t *success,
                       double gamma, double lambda, int T, int n, float *adv, float *v_target,
                       double *adv_stats, rlp_stream_t stream);

/* adv = (adv - mean) / (std_unbiased + 1e-5) (Trick 1, :99-100; torch's two-pass std over the
 * whole buffer), mean / std from the first `parts` partials of adv_stats combined in a fixed
 * order (Chan); they are written to adv_stats[3 * parts], [3 * parts + 1]. Under data-parallel
 * ranks, all-gather every rank's partials (rank-major) and pass parts = world * parts: the
 * normalisation is then global and identical on every rank. */
int rlp_adv_normalize(float *adv, int64_t count, double *adv_stats, int parts, rlp_stream_t stream);

/* ------------------------------------------------------------------------------------------ */
/* PPO2 update (Proximal_Policy_Optimization2.learn, algorithm/policy_base/
 * Proximal_Policy_Optimization2.py:102-163) for the drivers' [S -> 256 -> 256 -> A] tanh nets
 * (PPOActor_Gaussian / PPOCritic, demonstration/PPO2/PPO2-4-CartPole/train.py:39-125) with
 * S <= 8 (CartPole, AngleOnly, SOI, UGV, UAV) or 41 <= S <= 44 (the obstacle-avoidance demos'
 * 4 + 37 lidar inputs, demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/train.py:48-50,95-97).
 * For S <= 8 layer 1 runs inside the two kernels; for 41..44 inputs it runs on exact-f32 MFMA
 * kernels of its own (h1 = tanh(W1 s + b1) stored once per call, dW1 | db1 from the stored
 * dL/dh1 and h1), which needs contiguous rows: `index` must be NULL (RLP_EINVAL otherwise; the
 * caller gathers a mini-batch first) and the workspace grows by 2 x rows x 256 floats (h1 and
 * dL/dh1) plus the dW1 partials (rlp_ppo2_workspace_floats includes them).
 * rlp_ppo2_grad writes the gradient of ONE optimiser step's loss over `rows` samples, in the
 * flat torch parameter order (W1, b1, W2, b2, W3, b3 = rlp_mlp_forward's layout):
 *   RLP_LOSS_ACTOR:  mean(-min(r*adv, clamp(r, 1-eps, 1+eps)*adv) - entropy_coef * entropy),
 *                    r = exp(sum_a logN(a; mu(s), std) - sum_a a_logprob)  (:141-148; std is a
 *                    constant, so the entropy term has no parameter gradient)
 *   RLP_LOSS_CRITIC: mean((v_target - V(s))^2)  (:155-156)
 * `index` (nullable) gathers the rows of a mini-batch (:110-111 BatchSampler); `loss_sum` (+=)
 * receives the summed per-row loss (divide by rows for the reported loss), summed from per-wave
 * partials in a fixed order (gradient and loss run-to-run identical). `packed` is
 * rlp_mfma_pack(params). The hidden-layer GEMMs use the f16x3 split (RLP_MLP_F16X3 accuracy),
 * the weight-gradient GEMMs exact f32 MFMA. `workspace` holds rlp_ppo2_workspace_floats(). */
#define RLP_LOSS_ACTOR 0
#define RLP_LOSS_CRITIC 1
typedef struct rlp_ppo2_loss_cfg {
    int32_t kind;            /* RLP_LOSS_ACTOR | RLP_LOSS_CRITIC */
    float eps_clip;          /* ppo_msg['eps_clip'] */
    float entropy_coef;      /* ppo_msg['entropy_coef'] */
    float std[4];            /* actor.std per action dim */
    float a_min[4], a_max[4];/* actor.a_min / a_max (mean = tanh(.) * gain + off) */
} rlp_ppo2_loss_cfg;
int64_t rlp_ppo2_workspace_floats(const rlp_mlp_desc *desc, int64_t rows);
int rlp_ppo2_grad(const rlp_mlp_desc *desc, const float *packed, const rlp_ppo2_loss_cfg *cfg,
                  const float *s, const float *a, const float *a_logprob, const float *adv,
                  const float *v_target, const int64_t *index, int64_t rows, float *grad,
                  double *loss_sum, float *workspace, rlp_stream_t stream);

/* The same gradient for any tanh Linear stack that rlp_ppo2_grad does not take (other widths, more
 * or fewer hidden layers, more inputs): the PPO2-SecondOrderIntegration demo's actor
 * 4 -> 128 -> 64 -> 32 -> A / critic 4 -> 64 -> 64 -> 1 (demonstration/PPO2/PPO2-4-
 * SecondOrderIntegration/train.py:37-125); also the exact-f32 alternative for nets that
 * rlp_ppo2_grad takes (the obstacle-avoidance demos' 41 -> 256 -> 256 -> A go to rlp_ppo2_grad
 * under the Python learner's 'auto' selection since round 5; update_kernels='dense' keeps them
 * here). rlp_ppo2_grad has no arithmetic knob: its hidden layer is always the f16x3 split, and
 * this entry point is the per-call exact-f32 choice. Hidden layers
 * tanh; the actor's last layer tanh (A <= 4), the critic's linear with one output; widths <= 1024.
 * `params` is the plain layout (rlp_mlp_param_count floats, torch order); rows are contiguous (a
 * mini-batch is gathered by the caller). Exact f32 MFMA products (v_mfma_f32_16x16x4_f32),
 * activations and the weight gradients' partials in `workspace`
 * (rlp_ppo2_dense_workspace_floats), fixed summation order (run-to-run identical). The SOI demo's
 * two shapes (<= 8 inputs; hidden 128-64-32 or 64-64; <= 4 outputs) run as ONE fused per-row launch
 * (forward, loss head, backward, weight-gradient partials with every activation in LDS) and two
 * fixed-order sums; other three- and four-layer nets with <= 64 inputs and hidden widths
 * 32k <= 256 run each 2^18-row chunk as five launches (forward chain, loss head, backward chain,
 * every layer's weight gradient, one reduce); other stacks one GEMM launch per layer and pass. The
 * loss is summed from per-block partials in a fixed order too (gradient and loss_sum run-to-run
 * identical). */
int64_t rlp_ppo2_dense_workspace_floats(const rlp_mlp_desc *desc, int64_t rows);
int rlp_ppo2_dense_grad(const rlp_mlp_desc *desc, const float *params, const rlp_ppo2_loss_cfg *cfg,
                        const float *s, const float *a, const float *a_logprob, const float *adv,
                        const float *v_target, int64_t rows, float *grad, double *loss_sum,
                        float *workspace, rlp_stream_t stream);

/* out[0] += sum(grad^2) (torch.nn.utils.clip_grad_norm_'s total norm, squared), accumulated in
 * double in a fixed order: bit-identical on every run and every data-parallel rank. */
int rlp_grad_sqnorm(const float *grad, int64_t n, double *out, rlp_stream_t stream);
/* grad *= min(1, max_norm / (sqrt(*sqnorm) + 1e-6)) in place — clip_grad_norm_ on a gradient
 * buffer that persists (the DPPO2 Worker's local grads,
 * demonstration/DPPO2/DPPO2-4-CartPole/Distributed_PPO2.py:88-91, 99-102). */
int rlp_grad_clip(float *grad, int64_t n, const double *sqnorm, float max_norm,
                  rlp_stream_t stream);
/* torch.optim.Adam step (exp_avg.lerp_, exp_avg_sq.mul_.addcmul_, bias corrections, addcdiv).
 * With clip_sqnorm != NULL the gradient is first scaled by min(1, max_norm / (sqrt(*clip_sqnorm)
 * + 1e-6)) (clip_grad_norm_, :150-151), evaluated on the device. */
typedef struct rlp_adam_cfg {
    float lr, beta1, beta2, eps, max_norm;
    int32_t step;            /* 1-based step count after this update (bias corrections) */
} rlp_adam_cfg;
int rlp_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                  const rlp_adam_cfg *cfg, const double *clip_sqnorm, rlp_stream_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Replay buffer resident in HBM (utils/classes.py:189-247 ReplayBuffer; DDPG.learn
 * algorithm/actor_critic/DDPG.py:72-109). Device columns of `capacity` rows, fp32:
 * s [cap][S], a [cap][A], r [cap], s_next [cap][S], end [cap] (= 1 - done, :209). */
typedef struct rlp_replay {
    float *s, *a, *r, *s_next, *end;
    int64_t capacity;
    int32_t S, A;
} rlp_replay;
/* store_transition (:201-210) of n transitions in order: row (counter + i) % capacity (the
 * caller advances its mem_counter by n). reward is the env's f64 reward. */
int rlp_replay_store(const rlp_replay *rb, int64_t counter, const float *s, const float *a,
                     const double *reward, const float *s_next, const uint8_t *done, int64_t n,
                     rlp_stream_t stream);
/* sample_buffer(is_reward_ascent=False) (:236-237): `batch` row indices uniform in
 * [0, max_mem) with replacement, Philox-keyed by (seed, counter). */
int rlp_replay_sample_uniform(int64_t max_mem, int64_t batch, uint64_t seed, uint64_t counter,
                              int64_t *index, rlp_stream_t stream);
/* sample_buffer(is_reward_ascent=True) (:212-235): rows sorted by reward ascending (stable),
 * pool = the top int(0.25 * max_mem), *n_out = min(pool, batch) rows drawn without replacement
 * in random order. Device workspace of rlp_replay_workspace_bytes(max_mem) bytes. */
int64_t rlp_replay_workspace_bytes(int64_t capacity);
int rlp_replay_sample_reward_top(const rlp_replay *rb, int64_t max_mem, int64_t batch,
                                 uint64_t seed, uint64_t counter, int64_t *index, int64_t *n_out,
                                 void *workspace, int64_t workspace_bytes, rlp_stream_t stream);
/* rows index[0..batch) of every column into dense [batch][..] tensors */
int rlp_replay_gather(const rlp_replay *rb, const int64_t *index, int64_t batch, float *s,
                      float *a, float *r, float *s_next, float *end, rlp_stream_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Native DDPG update (algorithm/actor_critic/DDPG.py:72-109 learn() body, :111-118 soft update)
 * for the drivers' ReLU nets (demonstration/DDPG/DDPG-4-{SecondOrderIntegration,...}/train.py:26-100): actor
 * S -> ... -> A with relu hidden layers and a = gain * tanh(z) + off; critic cat(s, a) -> ... -> 1
 * with relu hidden layers. Replaces the torch autograd + torch.optim.Adam sequence of one learn()
 * iteration on a sampled batch (s, a, r, s', end = 1 - done):
 *   y = r + gamma * end * Q'(s', mu'(s'));  critic: MSE(y, Q(s, a)) -> grad -> Adam;
 *   actor: -mean(Q(s, mu(s))) with the UPDATED critic -> grad -> Adam;  soft target updates.
 * Every product runs on v_mfma_f32_16x16x4_f32 (f32 products and accumulation); weight gradients
 * are reduced in a fixed order (run-to-run identical). A net is a flat fp32 parameter buffer in
 * module.parameters() order: layer l's W [out][in] at offset[l], its b [out] right after it;
 * parameters the chain does not use (e.g. the drivers' critic.action_value) may sit in between —
 * their gradient entries must be zero (Adam then leaves them unchanged, as torch skips them) and
 * the soft update still blends them, as torch does. */
#define RLP_DENSE_MAX_LAYERS 4
typedef struct rlp_dense_net {
    int32_t n_layers;                          /* Linear layers in the forward chain */
    int32_t dims[RLP_DENSE_MAX_LAYERS + 1];    /* dims[0] inputs ... dims[n_layers] outputs */
    int64_t offset[RLP_DENSE_MAX_LAYERS];      /* of layer l's W in params (floats) */
    int64_t n_params;                          /* length of params (and of its grad / Adam state) */
    float *params;
} rlp_dense_net;
typedef struct rlp_ddpg_nets {
    rlp_dense_net actor, target_actor, critic, target_critic;  /* targets: the nets' layouts */
    float *actor_grad, *actor_m, *actor_v;      /* [actor.n_params]: gradient, Adam exp_avg(_sq) */
    float *critic_grad, *critic_m, *critic_v;   /* [critic.n_params] */
    int32_t *steps;            /* device [2]: Adam step counts (actor, critic), +1 per update */
    const float *gain, *off;   /* device [A]: the actor's output affine */
} rlp_ddpg_nets;
typedef struct rlp_ddpg_cfg {
    int32_t batch;
    float gamma, actor_tau, critic_tau;
    rlp_adam_cfg actor_adam, critic_adam;   /* lr, beta1, beta2, eps (max_norm and step unused) */
} rlp_ddpg_cfg;
/* device workspace (floats) of rlp_ddpg_update for this net shape and batch */
int64_t rlp_ddpg_workspace(const rlp_ddpg_nets *nets, int batch);
/* one update; s [B][S], a [B][A], r [B], s_next [B][S], end [B] device fp32 (the replay gather's
 * output); losses (device [2]) = critic MSE, actor loss. Graph-capturable (all state on the
 * device). */
int rlp_ddpg_update(const rlp_ddpg_nets *nets, const rlp_ddpg_cfg *cfg, const float *s,
                    const float *a, const float *r, const float *s_next, const float *end,
                    float *work, float *losses, rlp_stream_t stream);

/* Native SAC update (algorithm/actor_critic/Soft_Actor_Critic.py:70-129 learn() body) for the
 * SAC drivers' nets (utils/classes.py SACActor / SACCritic): actor trunk S -> ... -> H with relu
 * after every layer, heads mean [A][H] and log_std [A][H] (log_std clamped to [ls_lo, ls_hi],
 * std = exp, a = tanh(mean + std * eps) * gain + off, log_pi with the tanh-squash correction);
 * twin critic chains cat(s, a) -> ... -> 1 (relu hidden layers) in ONE parameter buffer, and the
 * target critic in the same layout. One iteration on a sampled batch (s, a, r, s', dw):
 *   target_Q = r + gamma * (1 - dw) * (min(Q1', Q2')(s', a') - alpha * log_pi')  (a' ~ pi(s'))
 *   actor: mean(alpha * log_pi - min(Q1, Q2)(s, a~pi(s))) -> grad -> Adam
 *   critic: MSE(Q1(s, a), target_Q) + MSE(Q2(s, a), target_Q) -> grad -> Adam
 *   alpha (adaptive): -mean(exp(log_alpha) * (log_pi + target_entropy)) -> grad -> Adam
 *   soft update target = tau * critic + (1 - tau) * target.
 * Noise: `noise` [2][B][A] (eps for s', then for s: the reference's two rsample calls in order) or
 * NULL for Philox draws keyed by (seed, *counter, row + (d + 1) * 2^40) for draw d (0: s', 1: s) —
 * a stream disjoint from rlp_sac_sample's exploration draws, which key env ids < 2^40 — with
 * *counter advanced per update on the device (graph-capturable). */
typedef struct rlp_sac_nets {
    rlp_dense_net actor;       /* the trunk layers (relu after each); params = the actor's buffer */
    int64_t mean_offset;       /* mean head W [A][H] (b follows) in actor.params */
    int64_t log_std_offset;    /* log_std head W [A][H] (b follows) */
    int32_t action_dim;
    rlp_dense_net q1, q2;      /* critic chains; params = the critic's buffer (n_params = its length) */
    float *target_critic;      /* target critic params, the critic's layout */
    float *actor_grad, *actor_m, *actor_v;     /* [actor.n_params] */
    float *critic_grad, *critic_m, *critic_v;  /* [q1.n_params] */
    float *log_alpha, *alpha_grad, *alpha_m, *alpha_v;   /* device [1] each */
    int32_t *steps;            /* device [3]: Adam step counts (actor, critic, alpha), +1 per update */
    uint64_t *counter;         /* device [1]: Philox counter of the noise, +1 per update */
    const float *gain, *off, *ls_lo, *ls_hi;   /* device [A] */
} rlp_sac_nets;
typedef struct rlp_sac_cfg {
    int32_t batch, adaptive_alpha;
    float gamma, tau, target_entropy, alpha;   /* alpha: the fixed temperature when not adaptive */
    uint64_t seed;
    rlp_adam_cfg actor_adam, critic_adam, alpha_adam;
} rlp_sac_cfg;
int64_t rlp_sac_workspace(const rlp_sac_nets *nets, int batch);
/* losses (device [2]) = critic loss, actor loss */
int rlp_sac_update(const rlp_sac_nets *nets, const rlp_sac_cfg *cfg, const float *s, const float *a,
                   const float *r, const float *s_next, const float *dw, const float *noise,
                   float *work, float *losses, rlp_stream_t stream);

/* ------------------------------------------------------------------------------------------ */
const char *rlp_last_error_string(void);
int rlp_abi_version(void);
/* sizeof of the ABI structs as compiled into the library (0 cartpole, 1 angleonly, 2 soi, 3 ugv,
 * 4 uav, 5 mlp_desc, 6 rollout_cfg, 7 rollout_bufs, 8 ppo2_loss_cfg, 9 adam_cfg, 10 replay,
 * 11 ugv_oa, 12 dense_net, 13 ddpg_nets, 14 ddpg_cfg, 15 sac_nets, 16 sac_cfg): FFI bindings
 * verify their mirrors with it. */
int64_t rlp_struct_size(int which);
/* Test hook of the launch-status plumbing: runs the dense GEMM launcher with `nprobs` problems,
 * which must be outside its accepted range [1, 6], through a call chain that drops the launcher's
 * return value (as the DDPG / SAC / PPO2-dense chains do), and returns the status that reaches the
 * C-ABI (RLP_EINVAL; never RLP_OK). No device work. */
int rlp_selftest_gemm_guard(int nprobs);

/* The rlp_set_* knobs below are process-wide defaults (plain globals, not synchronised): set them
 * before any thread launches work. Concurrent callers choose per call instead, through
 * rlp_rollout_cfg's mlp_precision / physics / sub fields and the mlp_precision argument of
 * rlp_mfma_forward / rlp_value_fixup (rlp_ppo2_grad and the other entry points have no knob).
 *
 * Tuning knob of rlp_rollout: 16-env sub-blocks per wave: 0 = auto (default; the f16x3 path
 * takes 1 when 2 would leave fewer than two blocks per CU, e.g. 32 768 UAV envs), 1 (f16x3 only),
 * 2 or 4. */
int rlp_set_rollout_sub(int sub);
/* Tuning knob of rlp_rollout (f16x3 path): -1 = auto (default: 3 when the envs fill every CU with
 * a 256-env block, else — and always for RLP_ENV_UAV_HOVER_OUTER_LOOP — 5), 3 = one 8-wave block
 * of 32-env waves per CU (2 waves per SIMD), 5 = one 4-wave block of 32-env waves per CU (1 wave
 * per SIMD, VGPR + AGPR budget), 1 = two 4-wave blocks per CU (the block's env state in LDS, each
 * step's f64 physics on full 64-lane waves; the kernel for rlp_set_rollout_sub 1), 0 = the
 * register-resident kernel (physics on the 16*sub lanes of each env's own wave; the RLP_MLP_FP32
 * path's kernel). 2, 4 and 6 (measured-slower variants of earlier releases) return RLP_EINVAL.
 * Same results. */
int rlp_set_rollout_physics(int shared);
/* Arithmetic of rlp_rollout's hidden layer (the [256 x 256] GEMM, 99 % of its FLOPs):
 *   RLP_MLP_F16X3 (default): error-compensated split, w*x = wh*xh + wh*xl + wl*xh on f16 MFMA with
 *     f32 accumulation — fp32-class accuracy (see tests/test_gpu_rollout.py) at 16/3 x the f32
 *     MFMA rate;
 *   RLP_MLP_FP32: exact f32-input MFMA (v_mfma_f32_16x16x4_f32).
 * It is the default of rlp_rollout (cfg mlp_precision 0) and of rlp_mfma_forward / rlp_value_fixup
 * (mlp_precision 0); rlp_mlp_forward is always fp32. */
#define RLP_MLP_FP32 0
#define RLP_MLP_F16X3 1
int rlp_set_mlp_precision(int mode);
int rlp_get_mlp_precision(void);

#ifdef __cplusplus
}
#endif
#endif /* RLP_H_ */
