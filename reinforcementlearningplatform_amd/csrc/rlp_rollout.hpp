// rlp_rollout.hpp — definitions shared by the fused rollout (rlp_rollout.hip) and the lidar env's
// rollout (rlp_rollout_oa.hip, its own translation unit: built without MachineLICM, see Makefile).
#pragma once
#include "rlp_envs.hpp"
#include "rlp_lidar.hpp"
#include "rlp_mfma_layout.hpp"
#include "rlp_mfma_x3.hpp"

namespace rlp {

// UGVForwardObstacleAvoidance lidar step / observe / reset (rlp_lidar.hip)
int launch_ugvoa_step(const rlp_ugv_oa_params &p, double *state, int n, const float *action,
                      float *obs_cur, float *obs_next, double *reward, int32_t *flag,
                      uint8_t *done, hipStream_t st);
int launch_ugvoa_observe(const rlp_ugv_oa_params &p, const double *state, int n, float *obs,
                         hipStream_t st);
int launch_ugvoa_observe_after(const rlp_ugv_oa_params &p, const double *state, int n, float *obs,
                               const uint8_t *reset, const float *obs_next, hipStream_t st);
int launch_ugvoa_reset(const rlp_ugv_oa_params &p, double *state, int n, const uint8_t *mask,
                       const double *init, uint64_t seed, uint64_t counter, uint64_t env_id0,
                       hipStream_t st, float *obs = nullptr);

// Each wave stages only its own envs' observations in LDS, so a wave-level fence suffices; no
// block barrier keeps the two waves of a SIMD in lockstep (one's f64 physics overlaps the other's
// MFMAs).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct RolloutArgs {
    int T, n;
    uint64_t seed, step0, env_id0;
    int success_rule, success_flag;
    float std_[4], a_min[4], a_max[4], gain[4], off[4];
    float log_std[4], half_inv_var[4];  // launch constants of the Normal log-prob
};

// Normal(mean, std).log_prob(x) in torch's expression, with log(std) and 1 / (2 var) per launch
__device__ __forceinline__ float normal_logp_c(float x, float mean, float half_inv_var, float log_std) {
    const float d = x - mean;
    return -(d * d) * half_inv_var - log_std - 0.91893853320467274178f;
}

constexpr int RING = 3;  // fp32 path: W2 k-phases in flight per wave

// the UGVForwardObstacleAvoidance rollout (rlp_rollout_oa.hip), called by rlp_rollout
int rollout_oa(const void *params, double *state, uint8_t *need_reset, const float *actor,
               const MfmaNet &an, const float *critic, const MfmaNet &cn, const RolloutArgs &ra,
               const rlp_rollout_bufs &b, int prec, void *workspace, int64_t workspace_bytes,
               hipStream_t s);
int64_t rollout_oa_workspace_bytes();

}  // namespace rlp
