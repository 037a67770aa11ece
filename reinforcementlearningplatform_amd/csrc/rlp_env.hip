// rlp_env.hip — batched env step / observe / reset kernels and the shared C-ABI plumbing.
//
// Layout: physics state f64 SoA [D][n] (one env per lane => every component load/store is a
// coalesced 512 B wave access); actions/observations f32 env-major [n][A] / [n][S].
// Roofline: HBM-bound for every kind except CartPole (whose 10-11 RK4 sub-steps with fp64
// sincos make it VALU-bound); per-env bytes and FLOPs are listed in DESIGN.md.
#include <stdarg.h>
#include <stdio.h>

#include <type_traits>

#include "rlp_envs.hpp"

namespace rlp {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

// first refusal of a launch helper since the last take_pending() (thread-local, like g_err)
static thread_local int g_pending = RLP_OK;

int fail_pending(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    if (g_pending == RLP_OK) g_pending = code;
    return code;
}

int take_pending() {
    const int c = g_pending;
    g_pending = RLP_OK;
    return c;
}

// (the UAV step at 234 registers runs 2 waves per SIMD; compiled for 3 or 4 (168 / 128
// registers, 204 / 416 B of spills) it took 764 / 1088 us against 528 us per 4M-env launch,
// profiles/r6/r6l_learn_side_ab.txt)
template <int KIND>
__global__ void __launch_bounds__(256) env_step_kernel(typename Env<KIND>::P p, double *state,
                                                       int n, const float *__restrict__ action,
                                                       float *obs_cur, float *obs_next,
                                                       double *reward, int32_t *flag,
                                                       uint8_t *done) {
    using E = Env<KIND>;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s[E::D];
#pragma unroll
    for (int d = 0; d < E::D; ++d) s[d] = state[(size_t)d * n + i];
    float a[E::A], on[E::S];
#pragma unroll
    for (int j = 0; j < E::A; ++j) a[j] = action[(size_t)i * E::A + j];
    if (obs_cur) {
        float oc[E::S];
        E::observe(p, s, oc);
#pragma unroll
        for (int j = 0; j < E::S; ++j) obs_cur[(size_t)i * E::S + j] = oc[j];
    }
    double r;
    int f;
    bool dn;
    // p as the kernarg segment's first argument (not the by-value copy): Env steps that re-read
    // their parameters per phase (phase_ref) then load them from there instead of a stack copy
    const auto &pk = *(const typename E::P *)(const __attribute__((address_space(4))) typename E::P *)
        __builtin_amdgcn_kernarg_segment_ptr();
    E::step(pk, s, a, on, r, f, dn);
#pragma unroll
    for (int d = 0; d < EnvDW<E>::value; ++d) state[(size_t)d * n + i] = s[d];
#pragma unroll
    for (int j = 0; j < E::S; ++j) obs_next[(size_t)i * E::S + j] = on[j];
    reward[i] = r;
    flag[i] = f;
    done[i] = dn ? 1 : 0;
}

template <int KIND>
__global__ void __launch_bounds__(256) env_observe_kernel(typename Env<KIND>::P p,
                                                          const double *state, int n, float *obs) {
    using E = Env<KIND>;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s[E::D];
#pragma unroll
    for (int d = 0; d < E::D; ++d) s[d] = state[(size_t)d * n + i];
    float o[E::S];
    E::observe(p, s, o);
#pragma unroll
    for (int j = 0; j < E::S; ++j) obs[(size_t)i * E::S + j] = o[j];
}

template <int KIND>
__global__ void __launch_bounds__(256) env_reset_kernel(typename Env<KIND>::P p, double *state,
                                                        int n, const uint8_t *mask,
                                                        const double *init, uint64_t seed,
                                                        uint64_t counter, uint64_t env_id0) {
    using E = Env<KIND>;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mask && !mask[i]) return;
    if (init) {
#pragma unroll
        for (int d = 0; d < E::D; ++d) state[(size_t)d * n + i] = init[(size_t)d * n + i];
        return;
    }
    double s[E::D];
#pragma unroll
    for (int d = 0; d < E::D; ++d) s[d] = state[(size_t)d * n + i];
    E::reset(p, s, seed, counter, env_id0 + (uint64_t)i);
#pragma unroll
    for (int d = 0; d < E::D; ++d) state[(size_t)d * n + i] = s[d];
}

// UGVForwardObstacleAvoidance step / observe: rlp_lidar.hip
int launch_ugvoa_step(const rlp_ugv_oa_params &p, double *state, int n, const float *action,
                      float *obs_cur, float *obs_next, double *reward, int32_t *flag,
                      uint8_t *done, hipStream_t st);
int launch_ugvoa_observe(const rlp_ugv_oa_params &p, const double *state, int n, float *obs,
                         hipStream_t st);
int launch_ugvoa_reset(const rlp_ugv_oa_params &p, double *state, int n, const uint8_t *mask,
                       const double *init, uint64_t seed, uint64_t counter, uint64_t env_id0,
                       hipStream_t st, float *obs = nullptr);

// kind -> template dispatch
template <typename F>
int dispatch_kind(int kind, F &&f) {
    switch (kind) {
    case RLP_ENV_CARTPOLE: return f(std::integral_constant<int, RLP_ENV_CARTPOLE>());
    case RLP_ENV_CARTPOLE_ANGLEONLY: return f(std::integral_constant<int, RLP_ENV_CARTPOLE_ANGLEONLY>());
    case RLP_ENV_SOI: return f(std::integral_constant<int, RLP_ENV_SOI>());
    case RLP_ENV_UGV_FORWARD: return f(std::integral_constant<int, RLP_ENV_UGV_FORWARD>());
    case RLP_ENV_UGV_BIDIRECTIONAL: return f(std::integral_constant<int, RLP_ENV_UGV_BIDIRECTIONAL>());
    case RLP_ENV_UAV_HOVER_OUTER_LOOP: return f(std::integral_constant<int, RLP_ENV_UAV_HOVER_OUTER_LOOP>());
    case RLP_ENV_UGV_OBSTACLE_AVOIDANCE: return f(std::integral_constant<int, RLP_ENV_UGV_OBSTACLE_AVOIDANCE>());
    }
    return fail(RLP_EINVAL, "unknown env kind %d", kind);
}

}  // namespace rlp

using namespace rlp;

extern "C" {

const char *rlp_last_error_string(void) { return g_err; }
int rlp_abi_version(void) { return RLP_ABI_VERSION; }

int rlp_env_dims(int kind, int *D, int *S, int *A) {
    return dispatch_kind(kind, [&](auto k) {
        using E = Env<decltype(k)::value>;
        if (D) *D = E::D;
        if (S) *S = E::S;
        if (A) *A = E::A;
        return RLP_OK;
    });
}

// sizes of the ABI structs as compiled here (the Python mirror checks against them)
int64_t rlp_struct_size(int which) {
    switch (which) {
    case 0: return sizeof(rlp_cartpole_params);
    case 1: return sizeof(rlp_angleonly_params);
    case 2: return sizeof(rlp_soi_params);
    case 3: return sizeof(rlp_ugv_params);
    case 4: return sizeof(rlp_uav_hover_params);
    case 5: return sizeof(rlp_mlp_desc);
    case 6: return sizeof(rlp_rollout_cfg);
    case 7: return sizeof(rlp_rollout_bufs);
    case 8: return sizeof(rlp_ppo2_loss_cfg);
    case 9: return sizeof(rlp_adam_cfg);
    case 10: return sizeof(rlp_replay);
    case 11: return sizeof(rlp_ugv_oa_params);
    case 12: return sizeof(rlp_dense_net);
    case 13: return sizeof(rlp_ddpg_nets);
    case 14: return sizeof(rlp_ddpg_cfg);
    case 15: return sizeof(rlp_sac_nets);
    case 16: return sizeof(rlp_sac_cfg);
    }
    return -1;
}

int rlp_env_step(int kind, const void *params, double *state, int n, const float *action,
                 float *obs_cur, float *obs_next, double *reward, int32_t *flag, uint8_t *done,
                 rlp_stream_t stream) {
    RLP_REQUIRE(params && state && action && obs_next && reward && flag && done,
                "rlp_env_step: null argument");
    RLP_REQUIRE(n >= 0, "rlp_env_step: n < 0");
    if (n == 0) return RLP_OK;
    return dispatch_kind(kind, [&](auto k) {
        constexpr int K = decltype(k)::value;
        const auto &p = *static_cast<const typename Env<K>::P *>(params);
        if constexpr (K == RLP_ENV_UGV_OBSTACLE_AVOIDANCE) {  // beam-per-lane lidar kernel
            return launch_ugvoa_step(p, state, n, action, obs_cur, obs_next, reward, flag, done,
                                     as_stream(stream));
        } else {
            env_step_kernel<K><<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(
                p, state, n, action, obs_cur, obs_next, reward, flag, done);
            RLP_CHECK_LAUNCH("rlp_env_step");
            return RLP_OK;
        }
    });
}

int rlp_env_observe(int kind, const void *params, const double *state, int n, float *obs,
                    rlp_stream_t stream) {
    RLP_REQUIRE(params && state && obs, "rlp_env_observe: null argument");
    RLP_REQUIRE(n >= 0, "rlp_env_observe: n < 0");
    if (n == 0) return RLP_OK;
    return dispatch_kind(kind, [&](auto k) {
        constexpr int K = decltype(k)::value;
        const auto &p = *static_cast<const typename Env<K>::P *>(params);
        if constexpr (K == RLP_ENV_UGV_OBSTACLE_AVOIDANCE) {
            return launch_ugvoa_observe(p, state, n, obs, as_stream(stream));
        } else {
            env_observe_kernel<K><<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(p, state, n, obs);
            RLP_CHECK_LAUNCH("rlp_env_observe");
            return RLP_OK;
        }
    });
}

int rlp_env_reset(int kind, const void *params, double *state, int n, const uint8_t *mask,
                  const double *init_state, uint64_t seed, uint64_t counter, uint64_t env_id0,
                  rlp_stream_t stream) {
    RLP_REQUIRE(params && state, "rlp_env_reset: null argument");
    RLP_REQUIRE(n >= 0, "rlp_env_reset: n < 0");
    if (n == 0) return RLP_OK;
    return dispatch_kind(kind, [&](auto k) {
        constexpr int K = decltype(k)::value;
        const auto &p = *static_cast<const typename Env<K>::P *>(params);
        if constexpr (K == RLP_ENV_UGV_OBSTACLE_AVOIDANCE) {  // wave-per-env map generator
            return launch_ugvoa_reset(p, state, n, mask, init_state, seed, counter, env_id0,
                                      as_stream(stream));
        } else {
            env_reset_kernel<K><<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(
                p, state, n, mask, init_state, seed, counter, env_id0);
            RLP_CHECK_LAUNCH("rlp_env_reset");
            return RLP_OK;
        }
    });
}

}  // extern "C"
