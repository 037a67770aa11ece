// rlp_lidar.hip — UGVForwardObstacleAvoidance step / observe with the fake lidar cast one beam per
// lane (get_fake_laser environment/UGVForwardObstacleAvoidance/
// UGVForwardObstacleAvoidance.py:274-397).
//
// A block owns EB envs. Phase 1 (one lane per env): f64 RK4 step, terminal flag, reward, the
// per-pose lidar setup (beam angles, the four corner angles, collision, each obstacle's distance)
// into LDS. Phase 2 (every lane): the EB x 37 (env, beam) pairs are spread over the block; a beam
// reads its env's pose and obstacles from LDS (lanes of one env read the same words: broadcast)
// and writes one float of obs[env][4 + beam]. One env per lane would hold 45 obstacle doubles in
// VGPRs (1 wave / SIMD, scratch spills) and leave most of the chip idle at 16 K envs; a beam per
// lane keeps ~40 VGPRs of live state and launches 37x the lanes. The arithmetic of each beam is
// Env<7>::beam — the same code the generic kernels run, restating the reference line by line.
#include "rlp_lidar.hpp"

namespace rlp {

constexpr int kOaThreads = 256;

template <int EB>
struct OaLds {
    OaEnvLds e[EB];
};

template <int EB>
__device__ __forceinline__ void oa_scan(const OA::P &p, const OaLds<EB> &L, int e0, int ne,
                                        float *__restrict__ obs) {
    for (int it = threadIdx.x; it < ne * OA::NL; it += kOaThreads) {
        const int e = it / OA::NL, i = it - e * OA::NL;
        obs[(size_t)(e0 + e) * OA::S + 4 + i] = oa_beam(p, L.e[e], i);
    }
}

// STEP: step_update (+ obs_cur if requested); !STEP: get_state only
// !STEP with `keep` (the rollout's next observation): a block none of whose envs was reset
// (keep[i] == 0 for all) copies its rows of `prev` (the step's obs_next — the driver's
// current_state = next_state) instead of scanning again
template <int EB, bool STEP>
__global__ void __launch_bounds__(kOaThreads) oa_kernel(OA::P p, double *state, int n,
                                                        const float *__restrict__ action,
                                                        float *obs_cur, float *obs_next,
                                                        double *reward, int32_t *flag,
                                                        uint8_t *done, const uint8_t *keep,
                                                        const float *prev) {
    __shared__ OaLds<EB> L;
    const int t = threadIdx.x;
    const int e0 = blockIdx.x * EB;
    const int ne = n - e0 < EB ? n - e0 : EB;
    const bool own = t < ne;
    const size_t i = (size_t)e0 + t;
    if (!STEP && keep) {
        if (!__syncthreads_or(own && keep[i])) {
            for (int k = t; k < ne * OA::S; k += kOaThreads)
                obs_next[(size_t)e0 * OA::S + k] = prev[(size_t)e0 * OA::S + k];
            return;
        }
    }
    double s[OA::DW];
    if (own) {
#pragma unroll
        for (int d = 0; d < OA::DW; ++d) s[d] = state[(size_t)d * n + i];
        for (int k = 0; k < p.n_obs; ++k) {
            L.e[t].ob[k].x0 = state[(size_t)(OA::OB + 3 * k) * n + i];
            L.e[t].ob[k].y0 = state[(size_t)(OA::OB + 3 * k + 1) * n + i];
            L.e[t].ob[k].r0 = state[(size_t)(OA::OB + 3 * k + 2) * n + i];
        }
    }
    float *first = STEP ? obs_cur : obs_next;
    if (first) {  // scan at the current pose (get_state / step's current_state)
        if (own) {
            oa_setup(p, L.e[t], s);
            oa_head(p, s, first + i * OA::S);
        }
        __syncthreads();
        oa_scan(p, L, e0, ne, first);
        if (!STEP) return;
        __syncthreads();
    }
    if (STEP) {
        if (own) {
            const float a[2] = {action[i * 2], action[i * 2 + 1]};
            double r, e, eph;
            int f;
            bool dn;
            OA::step_core(p, s, a, [&](double x, double y) {
                return OA::collision_at(p, x, y, [&](int k, double &x0, double &y0, double &r0) {
                    x0 = L.e[t].ob[k].x0; y0 = L.e[t].ob[k].y0; r0 = L.e[t].ob[k].r0;
                });
            }, r, f, dn, e, eph);
#pragma unroll
            for (int d = 0; d < OA::DW; ++d) state[(size_t)d * n + i] = s[d];
            reward[i] = r;
            flag[i] = f;
            done[i] = dn ? 1 : 0;
            oa_setup(p, L.e[t], s);
            float h[4];
            OA::obs_head(p, s, e, eph, h);
#pragma unroll
            for (int j = 0; j < 4; ++j) obs_next[i * OA::S + j] = h[j];
        }
        __syncthreads();
        oa_scan(p, L, e0, ne, obs_next);
    }
}

template <bool STEP>
static int launch_oa(const OA::P &p, double *state, int n, const float *action, float *obs_cur,
                     float *obs_next, double *reward, int32_t *flag, uint8_t *done, hipStream_t st,
                     const uint8_t *keep = nullptr, const float *prev = nullptr) {
    if (p.n_obs < 0 || p.n_obs > OA::NOBS)
        return fail(RLP_EINVAL, "UGVForwardObstacleAvoidance: n_obs=%d (0..%d)", p.n_obs, OA::NOBS);
    // fewer envs per block when the batch is small, so every CU gets several blocks
    if ((n + 63) / 64 >= 4 * device_cus())
        oa_kernel<64, STEP><<<(n + 63) / 64, kOaThreads, 0, st>>>(p, state, n, action, obs_cur,
                                                                 obs_next, reward, flag, done, keep,
                                                                 prev);
    else
        oa_kernel<16, STEP><<<(n + 15) / 16, kOaThreads, 0, st>>>(p, state, n, action, obs_cur,
                                                                 obs_next, reward, flag, done, keep,
                                                                 prev);
    RLP_CHECK_LAUNCH("UGVForwardObstacleAvoidance lidar");
    return RLP_OK;
}

int launch_ugvoa_step(const rlp_ugv_oa_params &p, double *state, int n, const float *action,
                      float *obs_cur, float *obs_next, double *reward, int32_t *flag,
                      uint8_t *done, hipStream_t st) {
    return launch_oa<true>(p, state, n, action, obs_cur, obs_next, reward, flag, done, st);
}

int launch_ugvoa_observe(const rlp_ugv_oa_params &p, const double *state, int n, float *obs,
                         hipStream_t st) {
    return launch_oa<false>(p, const_cast<double *>(state), n, nullptr, nullptr, obs, nullptr,
                            nullptr, nullptr, st);
}

// the rollout's next observation: envs reset this step (reset[i]) scanned, blocks without one
// copy the step's obs_next
int launch_ugvoa_observe_after(const rlp_ugv_oa_params &p, const double *state, int n, float *obs,
                               const uint8_t *reset, const float *obs_next, hipStream_t st) {
    return launch_oa<false>(p, const_cast<double *>(state), n, nullptr, nullptr, obs, nullptr,
                            nullptr, nullptr, st, reset, obs_next);
}

// reset(random=True) with one wave per env (oa_reset_wave); obs (nullable): also the reset env's
// observation — the rollout's next observation of the envs it resets
constexpr int kOaResetWaves = 4;

__global__ void __launch_bounds__(64 * kOaResetWaves) oa_reset_kernel(
    OA::P p, double *state, int n, const uint8_t *mask, const double *init, uint64_t seed,
    uint64_t counter, uint64_t env_id0, float *obs) {
    __shared__ double obl[kOaResetWaves][OA::NOBS * 3];
    __shared__ OaEnvLds L[kOaResetWaves];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int e = blockIdx.x * kOaResetWaves + w;
    if (e >= n || (mask && !mask[e])) return;  // uniform per wave
    const size_t i = (size_t)e;
    if (init) {
        for (int d = lane; d < OA::D; d += 64) state[(size_t)d * n + i] = init[(size_t)d * n + i];
        return;
    }
    oa_reset_wave(p, state, n, i, seed, counter, env_id0 + (uint64_t)e,
                  obs ? obs + i * OA::S : nullptr, obl[w], L[w]);
}

int launch_ugvoa_reset(const rlp_ugv_oa_params &p, double *state, int n, const uint8_t *mask,
                       const double *init, uint64_t seed, uint64_t counter, uint64_t env_id0,
                       hipStream_t st, float *obs) {
    if (p.n_obs < 0 || p.n_obs > OA::NOBS || p.max_tries < 0 || p.max_tries > 65535)
        return fail(RLP_EINVAL, "rlp_env_reset: n_obs=%d (0..%d) max_tries=%d (0..65535)", p.n_obs,
                    OA::NOBS, p.max_tries);
    oa_reset_kernel<<<(n + kOaResetWaves - 1) / kOaResetWaves, 64 * kOaResetWaves, 0, st>>>(
        p, state, n, mask, init, seed, counter, env_id0, init ? nullptr : obs);
    RLP_CHECK_LAUNCH("rlp_env_reset (UGVForwardObstacleAvoidance)");
    return RLP_OK;
}

}  // namespace rlp
