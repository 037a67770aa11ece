// rlp_learn.hip — learn-side scans over a [T][n] rollout (HBM-bound, one env per lane):
//   reward normalisation   utils/classes.py:626-656 (Normalization / RunningMeanStd)
//   GAE(lambda)            algorithm/policy_base/Proximal_Policy_Optimization2.py:88-98
//   advantage norm         Proximal_Policy_Optimization2.py:99-100
// Built with -ffp-contract=off: the GAE recurrence reproduces the reference's NumPy-2 fp32 loop
// bit for bit.
#include "rlp_common.hpp"

namespace rlp {

__device__ __forceinline__ double warp_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <int BS>
__device__ __forceinline__ double block_sum(double v, double *red) {
    v = warp_sum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) red[w] = v;
    __syncthreads();
    double s = 0;
#pragma unroll
    for (int i = 0; i < BS / 64; ++i) s += red[i];
    __syncthreads();
    return s;
}

// per time step t: (mean_b, M2_b) of the n rewards, fp64 two-pass (the row is L2-resident)
__global__ void __launch_bounds__(256) reward_stats_kernel(const float *__restrict__ r, int n,
                                                           double *work) {
    __shared__ double red[4];
    const int t = blockIdx.x;
    const float *x = r + (size_t)t * n;
    double s = 0;
    for (int i = threadIdx.x; i < n; i += 256) s += (double)x[i];
    const double mean = block_sum<256>(s, red) / n;
    double q = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
        const double d = (double)x[i] - mean;
        q += d * d;
    }
    const double m2 = block_sum<256>(q, red);
    if (threadIdx.x == 0) {
        work[3 * t + 0] = mean;
        work[3 * t + 1] = m2;
    }
}

// sequential merge over t (RunningMeanStd.update, Welford for n == 1, Chan otherwise);
// writes (mean_t, std_t) after step t's merge into work[3t], work[3t+1]
__global__ void reward_merge_kernel(const float *__restrict__ r, int T, int n, double *rms,
                                    double *work) {
    double cnt = rms[0], mean = rms[1], S = rms[2], sd = rms[3];
    for (int t = 0; t < T; ++t) {
        if (n == 1) {
            const double x = (double)r[t];
            cnt += 1;
            if (cnt == 1) {
                mean = x;
                sd = x;  // reference quirk: std = x on the first sample
            } else {
                const double old = mean;
                mean = old + (x - old) / cnt;
                S = S + (x - old) * (x - mean);
                sd = sqrt(S / cnt);
            }
        } else {
            const double mb = work[3 * t], Sb = work[3 * t + 1];
            if (cnt == 0) {
                cnt = n; mean = mb; S = Sb;
            } else {
                const double nn = cnt + n;
                const double dl = mb - mean;
                mean = mean + dl * ((double)n / nn);
                S = S + Sb + dl * dl * (cnt * (double)n / nn);
                cnt = nn;
            }
            sd = sqrt(S / cnt);
        }
        work[3 * t] = mean;
        work[3 * t + 1] = sd;
    }
    rms[0] = cnt; rms[1] = mean; rms[2] = S; rms[3] = sd;
}

__global__ void __launch_bounds__(256) reward_apply_kernel(const float *__restrict__ r, int T,
                                                           int n, const double *work, float *out) {
    const size_t total = (size_t)T * n;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
        const int t = (int)(i / n);
        out[i] = (float)(((double)r[i] - work[3 * t]) / (work[3 * t + 1] + 1e-8));
    }
}

// GAE backward scan, one env per lane; coalesced [T][n] rows
__global__ void __launch_bounds__(256) gae_kernel(const float *__restrict__ r,
                                                  const float *__restrict__ v,
                                                  const float *__restrict__ vn,
                                                  const uint8_t *__restrict__ done,
                                                  const uint8_t *__restrict__ success, float g32,
                                                  float c, int T, int n, float *adv, float *vt,
                                                  double *stats) {
    __shared__ double red[4];
    const int i = blockIdx.x * 256 + threadIdx.x;
    double s1 = 0, s2 = 0;
    if (i < n) {
        float gae = 0.f;
        for (int t = T - 1; t >= 0; --t) {
            const size_t k = (size_t)t * n + i;
            const float one_s = 1.0f - (float)success[k];
            float delta = r[k] + (g32 * one_s) * vn[k];
            delta = delta - v[k];
            float tt = c * gae;
            tt = tt * (1.0f - (float)done[k]);
            gae = delta + tt;
            adv[k] = gae;
            vt[k] = gae + v[k];
            s1 += (double)gae;
            s2 += (double)gae * (double)gae;
        }
    }
    if (stats) {
        s1 = block_sum<256>(s1, red);
        s2 = block_sum<256>(s2, red);
        if (threadIdx.x == 0) {
            atomicAdd(&stats[0], s1);
            atomicAdd(&stats[1], s2);
        }
    }
}

__global__ void __launch_bounds__(256) adv_norm_kernel(float *adv, int64_t count,
                                                       const double *stats) {
    const double N = (double)count;
    const double mean = stats[0] / N;
    const double var = (stats[1] - stats[0] * stats[0] / N) / (N - 1);
    const float m32 = (float)mean;
    const float den = (float)sqrt(var > 0 ? var : 0) + 1e-5f;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < count; i += (int64_t)gridDim.x * 256)
        adv[i] = (adv[i] - m32) / den;
}

}  // namespace rlp

using namespace rlp;

extern "C" {

int rlp_reward_norm(const float *reward_in, int T, int n, double *rms, double *work,
                    float *reward_out, rlp_stream_t stream) {
    RLP_REQUIRE(reward_in && rms && work && reward_out, "rlp_reward_norm: null argument");
    RLP_REQUIRE(T >= 0 && n >= 0, "rlp_reward_norm: T=%d n=%d", T, n);
    if (T == 0 || n == 0) return RLP_OK;
    hipStream_t s = as_stream(stream);
    if (n > 1) reward_stats_kernel<<<T, 256, 0, s>>>(reward_in, n, work);
    reward_merge_kernel<<<1, 1, 0, s>>>(reward_in, T, n, rms, work);
    const size_t total = (size_t)T * n;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    reward_apply_kernel<<<blocks, 256, 0, s>>>(reward_in, T, n, work, reward_out);
    RLP_CHECK_LAUNCH("rlp_reward_norm");
    return RLP_OK;
}

int rlp_gae(const float *reward, const float *value, const float *value_next, const uint8_t *done,
            const uint8_t *success, double gamma, double lambda, int T, int n, float *adv,
            float *v_target, double *adv_stats, rlp_stream_t stream) {
    RLP_REQUIRE(reward && value && value_next && done && success && adv && v_target,
                "rlp_gae: null argument");
    RLP_REQUIRE(T >= 0 && n >= 0, "rlp_gae: T=%d n=%d", T, n);
    if (T == 0 || n == 0) return RLP_OK;
    const float g32 = (float)gamma;       // torch: gamma * (1 - success) in fp32
    const float c = (float)(gamma * lambda);  // numpy: (gamma * lmd) * gae, NEP-50 fp32
    gae_kernel<<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(reward, value, value_next, done,
                                                               success, g32, c, T, n, adv,
                                                               v_target, adv_stats);
    RLP_CHECK_LAUNCH("rlp_gae");
    return RLP_OK;
}

int rlp_adv_normalize(float *adv, int64_t count, const double *adv_stats, rlp_stream_t stream) {
    RLP_REQUIRE(adv && adv_stats, "rlp_adv_normalize: null argument");
    if (count <= 1) return RLP_OK;
    const int64_t b = (count + 255) / 256;
    adv_norm_kernel<<<(int)(b < 4096 ? b : 4096), 256, 0, as_stream(stream)>>>(adv, count, adv_stats);
    RLP_CHECK_LAUNCH("rlp_adv_normalize");
    return RLP_OK;
}

}  // extern "C"
