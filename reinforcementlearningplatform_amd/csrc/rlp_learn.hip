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

// ---- reward normalisation -----------------------------------------------------------------
// Three launches: (1) chunk statistics — a [P x T] grid of 256-thread blocks, each two-pass over
// a 4096-reward chunk of one time step held in registers (16 per lane, one HBM read, fp64
// sums); (2) one block: per time step the chunks' (mean, M2) combined in chunk order (Chan),
// then the running-statistics recurrence over t (the merge weights n/(cnt+n), cnt*n/(cnt+n)
// depend only on the count and are computed in parallel; the serial chain is a few fp64 ops per
// step, staged through LDS), then std_t = sqrt(S_t / cnt_t) in parallel; (3) the elementwise
// normalisation. Workspace layout (rlp_reward_norm_workspace): part [T][P][2] | agg [T][2] |
// out [T][2] (mean_t, std_t after step t's merge).
constexpr int kRsChunk = 4096, kRsPer = kRsChunk / 256, kRsTile = 512;

__host__ __device__ inline int rs_chunks(int n) { return (n + kRsChunk - 1) / kRsChunk; }

__global__ void __launch_bounds__(256) reward_stats_kernel(const float *__restrict__ r, int n,
                                                           double *__restrict__ part) {
    __shared__ double red[4];
    const int p = blockIdx.x, t = blockIdx.y, P = gridDim.x;
    const int lo = p * kRsChunk, cnt = min(kRsChunk, n - lo);
    const float *x = r + (size_t)t * n + lo;
    float v[kRsPer];
    double s = 0;
#pragma unroll
    for (int j = 0; j < kRsPer; ++j) {
        const int i = j * 256 + threadIdx.x;
        v[j] = i < cnt ? x[i] : 0.f;
        s += (double)v[j];
    }
    const double mean = block_sum<256>(s, red) / cnt;
    double q = 0;
#pragma unroll
    for (int j = 0; j < kRsPer; ++j) {
        const double d = (double)v[j] - mean;
        if (j * 256 + (int)threadIdx.x < cnt) q += d * d;
    }
    const double m2 = block_sum<256>(q, red);
    if (threadIdx.x == 0) {
        part[((size_t)t * P + p) * 2 + 0] = mean;
        part[((size_t)t * P + p) * 2 + 1] = m2;
    }
}

// sequential merge over t (RunningMeanStd.update, utils/classes.py:626-645): Welford for n == 1
// (the reference exactly, first-call std = x quirk included), Chan's parallel merge otherwise
__global__ void __launch_bounds__(256) reward_merge_kernel(const float *__restrict__ r, int T, int n,
                                                           double *rms, double *work) {
    __shared__ double sa[kRsTile], sb[kRsTile], sw1[kRsTile], sw2[kRsTile];
    __shared__ double carry[4];
    const int P = rs_chunks(n);
    double *part = work, *agg = work + (size_t)T * P * 2, *out = agg + (size_t)T * 2;
    if (threadIdx.x == 0)
        for (int k = 0; k < 4; ++k) carry[k] = rms[k];
    if (n > 1) {  // per time step: combine the chunks in chunk order
        for (int t = threadIdx.x; t < T; t += 256) {
            const double *pp = part + (size_t)t * P * 2;
            double c = min(kRsChunk, n), mean = pp[0], m2 = pp[1];
            for (int p = 1; p < P; ++p) {
                const double cb = min(kRsChunk, n - p * kRsChunk), nn = c + cb;
                const double dl = pp[2 * p] - mean;
                mean = mean + dl * (cb / nn);
                m2 = m2 + pp[2 * p + 1] + dl * dl * (c * cb / nn);
                c = nn;
            }
            agg[2 * t] = mean;
            agg[2 * t + 1] = m2;
        }
    }
    __syncthreads();
    for (int t0 = 0; t0 < T; t0 += kRsTile) {
        const int tn = min(kRsTile, T - t0);
        const double cnt0 = carry[0];
        for (int j = threadIdx.x; j < tn; j += 256) {
            const int t = t0 + j;
            if (n == 1) {
                sa[j] = (double)r[t];
            } else {  // the merge weights need only the running count (cnt0 + j n)
                sa[j] = agg[2 * t];
                sb[j] = agg[2 * t + 1];
                const double cnt = cnt0 + (double)j * n, nn = cnt + n;
                sw1[j] = (double)n / nn;
                sw2[j] = cnt * (double)n / nn;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double cnt = carry[0], mean = carry[1], S = carry[2], sd = carry[3];
            for (int j = 0; j < tn; ++j) {
                if (n == 1) {
                    const double x = sa[j];
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
                    sb[j] = sd;
                } else {
                    if (cnt == 0) {
                        mean = sa[j]; S = sb[j];
                    } else {
                        const double dl = sa[j] - mean;
                        mean = mean + dl * sw1[j];
                        S = S + sb[j] + dl * dl * sw2[j];
                    }
                    cnt += n;
                    sb[j] = S;
                }
                sa[j] = mean;
            }
            if (n > 1 && tn > 0) sd = sqrt(S / cnt);
            carry[0] = cnt; carry[1] = mean; carry[2] = S; carry[3] = sd;
        }
        __syncthreads();
        for (int j = threadIdx.x; j < tn; j += 256) {
            const int t = t0 + j;
            out[2 * t] = sa[j];
            out[2 * t + 1] = n == 1 ? sb[j] : sqrt(sb[j] / (cnt0 + (double)(j + 1) * n));
        }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int k = 0; k < 4; ++k) rms[k] = carry[k];
}

__global__ void __launch_bounds__(256) reward_apply_kernel(const float *__restrict__ r, int T,
                                                           int n, const double *__restrict__ out_t,
                                                           float *__restrict__ out) {
    const size_t total = (size_t)T * n;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
        const int t = (int)(i / n);
        out[i] = (float)(((double)r[i] - out_t[2 * t]) / (out_t[2 * t + 1] + 1e-8));
    }
}

// GAE backward scan, one env per lane; coalesced [T][n] rows. The recurrence is serial in t, so
// each lane's loads are issued kGaeU steps ahead of the arithmetic (registers), which is what
// keeps HBM busy with only n / 64 waves in the grid.
constexpr int kGaeU = 16;
__global__ void __launch_bounds__(256) gae_kernel(const float *__restrict__ r,
                                                  const float *__restrict__ v,
                                                  const float *__restrict__ vn,
                                                  const uint8_t *__restrict__ done,
                                                  const uint8_t *__restrict__ success, float g32,
                                                  float c, int T, int n, float *__restrict__ adv,
                                                  float *__restrict__ vt, double *stats) {
    __shared__ double red[4];
    const int i = blockIdx.x * 256 + threadIdx.x;
    double s1 = 0, s2 = 0;
    if (i < n) {
        float gae = 0.f;
        for (int t1 = T; t1 > 0; t1 -= kGaeU) {
            const int u = min(kGaeU, t1);
            float rr[kGaeU], vv[kGaeU], vx[kGaeU];
            uint8_t dd[kGaeU], ss[kGaeU];
#pragma unroll
            for (int j = 0; j < kGaeU; ++j) {
                if (j < u) {
                    const size_t k = (size_t)(t1 - 1 - j) * n + i;
                    rr[j] = r[k]; vv[j] = v[k]; vx[j] = vn[k]; dd[j] = done[k]; ss[j] = success[k];
                }
            }
#pragma unroll
            for (int j = 0; j < kGaeU; ++j) {
                if (j < u) {
                    const size_t k = (size_t)(t1 - 1 - j) * n + i;
                    const float one_s = 1.0f - (float)ss[j];
                    float delta = rr[j] + (g32 * one_s) * vx[j];
                    delta = delta - vv[j];
                    float tt = c * gae;
                    tt = tt * (1.0f - (float)dd[j]);
                    gae = delta + tt;
                    adv[k] = gae;
                    vt[k] = gae + vv[j];
                    s1 += (double)gae;
                    s2 += (double)gae * (double)gae;
                }
            }
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

int64_t rlp_reward_norm_workspace(int T, int n) {
    if (T < 0 || n < 0) return RLP_EINVAL;
    return (int64_t)T * (2 * (int64_t)rs_chunks(n > 0 ? n : 1) + 4);
}

int rlp_reward_norm(const float *reward_in, int T, int n, double *rms, double *work,
                    float *reward_out, rlp_stream_t stream) {
    RLP_REQUIRE(reward_in && rms && work && reward_out, "rlp_reward_norm: null argument");
    RLP_REQUIRE(T >= 0 && n >= 0, "rlp_reward_norm: T=%d n=%d", T, n);
    if (T == 0 || n == 0) return RLP_OK;
    hipStream_t s = as_stream(stream);
    const int P = rs_chunks(n);
    if (n > 1) reward_stats_kernel<<<dim3(P, T), 256, 0, s>>>(reward_in, n, work);
    reward_merge_kernel<<<1, 256, 0, s>>>(reward_in, T, n, rms, work);
    const size_t total = (size_t)T * n;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    reward_apply_kernel<<<blocks, 256, 0, s>>>(reward_in, T, n, work + (size_t)T * P * 2 + (size_t)T * 2,
                                               reward_out);
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
