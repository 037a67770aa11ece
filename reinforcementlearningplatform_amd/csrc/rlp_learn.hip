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

// (count, mean, M2) of two disjoint sets, Chan et al.'s pairwise combine
struct Moments {
    double c, m, q;
};
__device__ __forceinline__ Moments chan(Moments a, Moments b) {
    if (b.c == 0) return a;
    if (a.c == 0) return b;
    const double nn = a.c + b.c, d = b.m - a.m;
    return {nn, a.m + d * (b.c / nn), a.q + b.q + d * d * (a.c * b.c / nn)};
}

// fixed-order block combine: xor butterfly inside each wave (every lane's operands are fixed by
// the data, so lane 0's result is run-independent), then waves 0, 1, 2, 3 in order
template <int BS>
__device__ __forceinline__ Moments block_moments(Moments v, Moments *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        Moments u{__shfl_xor(v.c, o), __shfl_xor(v.m, o), __shfl_xor(v.q, o)};
        v = (threadIdx.x & o) ? chan(u, v) : chan(v, u);
    }
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) red[w] = v;
    __syncthreads();
    Moments s = red[0];
#pragma unroll
    for (int i = 1; i < BS / 64; ++i) s = chan(s, red[i]);
    __syncthreads();
    return s;
}

// ---- reward normalisation -----------------------------------------------------------------
// Three launches: (1) chunk statistics — a [P x T] grid of 256-thread blocks, each two-pass over
// a 4096-reward chunk of one time step held in registers (16 per lane as four 16-byte loads when
// the rows are 16-byte aligned, one HBM read, fp64 sums); (2) one block: per time step the
// chunks' (mean, M2) combined in chunk order (Chan), then the running statistics over t as a
// block-wide inclusive scan of Chan merges (each thread folds two time steps, a shuffle scan in
// each wave, the four wave totals through LDS; fixed order, so run-independent), 512 steps per
// tile with the carry between tiles; the single-env case keeps the reference's serial Welford
// recurrence (first-call std = x quirk); (3) the elementwise normalisation on a [chunks x T] grid
// (the time step is the block row: no per-element index division). Workspace layout
// (rlp_reward_norm_workspace): part [T][P][2] | agg [T][2] | out [T][2] (mean_t, std_t after
// step t's merge).
__host__ inline bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

constexpr int kRsChunk = 4096, kRsPer = kRsChunk / 256, kRsTile = 512;

__host__ __device__ inline int rs_chunks(int n) { return (n + kRsChunk - 1) / kRsChunk; }

template <bool VEC>
__global__ void __launch_bounds__(256) reward_stats_kernel(const float *__restrict__ r, int T, int n,
                                                           double *__restrict__ part) {
    __shared__ double red[4];
    const int p = blockIdx.x, P = gridDim.x;
    const int lo = p * kRsChunk, cnt = min(kRsChunk, n - lo);
    for (int t = blockIdx.y; t < T; t += gridDim.y) {
        const float *x = r + (size_t)t * n + lo;
        float v[kRsPer];
        if (VEC) {  // lane owns 4 consecutive rewards per 1024-reward slice; cnt % 4 == 0
#pragma unroll
            for (int j = 0; j < kRsPer / 4; ++j) {
                const int i = (j * 256 + (int)threadIdx.x) * 4;
                const float4 q = i < cnt ? *(const float4 *)(x + i) : make_float4(0.f, 0.f, 0.f, 0.f);
                v[4 * j] = q.x; v[4 * j + 1] = q.y; v[4 * j + 2] = q.z; v[4 * j + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < kRsPer; ++j) {
                const int i = j * 256 + threadIdx.x;
                v[j] = i < cnt ? x[i] : 0.f;
            }
        }
        double s = 0;
#pragma unroll
        for (int j = 0; j < kRsPer; ++j) s += (double)v[j];
        const double mean = block_sum<256>(s, red) / cnt;
        double q = 0;
#pragma unroll
        for (int j = 0; j < kRsPer; ++j) {
            const int i = VEC ? (j / 4 * 256 + (int)threadIdx.x) * 4 + (j & 3) : j * 256 + threadIdx.x;
            const double d = (double)v[j] - mean;
            if (i < cnt) q += d * d;
        }
        const double m2 = block_sum<256>(q, red);
        if (threadIdx.x == 0) {
            part[((size_t)t * P + p) * 2 + 0] = mean;
            part[((size_t)t * P + p) * 2 + 1] = m2;
        }
    }
}

// time step t's chunk statistics of `world` ranks (rank-major [world][T][P][2]) combined in global
// env order -> (mean, M2) of its world * n rewards (one thread; loads kRsPre ahead of the combine)
__device__ __forceinline__ void rs_step_merge(const double *parts, int T, int n, int world, int t,
                                              double &mean, double &m2) {
    constexpr int kRsPre = 16;  // one round of loads for n <= 65536 (P <= 16 chunks)
    const int P = rs_chunks(n), Q = world * P;
    double c = 0;
    mean = 0;
    m2 = 0;
    for (int q0 = 0; q0 < Q; q0 += kRsPre) {
        double pm[kRsPre], pq[kRsPre];
#pragma unroll
        for (int u = 0; u < kRsPre; ++u) {
            const int q = q0 + u, rk = q / P, p = q - rk * P;
            const double *pp = parts + (((size_t)rk * T + t) * P + p) * 2;
            pm[u] = q < Q ? pp[0] : 0.0;
            pq[u] = q < Q ? pp[1] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kRsPre; ++u) {
            const int q = q0 + u, p = q % P;
            if (q >= Q) break;
            const double cb = min(kRsChunk, n - p * kRsChunk);
            if (q == 0) {
                c = cb; mean = pm[u]; m2 = pq[u];
                continue;
            }
            const double nn = c + cb;
            const double dl = pm[u] - mean;
            mean = mean + dl * (cb / nn);
            m2 = m2 + pq[u] + dl * dl * (c * cb / nn);
            c = nn;
        }
    }
}

// the running statistics over t (whole block, 256 threads): a block-wide inclusive scan of Chan
// merges of the per-step aggregates agg [T][2] (world * n rewards each) onto rms; writes step t's
// (mean_t, std_t) to out [T][2] and the final statistics to rms
__device__ __forceinline__ void rs_running_scan(const double *agg, int T, double ntot, double *rms,
                                                double *out) {
    __shared__ Moments wred[4];
    __shared__ double carry[4];
    if (threadIdx.x == 0)
        for (int k = 0; k < 4; ++k) carry[k] = rms[k];
    __syncthreads();
    Moments cr{carry[0], carry[1], carry[2]};
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    auto ag = [&](int i) { return agg[i]; };
    for (int t0 = 0; t0 < T; t0 += kRsTile) {
        const int ta = t0 + 2 * (int)threadIdx.x, tb = ta + 1;
        const Moments e0 = ta < T ? Moments{ntot, ag(2 * ta), ag(2 * ta + 1)} : Moments{0, 0, 0};
        const Moments e1 = tb < T ? Moments{ntot, ag(2 * tb), ag(2 * tb + 1)} : Moments{0, 0, 0};
        Moments v = chan(e0, e1);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {  // inclusive scan inside the wave
            const Moments u{__shfl_up(v.c, o), __shfl_up(v.m, o), __shfl_up(v.q, o)};
            if (l >= o) v = chan(u, v);
        }
        Moments ex{__shfl_up(v.c, 1), __shfl_up(v.m, 1), __shfl_up(v.q, 1)};
        if (l == 0) ex = Moments{0, 0, 0};
        if (l == 63) wred[w] = v;
        __syncthreads();
        Moments base = cr;
        for (int i = 0; i < w; ++i) base = chan(base, wred[i]);
        base = chan(base, ex);
        Moments tot = cr;
#pragma unroll
        for (int i = 0; i < 4; ++i) tot = chan(tot, wred[i]);
        __syncthreads();
        const Moments s0 = chan(base, e0), s1 = chan(s0, e1);
        if (ta < T) {
            out[2 * ta] = s0.m;
            out[2 * ta + 1] = sqrt(s0.q / s0.c);
        }
        if (tb < T) {
            out[2 * tb] = s1.m;
            out[2 * tb + 1] = sqrt(s1.q / s1.c);
        }
        cr = tot;
    }
    if (threadIdx.x == 0) {
        rms[0] = cr.c; rms[1] = cr.m; rms[2] = cr.q;
        rms[3] = T > 0 ? sqrt(cr.q / cr.c) : carry[3];
    }
}

// Welford for a single env (the reference exactly, first-call std = x quirk included, serial),
// Chan's parallel merge otherwise (utils/classes.py:626-645 RunningMeanStd.update). `parts` holds
// the chunk statistics of `world` ranks of n envs each, rank-major ([world][T][P][2]); per time
// step the world * P chunks are combined in global env order, so W ranks of n envs reproduce one
// rank of W * n envs bit for bit (when n is a multiple of the chunk).
__global__ void __launch_bounds__(256) reward_merge_kernel(const float *__restrict__ r, int T, int n,
                                                           int world, const double *parts,
                                                           double *rms, double *work) {
    __shared__ double sa[kRsTile], sb[kRsTile];
    __shared__ double carry[4];
    const int P = rs_chunks(n);
    double *agg = work + (size_t)T * P * 2, *out = agg + (size_t)T * 2;
    const double ntot = (double)n * world;
    if (ntot == 1) {  // the reference's own shape: one reward per step, serial Welford
        if (threadIdx.x == 0)
            for (int k = 0; k < 4; ++k) carry[k] = rms[k];
        __syncthreads();
        for (int t0 = 0; t0 < T; t0 += kRsTile) {
            const int tn = min(kRsTile, T - t0);
            for (int j = threadIdx.x; j < tn; j += 256) sa[j] = (double)r[t0 + j];
            __syncthreads();
            if (threadIdx.x == 0) {
                double cnt = carry[0], mean = carry[1], S = carry[2], sd = carry[3];
                for (int j = 0; j < tn; ++j) {
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
                    sa[j] = mean;
                    sb[j] = sd;
                }
                carry[0] = cnt; carry[1] = mean; carry[2] = S; carry[3] = sd;
            }
            __syncthreads();
            for (int j = threadIdx.x; j < tn; j += 256) {
                out[2 * (t0 + j)] = sa[j];
                out[2 * (t0 + j) + 1] = sb[j];
            }
            __syncthreads();
        }
        if (threadIdx.x == 0)
            for (int k = 0; k < 4; ++k) rms[k] = carry[k];
        return;
    }
    for (int t = threadIdx.x; t < T; t += 256) {
        double mean, m2;
        rs_step_merge(parts, T, n, world, t, mean, m2);
        agg[2 * t] = mean;
        agg[2 * t + 1] = m2;
    }
    __syncthreads();
    rs_running_scan(agg, T, ntot, rms, out);
}

// [chunks x T] grid: the block row is the time step, so the per-step (mean, std) are two scalar
// loads and no element index is divided; 4 rewards per lane as 16-byte accesses when aligned
template <bool VEC>
__global__ void __launch_bounds__(256) reward_apply_kernel(const float *__restrict__ r, int T,
                                                           int n, const double *__restrict__ out_t,
                                                           float *__restrict__ out) {
    for (int t = blockIdx.y; t < T; t += gridDim.y) {
        const double m = out_t[2 * t], den = out_t[2 * t + 1] + 1e-8;
        const float *x = r + (size_t)t * n;
        float *y = out + (size_t)t * n;
        if (VEC) {
            for (int i = (blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += gridDim.x * 1024) {
                const float4 q = *(const float4 *)(x + i);
                float4 o;
                o.x = (float)(((double)q.x - m) / den);
                o.y = (float)(((double)q.y - m) / den);
                o.z = (float)(((double)q.z - m) / den);
                o.w = (float)(((double)q.w - m) / den);
                *(float4 *)(y + i) = o;
            }
        } else {
            for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
                y[i] = (float)(((double)x[i] - m) / den);
        }
    }
}

// the partials combined in a fixed order by one 256-thread block: thread j folds parts
// [j*per, (j+1)*per) left to right, then the block combine; (mean, unbiased std) after the partials
__global__ void __launch_bounds__(256) adv_stats_merge_kernel(double *stats, int parts) {
    __shared__ Moments red[4];
    const int per = (parts + 255) / 256, lo = threadIdx.x * per, hi = min(parts, lo + per);
    Moments a{0, 0, 0};
    for (int j = lo; j < hi; ++j) a = chan(a, Moments{stats[3 * j], stats[3 * j + 1], stats[3 * j + 2]});
    a = block_moments<256>(a, red);
    if (threadIdx.x == 0) {
        stats[3 * parts] = a.m;
        stats[3 * parts + 1] = a.c > 1 ? sqrt(a.q / (a.c - 1)) : 0.0;
    }
}

// GAE backward scan, one env per lane; coalesced [T][n] rows. The recurrence is serial in t, so
// each lane's loads are issued kGaeU steps ahead of the arithmetic (registers), which is what
// keeps HBM busy with only n / 64 waves in the grid.
// NORM: r is the raw reward and rs [T][2] step t's (mean_t, std_t) of rlp_reward_norm_statistics:
// the reward is normalised as it is loaded, (float)((r - mean_t) / (std_t + 1e-8)) — the apply
// pass's expression, so the normalised-reward array is neither written nor re-read.
// (Round 6 also tried merging the advantage partials in the grid's last block, and the reward
// statistics' per-step merges and scan in the last blocks of the statistics launch, handing over
// through atomic counters: the agent-scope release fence each block then needs writes back its
// XCD's L2, and GAE went 31 -> 54 us, the statistics 17 -> 76 us (profiles/r6/r6l_learn_side_ab.txt).)
constexpr int kGaeU = 16;
constexpr int kGaeLdsSteps = 512;  // NORM = 1: the per-step statistics staged in LDS (T <= this)
template <int NORM>  // 0: r normalised already; 1: raw r, statistics from LDS; 2: from global
__global__ void __launch_bounds__(256) gae_kernel(const float *__restrict__ r,
                                                  const double *__restrict__ rs,
                                                  const float *__restrict__ v,
                                                  const float *__restrict__ vn,
                                                  const uint8_t *__restrict__ done,
                                                  const uint8_t *__restrict__ success, float g32,
                                                  float c, int T, int n, float *__restrict__ adv,
                                                  float *__restrict__ vt, double *stats) {
    __shared__ Moments red[4];
    __shared__ __attribute__((aligned(16))) double srs[NORM == 1 ? 2 * kGaeLdsSteps : 2];
    if (NORM == 1) {  // (uniform per step: one LDS broadcast read instead of registers per step)
        for (int j = threadIdx.x; j < 2 * T; j += 256) srs[j] = rs[j];
        __syncthreads();
    }
    const double *st = NORM == 1 ? srs : rs;
    const int i = blockIdx.x * 256 + threadIdx.x;
    double s1 = 0, s2 = 0, k0 = 0;  // sums of (adv - k0), k0 = the lane's first advantage
    if (i < n) {
        float gae = 0.f;
        for (int t1 = T; t1 > 0; t1 -= kGaeU) {
            const int u = min(kGaeU, t1);
            float rr[kGaeU], vv[kGaeU], vx[kGaeU];
            uint8_t dd[kGaeU], ss[kGaeU];
            double2 ms[NORM ? kGaeU : 1];  // step t's (mean_t, std_t), read with the rows
#pragma unroll
            for (int j = 0; j < kGaeU; ++j) {
                if (j < u) {
                    const size_t k = (size_t)(t1 - 1 - j) * n + i;
                    rr[j] = r[k]; vv[j] = v[k]; vx[j] = vn[k]; dd[j] = done[k]; ss[j] = success[k];
                    if (NORM) ms[j] = *reinterpret_cast<const double2 *>(st + 2 * (t1 - 1 - j));
                }
            }
            if (NORM) {  // the chunk's rewards normalised before the recurrence (independent: ILP)
#pragma unroll
                for (int j = 0; j < kGaeU; ++j)
                    if (j < u) rr[j] = (float)(((double)rr[j] - ms[j].x) / (ms[j].y + 1e-8));
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
                    if (t1 == T && j == 0) k0 = (double)gae;
                    const double d = (double)gae - k0;
                    s1 += d;
                    s2 += d * d;
                }
            }
        }
    }
    if (stats) {  // this block's (count, mean, M2): shifted sums per lane, Chan across lanes
        Moments mo{0, 0, 0};
        if (i < n) {
            const double c = (double)T;
            mo = {c, k0 + s1 / c, fmax(s2 - s1 * (s1 / c), 0.0)};
        }
        mo = block_moments<256>(mo, red);
        if (threadIdx.x == 0) {
            stats[3 * blockIdx.x + 0] = mo.c;
            stats[3 * blockIdx.x + 1] = mo.m;
            stats[3 * blockIdx.x + 2] = mo.q;
        }
    }
}

// 4 advantages per lane as one 16-byte access (the tail of count % 4 by the first lanes) when
// adv is 16-byte aligned
template <bool VEC>
__global__ void __launch_bounds__(256) adv_norm_kernel(float *adv, int64_t count,
                                                       const double *mean_std) {
    const float m32 = (float)mean_std[0];
    const float den = (float)mean_std[1] + 1e-5f;
    if (VEC) {
        const int64_t c4 = count >> 2;
        float4 *a4 = (float4 *)adv;
        for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < c4; i += (int64_t)gridDim.x * 256) {
            float4 q = a4[i];
            q.x = (q.x - m32) / den;
            q.y = (q.y - m32) / den;
            q.z = (q.z - m32) / den;
            q.w = (q.w - m32) / den;
            a4[i] = q;
        }
        const int64_t i = 4 * c4 + blockIdx.x * 256 + threadIdx.x;
        if (i < count) adv[i] = (adv[i] - m32) / den;
    } else {
        for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < count; i += (int64_t)gridDim.x * 256)
            adv[i] = (adv[i] - m32) / den;
    }
}

}  // namespace rlp

using namespace rlp;

extern "C" {

int64_t rlp_reward_norm_workspace(int T, int n) {
    if (T < 0 || n < 0) return RLP_EINVAL;
    return (int64_t)T * (2 * (int64_t)rs_chunks(n > 0 ? n : 1) + 4);  // part | agg | out
}

int64_t rlp_reward_norm_parts(int T, int n) {
    if (T < 0 || n < 0) return RLP_EINVAL;
    return (int64_t)T * 2 * rs_chunks(n > 0 ? n : 1);
}

int rlp_reward_norm_stats(const float *reward_in, int T, int n, double *work, rlp_stream_t stream) {
    RLP_REQUIRE(reward_in && work, "rlp_reward_norm_stats: null argument");
    RLP_REQUIRE(T >= 0 && n >= 0, "rlp_reward_norm_stats: T=%d n=%d", T, n);
    if (T == 0 || n == 0) return RLP_OK;
    const dim3 grid(rs_chunks(n), T < 65535 ? T : 65535);
    if (n % 4 == 0 && aligned16(reward_in))
        reward_stats_kernel<true><<<grid, 256, 0, as_stream(stream)>>>(reward_in, T, n, work);
    else
        reward_stats_kernel<false><<<grid, 256, 0, as_stream(stream)>>>(reward_in, T, n, work);
    RLP_CHECK_LAUNCH("rlp_reward_norm_stats");
    return RLP_OK;
}

int rlp_reward_norm_statistics(const float *reward_in, int T, int n, double *rms, double *work,
                               rlp_stream_t stream) {
    RLP_REQUIRE(reward_in && rms && work, "rlp_reward_norm_statistics: null argument");
    RLP_REQUIRE(T >= 0 && n >= 0, "rlp_reward_norm_statistics: T=%d n=%d", T, n);
    if (T == 0 || n == 0) return RLP_OK;
    if (n > 1) {
        const int rc = rlp_reward_norm_stats(reward_in, T, n, work, stream);
        if (rc != RLP_OK) return rc;
    }
    reward_merge_kernel<<<1, 256, 0, as_stream(stream)>>>(reward_in, T, n, 1, work, rms, work);
    RLP_CHECK_LAUNCH("rlp_reward_norm_statistics");
    return RLP_OK;
}

static void reward_apply(const float *reward_in, int T, int n, const double *out_t,
                         float *reward_out, hipStream_t s) {
    const bool vec = n % 4 == 0 && aligned16(reward_in) && aligned16(reward_out);
    const int per = vec ? 1024 : 256, bx = (n + per - 1) / per;
    const int cap = T >= 256 ? 64 : 16384 / (T > 0 ? T : 1);  // >= 16k blocks in flight
    const dim3 grid(bx < cap ? bx : cap, T < 65535 ? T : 65535);
    if (vec)
        reward_apply_kernel<true><<<grid, 256, 0, s>>>(reward_in, T, n, out_t, reward_out);
    else
        reward_apply_kernel<false><<<grid, 256, 0, s>>>(reward_in, T, n, out_t, reward_out);
}

static const double *reward_step_stats(const double *work, int T, int n) {
    return work + (size_t)T * rs_chunks(n) * 2 + (size_t)T * 2;
}

int rlp_reward_norm_finish(const float *reward_in, int T, int n, int world, const double *parts,
                           double *rms, double *work, float *reward_out, rlp_stream_t stream) {
    RLP_REQUIRE(reward_in && rms && work && reward_out, "rlp_reward_norm_finish: null argument");
    RLP_REQUIRE(T >= 0 && n >= 0 && world >= 1, "rlp_reward_norm_finish: T=%d n=%d world=%d", T, n,
                world);
    RLP_REQUIRE(parts || (world == 1 && n == 1), "rlp_reward_norm_finish: null parts");
    if (T == 0 || n == 0) return RLP_OK;
    hipStream_t s = as_stream(stream);
    reward_merge_kernel<<<1, 256, 0, s>>>(reward_in, T, n, world, parts, rms, work);
    reward_apply(reward_in, T, n, reward_step_stats(work, T, n), reward_out, s);
    RLP_CHECK_LAUNCH("rlp_reward_norm_finish");
    return RLP_OK;
}

int rlp_reward_norm(const float *reward_in, int T, int n, double *rms, double *work,
                    float *reward_out, rlp_stream_t stream) {
    RLP_REQUIRE(reward_in && rms && work && reward_out, "rlp_reward_norm: null argument");
    RLP_REQUIRE(T >= 0 && n >= 0, "rlp_reward_norm: T=%d n=%d", T, n);
    if (T == 0 || n == 0) return RLP_OK;
    const int rc = rlp_reward_norm_statistics(reward_in, T, n, rms, work, stream);
    if (rc != RLP_OK) return rc;
    reward_apply(reward_in, T, n, reward_step_stats(work, T, n), reward_out, as_stream(stream));
    RLP_CHECK_LAUNCH("rlp_reward_norm");
    return RLP_OK;
}

int rlp_reward_norm_apply(const float *reward_in, int T, int n, const double *work,
                          float *reward_out, rlp_stream_t stream) {
    RLP_REQUIRE(reward_in && work && reward_out, "rlp_reward_norm_apply: null argument");
    RLP_REQUIRE(T >= 0 && n >= 0, "rlp_reward_norm_apply: T=%d n=%d", T, n);
    if (T == 0 || n == 0) return RLP_OK;
    reward_apply(reward_in, T, n, reward_step_stats(work, T, n), reward_out, as_stream(stream));
    RLP_CHECK_LAUNCH("rlp_reward_norm_apply");
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
    gae_kernel<0><<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(
        reward, nullptr, value, value_next, done, success, g32, c, T, n, adv, v_target, adv_stats);
    RLP_CHECK_LAUNCH("rlp_gae");
    return RLP_OK;
}

int rlp_gae_normalized(const float *reward_raw, const double *reward_work, const float *value,
                       const float *value_next, const uint8_t *done, const uint8_t *success,
                       double gamma, double lambda, int T, int n, float *adv, float *v_target,
                       double *adv_stats, rlp_stream_t stream) {
    RLP_REQUIRE(reward_raw && reward_work && value && value_next && done && success && adv &&
                v_target, "rlp_gae_normalized: null argument");
    RLP_REQUIRE(T >= 0 && n >= 0, "rlp_gae_normalized: T=%d n=%d", T, n);
    if (T == 0 || n == 0) return RLP_OK;
    const float g32 = (float)gamma, c = (float)(gamma * lambda);
    const double *rs = reward_step_stats(reward_work, T, n);
    if (T <= kGaeLdsSteps)
        gae_kernel<1><<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(
            reward_raw, rs, value, value_next, done, success, g32, c, T, n, adv, v_target, adv_stats);
    else
        gae_kernel<2><<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(
            reward_raw, rs, value, value_next, done, success, g32, c, T, n, adv, v_target, adv_stats);
    RLP_CHECK_LAUNCH("rlp_gae_normalized");
    return RLP_OK;
}

int rlp_adv_stats_parts(int n) { return n < 0 ? RLP_EINVAL : (n + 255) / 256; }

int rlp_adv_normalize(float *adv, int64_t count, double *adv_stats, int parts,
                      rlp_stream_t stream) {
    RLP_REQUIRE(adv && adv_stats, "rlp_adv_normalize: null argument");
    RLP_REQUIRE(parts >= 1, "rlp_adv_normalize: parts=%d", parts);
    if (count <= 1) return RLP_OK;
    hipStream_t s = as_stream(stream);
    adv_stats_merge_kernel<<<1, 256, 0, s>>>(adv_stats, parts);
    const double *ms = adv_stats + 3 * (size_t)parts;
    if (aligned16(adv)) {
        const int64_t b = (count / 4 + 255) / 256;
        adv_norm_kernel<true><<<(int)(b < 1 ? 1 : b < 8192 ? b : 8192), 256, 0, s>>>(adv, count, ms);
    } else {
        const int64_t b = (count + 255) / 256;
        adv_norm_kernel<false><<<(int)(b < 8192 ? b : 8192), 256, 0, s>>>(adv, count, ms);
    }
    RLP_CHECK_LAUNCH("rlp_adv_normalize");
    return RLP_OK;
}

}  // extern "C"
