// rlp_rollout_oa.hip — the UGVForwardObstacleAvoidance PPO2 / DPPO2 rollout (rlp_rollout's
// lidar-env path). Its own translation unit because it is built with -mllvm -disable-machine-licm
// (Makefile): hoisting loop invariants (lane masks, the f64 polynomials' constants) out of the step
// kernel's loops spilled them to scratch, and the policy kernel that follows each step re-fetched
// its weights: 6.70 -> 5.72 ms per 16 384 x 64 segment (profiles/r6/r6q_lidar_nolicm_ab.txt). The
// other rollout kernels keep MachineLICM (0.7 % faster with it, r6l).
#include "rlp_rollout.hpp"

namespace rlp {

// ------------------------------------------------------------------------------------------
// UGVForwardObstacleAvoidance PPO2 / DPPO2 rollout (demonstration/PPO2/PPO2-4-UGVForward
// ObstacleAvoidance/train.py:48-50,95-97: 41 -> 256 -> 256 -> 2 actor, 41 -> 256 -> 256 -> 1
// critic, tanh; DPPO2 copy likewise). ONE rlp_rollout call runs the driver loop on the caller's
// stream (no host round trip, no synchronisation): two launches per step,
//   oa_policy2_kernel  (f16x3, the default: 8-wave blocks over 64 rows, waves 0-3 the actor,
//   / oa_policy_kernel 4-7 the critic; RLP_MLP_FP32: per 16-env wave, both nets in turn): actor
//                      and critic forward (layer 1 as 11 K-steps of the exact f32 16x16x4 MFMA,
//                      the 256 x 256 hidden layer on f16x3 / exact f32 MFMA), then the Philox
//                      sample (the fused kernel's stream), clamp, log-prob, V(s_t), and
//                      V(s'_{t-1}) = V(s_t) where the env did not end at t-1
//   oa_step_kernel     lidar env step (dynamics, terminal, reward: one lane per env), the
//                      success rule, the 37-beam scan of s' (one (env, beam) pair per lane) into
//                      obs_next and — for envs still running — obs_{t+1}; ended envs reset with the
//                      map generator (one wave per env, counter step0 + t + 1) and scan the new pose
//                      into obs_{t+1}
// and after the segment the bootstrap V(s'_{T-1}) of the envs still running (the policy kernel,
// critic only). RLP_OA_ONE_LAUNCH=1 runs the f16x3 segment as ONE launch instead
// (oa_rollout_kernel, below: 5.31 against 6.66 ms per 16 384 x 64 segment), opt-in only: it
// faulted (illegal address) when run after other streams of the process had run work; the cause
// is not found. Same semantics, random draws and buffers in every form.
struct OaPolicyArgs {
    const float *actor, *critic;
    MfmaNet an, cn;
    RolloutArgs ra;
    rlp_rollout_bufs b;
    int t;     // step of this launch
    int boot;  // 1: critic on obs_next[T-1] -> value_next of the envs still running
};

constexpr int kOaPolWaves = 4;  // 16-env waves per block, one block per CU (1 wave per SIMD)
constexpr int kOaKs1 = (OA::S + 3) / 4;
constexpr int kOaSmall = mlp_small_floats<256, kOaKs1, OA::A>();
constexpr int kOaRing = kOaPolWaves * RING * mlp_phase_floats<256>();  // per-wave W2 rings

// exact f32 (RLP_MLP_FP32): both nets per wave in turn, one wave per SIMD
__global__ void __launch_bounds__(64 * kOaPolWaves, 1) oa_policy_kernel(OaPolicyArgs pa) {
    constexpr int A = OA::A, S = OA::S, KS1 = kOaKs1, ROWS = 16 * kOaPolWaves;
    __shared__ __attribute__((aligned(16))) float lds[2 * kOaSmall + kOaRing];
    float *small_a = lds, *small_c = lds + kOaSmall, *ring0 = lds + 2 * kOaSmall;
    const MfmaNet an = pa.an, cn = pa.cn;
    if (!pa.boot) mlp_small_to_lds(pa.actor, an, small_a, false);
    mlp_small_to_lds(pa.critic, cn, small_c, false);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, e = lane & 15;
    float *ring = ring0 + wave * RING * mlp_phase_floats<256>();
    const RolloutArgs &ra = pa.ra;
    const int n = ra.n, t = pa.t;
    const float *x = pa.boot ? pa.b.obs_next + (size_t)(ra.T - 1) * n * S : pa.b.obs + (size_t)t * n * S;
    for (int r0 = blockIdx.x * ROWS; r0 < n; r0 += gridDim.x * ROWS) {
        const int row = r0 + 16 * wave + e;
        float bobs[1][KS1];
#pragma unroll
        for (int kk = 0; kk < KS1; ++kk)
            bobs[0][kk] = (row < n && 4 * kk + g < S) ? x[(size_t)row * S + 4 * kk + g] : 0.f;
        float mraw[A] = {}, v = 0.f;
#pragma unroll 1
        for (int which = pa.boot ? 1 : 0; which < 2; ++which) {
            float out[1][A];
            mlp_fused_forward<256, 1, KS1, A, RING>(which ? pa.critic : pa.actor,
                                                    which ? small_c : small_a, ring,
                                                    which ? cn : an, which ? 1 : A, bobs, out);
            if (which) v = out[0][0];
            else
#pragma unroll
                for (int a = 0; a < A; ++a) mraw[a] = out[0][a];
        }
        if (g != 0 || row >= n) continue;  // lane e of group 0 owns env `row`
        const rlp_rollout_bufs &b = pa.b;
        if (pa.boot) {
            const size_t k = (size_t)(ra.T - 1) * n + row;
            if (!b.done[k]) b.value_next[k] = v;
            continue;
        }
        const size_t k = (size_t)t * n + row;
        float eps[A];
        philox_normal_f32<A>(ra.seed, ra.step0 + (uint64_t)t, ra.env_id0 + (uint64_t)row, eps);
#pragma unroll
        for (int a = 0; a < A; ++a) {
            const float m = (an.out_tanh ? tanhf(mraw[a]) : mraw[a]) * ra.gain[a] + ra.off[a];
            float xa = m + ra.std_[a] * eps[a];
            xa = fmaxf(fminf(xa, ra.a_max[a]), ra.a_min[a]);
            b.action[k * A + a] = xa;
            b.logp[k * A + a] = normal_logp_c(xa, m, ra.half_inv_var[a], ra.log_std[a]);
        }
        b.value[k] = v;
        if (t > 0 && !b.done[k - n]) b.value_next[k - n] = v;  // V(s'_{t-1}) == V(s_t)
    }
}

// f16x3 policy with two waves per SIMD: 8-wave blocks over 64 rows, waves 0-3 run the actor and
// sample, waves 4-7 the critic and the value bookkeeping, each group through its own W2 chunk ring
// (the two groups execute the same barrier sequence: both nets have 16 chunks per pass). Boot
// (critic only): both groups run the critic, on 128 rows per block. One wave per SIMD with both
// nets in turn (the first version) left the layer-1 LDS reads, the ring waits and the tanh
// stretches of the single wave exposed: 41 -> 29 us per step at 16 384 envs
// (profiles/r6/r6c_lidar_rollout_trace_stats.txt). The same policy is the one-launch segment's
// policy phase (oa_rollout_kernel, below).
constexpr int kOaPol2Ring = 2;  // ring slots per group: both nets' resident parts + 2 x 2 slots fill the 160 KiB
constexpr int kOaSmallA = mlp_small_floats<256, kOaKs1, OA::A>(), kOaSmallC = mlp_small_floats<256, kOaKs1, 1>();
static_assert(4 * (kOaSmallA + kOaSmallC + 2 * kOaPol2Ring * kX3ChunkFloats) <= 160 * 1024,
              "oa_policy2_kernel / oa_rollout_kernel LDS");
__global__ void __launch_bounds__(512, 1) oa_policy2_kernel(OaPolicyArgs pa) {
    constexpr int A = OA::A, S = OA::S, KS1 = kOaKs1;
    __shared__ __attribute__((aligned(16))) float lds[kOaSmallA + kOaSmallC + 2 * kOaPol2Ring * kX3ChunkFloats];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, e = lane & 15;
    const int grp = __builtin_amdgcn_readfirstlane(wave >> 2), wq = wave & 3;
    const bool boot = pa.boot != 0;
    const bool critic = boot || grp == 1;
    float *small0 = lds, *small1 = lds + kOaSmallA;
    float *ring = lds + kOaSmallA + kOaSmallC + grp * kOaPol2Ring * kX3ChunkFloats;
    // group 0's region holds the actor (boot: a second copy of the critic), group 1's the critic
    mlp_small_to_lds(boot ? pa.critic : pa.actor, boot ? pa.cn : pa.an, small0, true);
    mlp_small_to_lds(pa.critic, pa.cn, small1, true);
    __syncthreads();
    const float *P = critic ? pa.critic : pa.actor;
    const MfmaNet &net = critic ? pa.cn : pa.an;
    const float *small = grp ? small1 : small0;
    const RolloutArgs &ra = pa.ra;
    const int n = ra.n, t = pa.t;
    const int rows_blk = boot ? 128 : 64;
    const float *x = boot ? pa.b.obs_next + (size_t)(ra.T - 1) * n * S : pa.b.obs + (size_t)t * n * S;
    for (int r0 = blockIdx.x * rows_blk; r0 < n; r0 += gridDim.x * rows_blk) {  // block-uniform
        const int row = r0 + (boot ? 64 * grp : 0) + 16 * wq + e;
        float bobs[1][KS1];
#pragma unroll
        for (int kk = 0; kk < KS1; ++kk)
            bobs[0][kk] = (row < n && 4 * kk + g < S) ? x[(size_t)row * S + 4 * kk + g] : 0.f;
        float out[1][A];
        mlp_x3_forward<256, 1, KS1, A, kOaPol2Ring, 4, 1>(P, small, ring, net, critic ? 1 : A, bobs, out);
        if (g != 0 || row >= n) continue;  // lane e of group 0 owns row `row`
        const rlp_rollout_bufs &b = pa.b;
        if (boot) {
            const size_t k = (size_t)(ra.T - 1) * n + row;
            if (!b.done[k]) b.value_next[k] = out[0][0];
            continue;
        }
        const size_t k = (size_t)t * n + row;
        if (critic) {
            const float v = out[0][0];
            b.value[k] = v;
            if (t > 0 && !b.done[k - n]) b.value_next[k - n] = v;  // V(s'_{t-1}) == V(s_t)
            continue;
        }
        float eps[A];
        philox_normal_f32<A>(ra.seed, ra.step0 + (uint64_t)t, ra.env_id0 + (uint64_t)row, eps);
#pragma unroll
        for (int a = 0; a < A; ++a) {
            const float m = (pa.an.out_tanh ? tanhf(out[0][a]) : out[0][a]) * ra.gain[a] + ra.off[a];
            float xa = m + ra.std_[a] * eps[a];
            xa = fmaxf(fminf(xa, ra.a_max[a]), ra.a_min[a]);
            b.action[k * A + a] = xa;
            b.logp[k * A + a] = normal_logp_c(xa, m, ra.half_inv_var[a], ra.log_std[a]);
        }
    }
}

// EB envs per block: phase 1 one lane per env, phase 2 the EB x 37 (env, beam) pairs over the
// block, phase 3 the ended envs' resets, one wave per env
#ifdef RLP_OA_CHECK  // diagnostic build: bounds of the lidar step / segment kernels' global accesses
#define OA_GUARD(cond, what) ((cond) ? true : (printf("oa_rollout_kernel OOB %s blk %d tid %d\n", what, (int)blockIdx.x, (int)threadIdx.x), false))
#else
#define OA_GUARD(cond, what) true
#endif
constexpr int kOaSegEnvs = 64;
constexpr int kOaArgsBytes = 1024;  // rlp_rollout_workspace_bytes of the lidar env

// 4 waves per SIMD (<= 128 registers, ~240 B of scratch spills): the kernel's phases are latency
// chains (per-env f64 dynamics and setup, divergent beams, the map generator's rounds) that only
// more resident waves hide: 16 384 x 64 segment 7.48 -> 6.66 ms against 2 waves per SIMD (213
// registers, no spills), 6.75 ms at 3 (profiles/r6/r6d_lidar_occupancy_ab.txt)
template <int EB>
__global__ void __launch_bounds__(256, 4) oa_step_kernel(OA::P p, double *state, uint8_t *need_reset,
                                                      RolloutArgs ra, int t, rlp_rollout_bufs b) {
    constexpr int S = OA::S, A = OA::A, NW = 4;
    __shared__ OaEnvLds L[EB];
    __shared__ OaEnvLds Lr[NW];
    __shared__ double obl[NW][OA::NOBS * 3];
    __shared__ uint8_t s_done[EB];
    const int tid = threadIdx.x, n = ra.n, T = ra.T;
    const int e0 = blockIdx.x * EB, ne = n - e0 < EB ? n - e0 : EB;
    const bool more = t + 1 < ra.T;  // a step t + 1 follows in this segment
    const size_t k0 = (size_t)t * n;
    if (tid < ne) {
        const size_t i = (size_t)e0 + tid, k = k0 + i;
        double s[OA::DW];
#pragma unroll
        for (int d = 0; d < OA::DW; ++d) s[d] = state[(size_t)d * n + i];
        for (int kk = 0; kk < p.n_obs; ++kk) {
            L[tid].ob[kk].x0 = state[(size_t)(OA::OB + 3 * kk) * n + i];
            L[tid].ob[kk].y0 = state[(size_t)(OA::OB + 3 * kk + 1) * n + i];
            L[tid].ob[kk].r0 = state[(size_t)(OA::OB + 3 * kk + 2) * n + i];
        }
        const float a[A] = {b.action[k * A], b.action[k * A + 1]};
        double r, e, eph;
        int f;
        bool dn;
        OA::step_core(p, s, a, [&](double x, double y) {
            return OA::collision_at(p, x, y, [&](int kk, double &x0, double &y0, double &r0) {
                x0 = L[tid].ob[kk].x0; y0 = L[tid].ob[kk].y0; r0 = L[tid].ob[kk].r0;
            });
        }, r, f, dn, e, eph);
        if (!(dn && more)) {  // an env that resets below gets its whole state from the reset
#pragma unroll
            for (int d = 0; d < OA::DW; ++d) state[(size_t)d * n + i] = s[d];
        }
        if (OA_GUARD(k < (size_t)T * n && i < (size_t)n, "p1 bufs")) {
            b.reward[k] = (float)r;
            b.flag[k] = (int8_t)f;
            b.done[k] = dn;
            b.success[k] = success_of(ra.success_rule, ra.success_flag, dn, f);
        }
        if (!more) need_reset[i] = dn;  // ended envs of the last step reset next segment
        s_done[tid] = dn;
        oa_setup(p, L[tid], s);
        float h[4];
        OA::obs_head(p, s, e, eph, h);
#pragma unroll
        for (int j = 0; j < 4; ++j) b.obs_next[k * S + j] = h[j];
        if (more && !dn) {  // current_state = next_state
#pragma unroll
            for (int j = 0; j < 4; ++j) b.obs[(k + n) * S + j] = h[j];
        }
    }
    __syncthreads();
    for (int it = tid; it < ne * OA::NL; it += 256) {
        const int le = it / OA::NL, i = it - le * OA::NL;
        const size_t k = k0 + e0 + le;
        const float v = oa_beam(p, L[le], i);
        b.obs_next[k * S + 4 + i] = v;
        if (more && !s_done[le]) b.obs[(k + n) * S + 4 + i] = v;
    }
    if (!more) return;
    // the ended envs' resets (counter step0 + t + 1) and their obs_{t+1}: wave w takes the block's
    // ended envs w, w + NW, ... in env order (s_done is final since the barrier above)
    const int w = tid >> 6;
    int c = 0;
    for (int le = 0; le < ne; ++le) {
        if (!s_done[le]) continue;
        if (c++ % NW != w) continue;
        const size_t i = (size_t)e0 + le;
        oa_reset_wave(p, state, n, i, ra.seed, ra.step0 + (uint64_t)t + 1, ra.env_id0 + i,
                      b.obs + (k0 + n + i) * S, obl[w], Lr[w]);
    }
}

// ------------------------------------------------------------------------------------------
// The whole segment in ONE launch (f16x3): a block owns kOaSegEnvs envs for all T steps — its
// weights' resident parts are loaded once per segment, and blocks drift independently, so an env's
// reset (the map generator, tens of microseconds of one wave's latency) delays only its own block
// instead of the whole grid at every step (oa_step_kernel ends when its slowest block does).
// Per step, 8 waves (2 per SIMD): the policy phase (waves 0-3 actor + sample,
// 4-7 critic + values) on the block's 64 envs, then the env step of oa_step_kernel on the same
// 64 envs (512 threads: phase 1 one lane per env, spread 8 per wave; the beams over the block;
// ended envs reset one wave each). The step's scratch (the envs' obstacle / pose records) and the
// next observations reuse the two W2 rings' LDS between the policy passes; actions and done flags
// hand over through LDS of their own; state written by another wave (a reset) is waited for
// (vmcnt) before the step's closing barrier.

struct OaSegLds {
    OaEnvLds L[kOaSegEnvs];
    OaEnvLds Lr[8];
    double obl[8][OA::NOBS * 3];
    float sobs[kOaSegEnvs][OA::S];  // s_{t+1} (s'_{T-1} after the last step): the policy's input
    uint8_t done[kOaSegEnvs];
};
static_assert(sizeof(OaSegLds) <= 4 * 2 * kOaPol2Ring * kX3ChunkFloats, "segment scratch within the rings");
struct OaSegArgs {
    OA::P p;
    double *state;
    uint8_t *need_reset;
    const float *actor, *critic;
    MfmaNet an, cn;
    RolloutArgs ra;
    rlp_rollout_bufs b;
};

// the two phases; the launch's arguments are re-read from their workspace copy at each phase (an
// opaque scalar pointer per phase), so no parameter is held in registers across the other phase
__device__ __forceinline__ void oa_seg_policy(const OaSegArgs &g, OaSegLds &Z, float *small0,
                                                        float *small1, float *ring, float (*sact)[OA::A],
                                                        const uint8_t *sdone, int e0, int ne, int t) {
    constexpr int A = OA::A, S = OA::S, KS1 = kOaKs1;
    // an opaque thread index per phase: nothing derived from it is hoisted across the other phase
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wave = tid >> 6, gl = lane >> 4, e = lane & 15;
    const int grp = __builtin_amdgcn_readfirstlane(wave >> 2), wq = wave & 3;
    const RolloutArgs &ra = g.ra;
    const rlp_rollout_bufs &b = g.b;
    const int n = ra.n, T = ra.T;
    const bool boot = t == T;  // the bootstrap pass: critic on s'_{T-1}
    const int le = 16 * wq + e, row = e0 + le;
    float bobs[1][KS1];
#pragma unroll
    for (int kk = 0; kk < KS1; ++kk)
        bobs[0][kk] = (le < ne && 4 * kk + gl < S) ? Z.sobs[le][4 * kk + gl] : 0.f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read before the rings refill
    const bool critic = grp == 1;
    // the net's pointer as a wave-uniform (scalar) value: the forward pins it in SGPRs
    const uint64_t pv = (uint64_t)(critic ? g.critic : g.actor);
    const float *P = (const float *)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pv >> 32)) << 32) |
                                     (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)pv));
    float out[1][A];
    mlp_x3_forward<256, 1, KS1, A, kOaPol2Ring, 4, 1>(P, critic ? small1 : small0, ring,
                                                      critic ? g.cn : g.an, critic ? 1 : A, bobs, out);
    if (gl != 0 || le >= ne) return;
    if (boot) {
        const size_t k = (size_t)(T - 1) * n + row;
        if (critic && !sdone[le] && OA_GUARD(k < (size_t)T * n, "boot vn")) b.value_next[k] = out[0][0];
        return;
    }
    const size_t k = (size_t)t * n + row;
    if (critic) {
        const float v = out[0][0];
        if (OA_GUARD(k < (size_t)T * n, "value")) b.value[k] = v;
        if (t > 0 && !sdone[le] && OA_GUARD(k >= (size_t)n && k < (size_t)T * n, "vn")) b.value_next[k - n] = v;  // V(s'_{t-1}) == V(s_t)
        return;
    }
    float eps[A];
    philox_normal_f32<A>(ra.seed, ra.step0 + (uint64_t)t, ra.env_id0 + (uint64_t)row, eps);
#pragma unroll
    for (int a = 0; a < A; ++a) {
        const float m = (g.an.out_tanh ? tanhf(out[0][a]) : out[0][a]) * ra.gain[a] + ra.off[a];
        float xa = m + ra.std_[a] * eps[a];
        xa = fmaxf(fminf(xa, ra.a_max[a]), ra.a_min[a]);
        if (OA_GUARD(k < (size_t)T * n, "action")) {
            b.action[k * A + a] = xa;
            b.logp[k * A + a] = normal_logp_c(xa, m, ra.half_inv_var[a], ra.log_std[a]);
        }
        sact[le][a] = xa;
    }
}

__device__ __forceinline__ void oa_seg_step(const OaSegArgs &g, OaSegLds &Z,
                                                      const float (*sact)[OA::A], uint8_t *sdone,
                                                      int e0, int ne, int t) {
    constexpr int A = OA::A, S = OA::S, NW = 8;
    int tid = threadIdx.x;  // (opaque per phase, as in oa_seg_policy)
    asm volatile("" : "+v"(tid));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const OA::P &p = g.p;
    const RolloutArgs &ra = g.ra;
    const rlp_rollout_bufs &b = g.b;
    const int n = ra.n, T = ra.T;
    const bool more = t + 1 < T;
    const size_t k0 = (size_t)t * n;
    if ((tid & 7) == 0 && (tid >> 3) < ne) {  // phase 1: env le on lane 8 le (8 per wave)
        const int le = tid >> 3;
        const size_t i = (size_t)e0 + le, k = k0 + i;
#ifdef RLP_OA_CHECK
        if (i >= (size_t)n || k >= (size_t)T * n || (more && k + n >= (size_t)T * n))
            printf("oa_seg_step p1: i %lu k %lu n %d T %d\n", (unsigned long)i, (unsigned long)k, n, T);
#endif
        OaEnvLds &L = Z.L[le];
        double s[OA::DW];
#pragma unroll
        for (int d = 0; d < OA::DW; ++d) s[d] = g.state[(size_t)d * n + i];
        for (int kk = 0; kk < p.n_obs; ++kk) {
            L.ob[kk].x0 = g.state[(size_t)(OA::OB + 3 * kk) * n + i];
            L.ob[kk].y0 = g.state[(size_t)(OA::OB + 3 * kk + 1) * n + i];
            L.ob[kk].r0 = g.state[(size_t)(OA::OB + 3 * kk + 2) * n + i];
        }
        const float a[A] = {sact[le][0], sact[le][1]};
        double r, ee, eph;
        int f;
        bool dn;
        OA::step_core(p, s, a, [&](double x, double y) {
            return OA::collision_at(p, x, y, [&](int kk, double &x0, double &y0, double &r0) {
                x0 = L.ob[kk].x0; y0 = L.ob[kk].y0; r0 = L.ob[kk].r0;
            });
        }, r, f, dn, ee, eph);
        if (!(dn && more)) {  // an env that resets below gets its whole state from the reset
#pragma unroll
            for (int d = 0; d < OA::DW; ++d) g.state[(size_t)d * n + i] = s[d];
        }
        if (OA_GUARD(k < (size_t)T * n && i < (size_t)n, "p1 bufs")) {
            b.reward[k] = (float)r;
            b.flag[k] = (int8_t)f;
            b.done[k] = dn;
            b.success[k] = success_of(ra.success_rule, ra.success_flag, dn, f);
        }
        if (!more) g.need_reset[i] = dn;  // ended envs of the last step reset next segment
        Z.done[le] = dn;
        sdone[le] = dn;
        oa_setup(p, L, s);
        float h[4];
        OA::obs_head(p, s, ee, eph, h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (OA_GUARD(k < (size_t)T * n, "p1 obs_next")) b.obs_next[k * S + j] = h[j];
            if (!more || !dn) Z.sobs[le][j] = h[j];  // s_{t+1} (or s'_{T-1} for the bootstrap)
            if (more && !dn && OA_GUARD(k + n < (size_t)T * n, "p1 obs")) b.obs[(k + n) * S + j] = h[j];
        }
    }
    __syncthreads();
    for (int it = tid; it < ne * OA::NL; it += 512) {  // phase 2: the beams of s'_t
        const int le = it / OA::NL, i = it - le * OA::NL;
        const size_t k = k0 + e0 + le;
        const float v = oa_beam(p, Z.L[le], i);
        if (OA_GUARD(k < (size_t)T * n && le < kOaSegEnvs, "p2 obs_next")) b.obs_next[k * S + 4 + i] = v;
        if (!more || !Z.done[le]) Z.sobs[le][4 + i] = v;
        if (more && !Z.done[le] && OA_GUARD(k + n < (size_t)T * n, "p2 obs")) b.obs[(k + n) * S + 4 + i] = v;
    }
    if (!more) return;
    int c = 0;  // phase 3: the ended envs' resets (counter step0 + t + 1), one wave each
    for (int le = 0; le < ne; ++le) {
        if (!Z.done[le]) continue;
        if (c++ % NW != wave) continue;
        const size_t i = (size_t)e0 + le;
#ifdef RLP_OA_CHECK
        if (i >= (size_t)n || k0 + n + i >= (size_t)T * n || wave >= 8)
            printf("oa_seg_step reset: i %lu k0 %lu n %d T %d wave %d\n", (unsigned long)i, (unsigned long)k0, n, T, wave);
#endif
        oa_reset_wave(p, g.state, n, i, ra.seed, ra.step0 + (uint64_t)t + 1, ra.env_id0 + i,
                      b.obs + (k0 + n + i) * S, Z.obl[wave], Z.Lr[wave], Z.sobs[le]);
    }
}

// The launch's arguments are read from a copy in the caller's workspace (oa_args_kernel writes
// it, stream-ordered, from its own kernarg segment), not from this launch's kernarg segment: a
// multi-millisecond launch that re-reads its kernarg segment at every phase depends on the
// runtime keeping that segment intact for the whole launch.
static_assert(sizeof(OaSegArgs) <= kOaArgsBytes && sizeof(OaSegArgs) % 16 == 0, "OaSegArgs copy");
__global__ void __launch_bounds__(64) oa_args_kernel(OaSegArgs a, OaSegArgs *dst) {
    if (threadIdx.x == 0) *dst = a;
}

#ifdef RLP_OA_KCHECK  // diagnostic build: does this launch's kernarg segment change while it runs?
struct OaKcheckArgs {  // the kernarg segment of the diagnostic build's oa_rollout_kernel
    const OaSegArgs *ga;
    OaSegArgs kg;
    unsigned *diag;
};
#define OA_KCHECK_PARAMS , OaSegArgs kg, unsigned *diag
#define OA_KCHECK_ARGS(a) , a, (unsigned *)nullptr
#else
#define OA_KCHECK_PARAMS
#define OA_KCHECK_ARGS(a)
#endif

__global__ void __launch_bounds__(512, 1) oa_rollout_kernel(const OaSegArgs *ga OA_KCHECK_PARAMS) {
    constexpr int EB = kOaSegEnvs, S = OA::S;
    __shared__ __attribute__((aligned(16))) float lds[kOaSmallA + kOaSmallC + 2 * kOaPol2Ring * kX3ChunkFloats];
    __shared__ float sact[EB][OA::A];
    __shared__ uint8_t sdone[EB];  // done of the previous step (V(s'_{t-1}) bookkeeping)
    float *small0 = lds, *small1 = lds + kOaSmallA, *rings = lds + kOaSmallA + kOaSmallC;
    OaSegLds &Z = *reinterpret_cast<OaSegLds *>(rings);
    const OaSegArgs &g = *ga;
    mlp_small_to_lds(g.actor, g.an, small0, true);
    mlp_small_to_lds(g.critic, g.cn, small1, true);
    const int tid = threadIdx.x, grp = __builtin_amdgcn_readfirstlane((tid >> 6) >> 2);
    float *ring = rings + grp * kOaPol2Ring * kX3ChunkFloats;
    const int n = g.ra.n, T = g.ra.T;
#ifdef RLP_OA_KCHECK
    bool reported = false;
#endif
    for (int e0 = blockIdx.x * EB; e0 < n; e0 += gridDim.x * EB) {  // block-uniform
        const int ne = n - e0 < EB ? n - e0 : EB;
        __syncthreads();  // (the resident parts loaded; the previous group's last pass done)
        for (int i = tid; i < EB * S; i += 512) {  // s_0 (the caller's reset + observation)
            const int le = i / S, j = i - le * S;
            Z.sobs[le][j] = le < ne ? g.b.obs[(size_t)(e0 + le) * S + j] : 0.f;
        }
        __syncthreads();
        for (int t = 0; t <= T; ++t) {
#ifdef RLP_OA_KCHECK
            if (tid == 0 && !reported) {
                const auto *k = (const __attribute__((address_space(4))) OaKcheckArgs *)
                    __builtin_amdgcn_kernarg_segment_ptr();
                asm volatile("" : "+s"(k));
                const bool same = k->kg.state == ga->state && k->kg.actor == ga->actor &&
                                  k->kg.critic == ga->critic && k->kg.b.obs == ga->b.obs &&
                                  k->kg.b.action == ga->b.action && k->kg.ra.n == ga->ra.n;
                if (!same) {
                    printf("oa_rollout_kernel: kernarg segment changed, block %d step %d\n",
                           (int)blockIdx.x, t);
                    reported = true;
                }
            }
#endif
            {
                const OaSegArgs *gp = ga;
                asm volatile("" : "+s"(gp));  // re-read per phase (scalar loads), not held
                oa_seg_policy(*gp, Z, small0, small1, ring, sact, sdone, e0, ne, t);
            }
            __syncthreads();  // actions in LDS; every wave is done with the rings
            if (t == T) break;
            {
                const OaSegArgs *gp = ga;
                asm volatile("" : "+s"(gp));
                oa_seg_step(*gp, Z, sact, sdone, e0, ne, t);
            }
            // the state a reset wave wrote is read by another wave at the next step: stores done
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }
}

// RLP_OA_ONE_LAUNCH=1 selects the one-launch segment for the f16x3 hidden layer (read once).
// Opt-in only: see the section comment above and DESIGN.md §4 round 6.
static bool oa_one_launch() {
    static const bool on = [] {
        const char *v = getenv("RLP_OA_ONE_LAUNCH");
        return v && v[0] == '1';
    }();
    return on;
}

int64_t rollout_oa_workspace_bytes() { return kOaArgsBytes; }

int rollout_oa(const void *params, double *state, uint8_t *need_reset, const float *actor,
               const MfmaNet &an, const float *critic, const MfmaNet &cn, const RolloutArgs &ra,
               const rlp_rollout_bufs &b, int prec, void *workspace, int64_t workspace_bytes,
               hipStream_t s) {
    const auto &p = *static_cast<const OA::P *>(params);
    if (an.S != OA::S || cn.S != OA::S || an.A != OA::A || cn.A != 1)
        return fail(RLP_EINVAL, "rlp_rollout: net dims (S=%d,A=%d / S=%d,A=%d) != env (S=%d,A=%d)",
                    an.S, an.A, cn.S, cn.A, OA::S, OA::A);
    if (an.H != 256 || cn.H != 256)
        return fail(RLP_EUNSUPPORTED, "rlp_rollout: hidden width %d/%d (built for 256)", an.H, cn.H);
    if (p.n_obs < 0 || p.n_obs > OA::NOBS)
        return fail(RLP_EINVAL, "UGVForwardObstacleAvoidance: n_obs=%d (0..%d)", p.n_obs, OA::NOBS);
    const int n = ra.n, T = ra.T;
    const int cus = device_cus();
    const int rows_pb = 16 * kOaPolWaves;
    const int pblocks = (n + rows_pb - 1) / rows_pb < cus ? (n + rows_pb - 1) / rows_pb : cus;
    // fewer envs per block when the batch is small, so every CU gets several blocks
    const bool eb64 = (n + 63) / 64 >= 4 * cus;
    auto policy = [&](int t, int boot) {
        const OaPolicyArgs pa{actor, critic, an, cn, ra, b, t, boot};
        if (prec == RLP_MLP_F16X3) {
            const int rb = boot ? 128 : 64, nb = (n + rb - 1) / rb;
            oa_policy2_kernel<<<nb < cus ? nb : cus, 512, 0, s>>>(pa);
        } else {
            oa_policy_kernel<<<pblocks, 64 * kOaPolWaves, 0, s>>>(pa);
        }
    };
    int rc = launch_ugvoa_reset(p, state, n, need_reset, nullptr, ra.seed, ra.step0, ra.env_id0, s);
    if (rc == RLP_OK) rc = launch_ugvoa_observe(p, state, n, b.obs, s);
    if (rc != RLP_OK) return rc;
    if (prec == RLP_MLP_F16X3 && oa_one_launch()) {  // the whole segment in one launch
        if (!workspace || workspace_bytes < kOaArgsBytes)
            return fail(RLP_EINVAL, "rlp_rollout: the lidar segment needs %d workspace bytes",
                        kOaArgsBytes);
        const int nb = (n + kOaSegEnvs - 1) / kOaSegEnvs;
        const OaSegArgs a{p, state, need_reset, actor, critic, an, cn, ra, b};
        OaSegArgs *ga = static_cast<OaSegArgs *>(workspace);
        oa_args_kernel<<<1, 64, 0, s>>>(a, ga);
        oa_rollout_kernel<<<nb < cus ? nb : cus, 512, 0, s>>>(ga OA_KCHECK_ARGS(a));
        RLP_CHECK_LAUNCH("rlp_rollout (UGVForwardObstacleAvoidance)");
        return RLP_OK;
    }
    for (int t = 0; t < T; ++t) {
        policy(t, 0);
        if (eb64) oa_step_kernel<64><<<(n + 63) / 64, 256, 0, s>>>(p, state, need_reset, ra, t, b);
        else oa_step_kernel<16><<<(n + 15) / 16, 256, 0, s>>>(p, state, need_reset, ra, t, b);
    }
    policy(T - 1, 1);  // V(s'_{T-1}) of the envs still running
    RLP_CHECK_LAUNCH("rlp_rollout (UGVForwardObstacleAvoidance)");
    return RLP_OK;
}


}  // namespace rlp
