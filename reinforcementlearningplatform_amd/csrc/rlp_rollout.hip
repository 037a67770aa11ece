// rlp_rollout.hip — fused batched rollout: the reference driver loop
// (demonstration/PPO2/PPO2-4-CartPole/train.py:184-217) for n envs and T steps in ONE launch.
//
// Per wave: WENV = 16*SUB envs, env state resident in registers (f64) for all T steps. Per step:
//   auto-reset (need_reset)            train.py:187-191, env.reset(random=True)
//   obs = get_state()                  CartPole.py:145-153 (etc.)
//   actor forward -> mean; sample      Proximal_Policy_Optimization2.py:69-76 (Philox eps)
//   critic forward -> V(s_t)           (learn() :91, same params => same values)
//   env.step_update(a)                 CartPole.py:257-264 (etc.)
//   buffer.append(...)                 utils/classes.py:264-272, time-major [T][n][...]
// The two MLPs are fp32 MFMA (v_mfma_f32_16x16x4_f32): this kernel is MFMA-bound.
#include "rlp_rollout.hpp"

namespace rlp {

// fp32 path: SUB == 4 -> 256 threads (1 wave per SIMD); SUB == 2 -> 512 threads, waves w and w+4
// share a SIMD (MI355X_MICROARCH.md "Two waves per SIMD"); one block per CU, per-wave W2 rings.
// f16x3 path: 4-wave blocks sharing one W2 ring, two blocks per CU (2 waves per SIMD).
template <int SUB, bool X3> constexpr int rollout_block() { return X3 ? 256 : (SUB == 4 ? 256 : 512); }
// f16x3: SUB == 2 -> two 4-wave blocks per CU (2 waves per SIMD, 256 registers each); SUB == 4 ->
// one block per CU (1 wave per SIMD, 512 registers: the SUB x 64 accumulators live in AGPRs) with
// all 64 lanes doing f64 physics
template <int SUB, bool X3> constexpr int rollout_min_blocks() { return X3 && SUB <= 2 ? 2 : 1; }


template <int KIND, int H, int SUB, bool X3>
__global__ void __launch_bounds__((rollout_block<SUB, X3>()), (rollout_min_blocks<SUB, X3>()))
rollout_kernel(typename Env<KIND>::P p, double *__restrict__ state, uint8_t *__restrict__ need_reset,
               const float *__restrict__ actor, MfmaNet an, const float *__restrict__ critic,
               MfmaNet cn, RolloutArgs ra, rlp_rollout_bufs b) {
    using E = Env<KIND>;
    constexpr int S = E::S, A = E::A, D = E::D, KS1 = (S + 3) / 4, WENV = 16 * SUB;
    constexpr int WAVES = rollout_block<SUB, X3>() / 64;
    constexpr int SMALL = mlp_small_floats<H, KS1, A>(), PF = mlp_phase_floats<H>();
    constexpr int RINGF = X3 ? kX3RingFloats : WAVES * RING * PF;
    // ONE __shared__ object (a second one next to the LDS-DMA ring can make hipcc drain vmcnt
    // before every ds_read): [actor small | critic small | obs staging | W2 ring(s)]
    __shared__ __attribute__((aligned(16))) float lds[2 * SMALL + WAVES * WENV * 8 + RINGF];
    float *small_a = lds, *small_c = lds + SMALL;
    float(*sobs)[WENV][8] = reinterpret_cast<float(*)[WENV][8]>(lds + 2 * SMALL);
    float *ring = lds + 2 * SMALL + WAVES * WENV * 8 + (X3 ? 0 : (threadIdx.x >> 6) * RING * PF);
    mlp_small_to_lds(actor, an, small_a, X3);
    mlp_small_to_lds(critic, cn, small_c, X3);
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, e = lane & 15;
    const int n = ra.n;
    const int env = (blockIdx.x * WAVES + wave) * WENV + lane;  // physics lane -> env

    const bool phys = lane < WENV && env < n;
    const uint64_t eid = ra.env_id0 + (uint64_t)env;

    double s[D];
#pragma unroll
    for (int d = 0; d < D; ++d) s[d] = phys ? state[(size_t)d * n + env] : 0.0;
    bool need = phys ? need_reset[env] != 0 : false;
    bool prev_done = true;  // no value_next write before step 0

    for (int t = 0; t < ra.T; ++t) {
        const uint64_t gstep = ra.step0 + (uint64_t)t;
        const size_t k = (size_t)t * n + env;
        if (phys && need) {
            E::reset(p, s, ra.seed, gstep, eid);
            need = false;
        }
        float o[S];
        E::observe(p, s, o);
        if (lane < WENV) {
#pragma unroll
            for (int j = 0; j < 8; ++j) sobs[wave][lane][j] = (phys && j < S) ? o[j] : 0.f;
        }
        wave_sync();
        float bobs[SUB][KS1];
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
            for (int kk = 0; kk < KS1; ++kk) bobs[sb][kk] = sobs[wave][16 * sb + e][4 * kk + g];
        wave_sync();

        // actor then critic through ONE copy of the fused forward (one register allocation)
        float mraw[A], v = 0.f;
#pragma unroll 1
        for (int which = 0; which < 2; ++which) {
            float out[SUB][A];
            if constexpr (X3)
                mlp_x3_forward<H, SUB, KS1, A>(which ? critic : actor, which ? small_c : small_a,
                                               ring, which ? cn : an, which ? 1 : A, bobs, out);
            else
                mlp_fused_forward<H, SUB, KS1, A, RING>(which ? critic : actor,
                                                        which ? small_c : small_a, ring,
                                                        which ? cn : an, which ? 1 : A, bobs, out);
            // the physics lane (sub-block g, env e) owns out[g]
            float sel[A];
#pragma unroll
            for (int a = 0; a < A; ++a) sel[a] = out[0][a];
#pragma unroll
            for (int sb = 1; sb < SUB; ++sb)
                if (g == sb) {
#pragma unroll
                    for (int a = 0; a < A; ++a) sel[a] = out[sb][a];
                }
            if (which) {
                v = sel[0];
            } else {
#pragma unroll
                for (int a = 0; a < A; ++a) mraw[a] = sel[a];
            }
        }
        if (phys) {
            float eps[A], act[A], lp[A];
            philox_normal_f32<A>(ra.seed, gstep, eid, eps);
#pragma unroll
            for (int a = 0; a < A; ++a) {
                const float m = (an.out_tanh ? tanhf(mraw[a]) : mraw[a]) * ra.gain[a] + ra.off[a];
                float x = m + ra.std_[a] * eps[a];
                x = fmaxf(fminf(x, ra.a_max[a]), ra.a_min[a]);
                act[a] = x;
                lp[a] = normal_logp_c(x, m, ra.half_inv_var[a], ra.log_std[a]);
            }
            float on[S];
            double r;
            int f;
            bool dn;
            E::step(p, s, act, on, r, f, dn);
#pragma unroll
            for (int j = 0; j < S; ++j) {
                b.obs[k * S + j] = o[j];
                b.obs_next[k * S + j] = on[j];
            }
#pragma unroll
            for (int a = 0; a < A; ++a) {
                b.action[k * A + a] = act[a];
                b.logp[k * A + a] = lp[a];
            }
            b.reward[k] = (float)r;
            b.value[k] = v;
            b.done[k] = dn;
            b.success[k] = success_of(ra.success_rule, ra.success_flag, dn, f);
            b.flag[k] = (int8_t)f;
            if (!prev_done) b.value_next[k - n] = v;  // V(s'_{t-1}) == V(s_t) when no reset
            prev_done = dn;
            need = dn;
        }
    }

    // bootstrap V(s'_{T-1}) for envs that did not terminate on the last step
    float o[S];
    E::observe(p, s, o);
    if (lane < WENV) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sobs[wave][lane][j] = (phys && j < S) ? o[j] : 0.f;
    }
    wave_sync();
    float bobs[SUB][KS1];
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
        for (int kk = 0; kk < KS1; ++kk) bobs[sb][kk] = sobs[wave][16 * sb + e][4 * kk + g];
    float cv[SUB][A];
    if constexpr (X3)
        mlp_x3_forward<H, SUB, KS1, A>(critic, small_c, ring, cn, 1, bobs, cv);
    else
        mlp_fused_forward<H, SUB, KS1, A, RING>(critic, small_c, ring, cn, 1, bobs, cv);
    float v = cv[0][0];
#pragma unroll
    for (int sb = 1; sb < SUB; ++sb)
        if (g == sb) v = cv[sb][0];
    if (phys) {
        if (!prev_done) b.value_next[(size_t)(ra.T - 1) * n + env] = v;
#pragma unroll
        for (int d = 0; d < D; ++d) state[(size_t)d * n + env] = s[d];
        need_reset[env] = need ? 1 : 0;
    }
}

// ------------------------------------------------------------------------------------------
// Shared-physics variant of the f16x3 rollout (rollout_sp_kernel): the block's envs keep their
// f64 state in LDS instead of one wave's registers, and each step's physics (sampling, RK4,
// reward/terminal, buffer stores, auto-reset) runs on FULL 64-lane waves — EB/64 of the block's
// waves per step, the role rotating over the waves so every SIMD gets the same share. In the
// register-resident kernel a 32-env wave runs the f64 physics on 32 of its 64 lanes: half of the
// VALU issue the physics costs (the kernel's binding resource) is idle lanes.
// Per step: [all waves] obs from LDS -> actor + critic (shared W2 chunk ring) -> (mean, V) to LDS
// | block barrier | [physics waves] sample, step, stores, reset, next obs to LDS | block barrier.
// Same arithmetic, same Philox counters and the same reset points as rollout_kernel: a finished
// env is reset right after its terminal step with the next step's counter (rollout_kernel does it
// at the start of that step), except after the segment's last step, where need_reset carries it.
// ------------------------------------------------------------------------------------------
template <int KIND, int SUB, int RG, int W = 4>
constexpr int rollout_sp_lds_bytes() {
    using E = Env<KIND>;
    constexpr int KS1 = (E::S + 3) / 4, EB = W * 16 * SUB;
    return 4 * (2 * mlp_small_floats<256, KS1, E::A>() + EB * 8 + EB * (E::A + 1) + RG * kX3ChunkFloats) +
           8 * E::D * EB + 2 * EB;
}
constexpr int kSpRing1 = 3;  // W2 ring slots of the one-block-per-CU variants (4 measured 1 % slower)
constexpr int kSpCpb1 = 2;   // 16-KiB chunks per ring slot / block barrier there (one barrier per k-phase)
// UAV physics lanes per physics wave: 64 (half waves, 32, measured 6 % slower: the UAV step is
// issue-bound, not latency-bound, so spreading it over more waves only adds issue)
// waves per SIMD of a variant: 4-wave blocks 2 (two blocks per CU, or one per CU with WPS = 1 and
// 512 registers); 8-wave blocks of 32-env waves 2 (one block per CU)
template <int SUB, int W, int WPS>
constexpr int rollout_sp_blocks_per_cu() { return 4 * WPS / W; }
// the CU's 160 KiB split over its blocks: a 3-chunk W2 ring where it fits, else 2 (UAV)
template <int KIND, int SUB, int W = 4, int WPS = 2>
constexpr int rollout_sp_ring() {
    constexpr int bpc = rollout_sp_blocks_per_cu<SUB, W, WPS>(), budget = 160 * 1024 / bpc;
    return bpc == 1 && rollout_sp_lds_bytes<KIND, SUB, kSpRing1 * kSpCpb1, W>() <= budget
               ? kSpRing1
         : rollout_sp_lds_bytes<KIND, SUB, 3, W>() <= budget ? 3
         : rollout_sp_lds_bytes<KIND, SUB, 2, W>() <= budget ? 2 : 0;
}
template <int KIND, int SUB>
constexpr bool rollout_sp_fits() { return SUB <= 2 && rollout_sp_ring<KIND, SUB>() != 0; }

// W = 4: 4-wave blocks, two per CU (2 waves per SIMD, <= 256 registers) or, WPS = 1, one per CU
// (1 wave per SIMD, 512 registers); W = 8, SUB = 2: ONE 8-wave block per CU (2 waves per SIMD,
// 256 registers). (8-wave blocks of 16-env waves, 2 or 4 waves per SIMD, and 4-wave blocks of
// 64-env waves measured slower and were removed: DESIGN.md §4.) Two co-resident 4-wave blocks do not share a CU fairly: the SQ's
// oldest-first issue arbitration lets one run ahead (measured: half the blocks finish their
// segment in 12.0M cycles, the other half in 16.9M, and the launch waits for the slow half); in
// one block the barriers keep all eight waves in step.
// The launch's arguments as ONE kernel parameter, so that the kernel can address them in the
// kernarg segment (__builtin_amdgcn_kernarg_segment_ptr) and re-read the env params, launch
// constants and buffer pointers per step with scalar loads instead of holding them in SGPRs across
// the MLP passes (which spilled them to VGPR lanes: a v_readlane per use, 248 in the CartPole
// kernel, 901 in the UAV kernel).
template <int KIND>
struct SpArgs {
    typename Env<KIND>::P p;
    double *state;
    uint8_t *need_reset;
    const float *actor;
    MfmaNet an;
    const float *critic;
    MfmaNet cn;
    RolloutArgs ra;
    rlp_rollout_bufs b;
};

template <int KIND, int H, int SUB, int W = 4, int WPS = 2>
__global__ void __launch_bounds__(64 * W, WPS)  // (HIP's second argument: waves per SIMD)
rollout_sp_kernel(SpArgs<KIND> args) {
    const typename Env<KIND>::P &p = args.p;
    double *__restrict__ state = args.state;
    uint8_t *__restrict__ need_reset = args.need_reset;
    const float *__restrict__ actor = args.actor;
    const float *__restrict__ critic = args.critic;
    const MfmaNet &an = args.an, &cn = args.cn;
    const RolloutArgs &ra = args.ra;
    const rlp_rollout_bufs &b = args.b;
    using E = Env<KIND>;
    constexpr int S = E::S, A = E::A, D = E::D, KS1 = (S + 3) / 4, WENV = 16 * SUB;
    constexpr int PHL = 64;  // physics lanes per physics wave
    constexpr int WAVES = W, EB = WAVES * WENV, PW = EB / PHL, ROT = WAVES / PW;
    static_assert(EB % PHL == 0 && WAVES % PW == 0, "physics waves cover the block's envs");
    constexpr int SMALL = mlp_small_floats<H, KS1, A>(), RG = rollout_sp_ring<KIND, SUB, W, WPS>();
    // one block per CU: ring slots of kSpCpb1 chunks (fewer block barriers per k-phase)
    constexpr int CPB = rollout_sp_blocks_per_cu<SUB, W, WPS>() == 1 &&
                                rollout_sp_lds_bytes<KIND, SUB, RG * kSpCpb1, W>() <= 160 * 1024
                            ? kSpCpb1 : 1;
    __shared__ __attribute__((aligned(16))) float lds[2 * SMALL + EB * 8 + EB * (A + 1) + RG * CPB * kX3ChunkFloats];
    __shared__ double st[D][EB];
    __shared__ uint8_t s_need[EB], s_pdone[EB];
    float *small_a = lds, *small_c = lds + SMALL;
    float(*sob)[8] = reinterpret_cast<float(*)[8]>(lds + 2 * SMALL);
    float(*mv)[A + 1] = reinterpret_cast<float(*)[A + 1]>(lds + 2 * SMALL + EB * 8);
    float *ring = lds + 2 * SMALL + EB * 8 + EB * (A + 1);
    mlp_small_to_lds(actor, an, small_a, true);
    mlp_small_to_lds(critic, cn, small_c, true);

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, e = lane & 15;
    const int n = ra.n;
    const int base = blockIdx.x * EB;

    // state -> LDS; the first step's resets and observations (threads 0..EB-1, one env each)
    for (int i = threadIdx.x; i < D * EB; i += blockDim.x) {
        const int d = i / EB, le = i % EB;
        st[d][le] = base + le < n ? state[d * n + base + le] : 0.0;
    }
    __syncthreads();
    if (threadIdx.x < EB) {
        const int le = threadIdx.x, env = base + le;
        double s[D];
#pragma unroll
        for (int d = 0; d < D; ++d) s[d] = st[d][le];
        float o[S];
        if (env < n && need_reset[env]) {
            E::reset(p, s, ra.seed, ra.step0, ra.env_id0 + (uint64_t)env);
#pragma unroll
            for (int d = 0; d < D; ++d) st[d][le] = s[d];
        }
        E::observe(p, s, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) sob[le][j] = (env < n && j < S) ? o[j] : 0.f;
        s_need[le] = 0;
        s_pdone[le] = 1;  // no value_next write before step 0
    }
    __syncthreads();

    auto mlp_pass = [&](bool both) {
        // the nets' pointers and layouts re-read from the kernarg segment (scalar loads) per pass
        auto ak = (const __attribute__((address_space(4))) SpArgs<KIND> *)
            __builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ak));
        const float *actor = ak->actor, *critic = ak->critic;
        const MfmaNet &an = *(const MfmaNet *)&ak->an, &cn = *(const MfmaNet *)&ak->cn;
        float bobs[SUB][KS1];
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
            for (int kk = 0; kk < KS1; ++kk) bobs[sb][kk] = sob[WENV * wave + 16 * sb + e][4 * kk + g];
#pragma unroll 1
        for (int which = both ? 0 : 1; which < 2; ++which) {
            float out[SUB][A];
            mlp_x3_forward<H, SUB, KS1, A, RG, W, CPB>(which ? critic : actor, which ? small_c : small_a,
                                                  ring, which ? cn : an, which ? 1 : A, bobs, out);
            // lane (sub-block g, env e) owns out[g]
            float sel[A];
#pragma unroll
            for (int a = 0; a < A; ++a) sel[a] = out[0][a];
#pragma unroll
            for (int sb = 1; sb < SUB; ++sb)
                if (g == sb) {
#pragma unroll
                    for (int a = 0; a < A; ++a) sel[a] = out[sb][a];
                }
            if (lane < WENV) {
                if (which) {
                    mv[WENV * wave + lane][A] = sel[0];
                } else {
#pragma unroll
                    for (int a = 0; a < A; ++a) mv[WENV * wave + lane][a] = sel[a];
                }
            }
        }
    };

    for (int t = 0; t < ra.T; ++t) {
        const uint64_t gstep = ra.step0 + (uint64_t)t;
        mlp_pass(true);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // (mean, V) of every env
        if (wave / PW == t % ROT && lane < PHL) {  // this step's physics waves
            const int le = PHL * (wave % PW) + lane, env = base + le;
            // the env params, launch constants and buffer pointers are read through opaque
            // pointers into the kernarg segment here (s_load per step) instead of being held in
            // SGPRs across the MLP passes, which spilled them to VGPR lanes (a v_readlane per use)
            auto ak = (const __attribute__((address_space(4))) SpArgs<KIND> *)
                __builtin_amdgcn_kernarg_segment_ptr();
            asm volatile("" : "+s"(ak));
            const typename E::P &p = *(const typename E::P *)&ak->p;
            const RolloutArgs &ra = *(const RolloutArgs *)&ak->ra;
            const rlp_rollout_bufs &b = *(const rlp_rollout_bufs *)&ak->b;
            if (env < n) {
                const uint64_t eid = ra.env_id0 + (uint64_t)env;
                const int k = t * n + env;  // 32-bit: T * n * 8 < 2^31 (rlp_rollout)
                double s[D];
#pragma unroll
                for (int d = 0; d < D; ++d) s[d] = st[d][le];
                float o[S], eps[A], act[A], lp[A];
#pragma unroll
                for (int j = 0; j < S; ++j) o[j] = sob[le][j];
                const float v = mv[le][A];
                philox_normal_f32<A>(ra.seed, gstep, eid, eps);
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    const float mr = mv[le][a];
                    const float m = (an.out_tanh ? tanhf(mr) : mr) * ra.gain[a] + ra.off[a];
                    float x = m + ra.std_[a] * eps[a];
                    x = fmaxf(fminf(x, ra.a_max[a]), ra.a_min[a]);
                    act[a] = x;
                    lp[a] = normal_logp_c(x, m, ra.half_inv_var[a], ra.log_std[a]);
                }
                float on[S];
                double r;
                int f;
                bool dn;
                E::step(p, s, act, on, r, f, dn);
#pragma unroll
                for (int j = 0; j < S; ++j) {
                    b.obs[k * S + j] = o[j];
                    b.obs_next[k * S + j] = on[j];
                }
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    b.action[k * A + a] = act[a];
                    b.logp[k * A + a] = lp[a];
                }
                b.reward[k] = (float)r;
                b.value[k] = v;
                b.done[k] = dn;
                b.success[k] = success_of(ra.success_rule, ra.success_flag, dn, f);
                b.flag[k] = (int8_t)f;
                if (!s_pdone[le]) b.value_next[k - n] = v;  // V(s'_{t-1}) == V(s_t) when no reset
                s_pdone[le] = dn;
                if (dn && t + 1 < ra.T) {  // the next step's reset (rollout_kernel: at its start)
                    E::reset(p, s, ra.seed, gstep + 1, eid);
                    E::observe(p, s, on);
                } else {
                    s_need[le] = dn;
                }
#pragma unroll
                for (int d = 0; d < D; ++d) st[d][le] = s[d];
#pragma unroll
                for (int j = 0; j < S; ++j) sob[le][j] = on[j];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // next observations
    }

    // bootstrap V(s'_{T-1}) for envs that did not terminate on the last step
    mlp_pass(false);
    __syncthreads();
    if (threadIdx.x < EB) {
        const int le = threadIdx.x, env = base + le;
        if (env < n) {
            if (!s_pdone[le]) b.value_next[(ra.T - 1) * n + env] = mv[le][A];
#pragma unroll
            for (int d = 0; d < D; ++d) state[d * n + env] = st[d][le];
            need_reset[env] = s_need[le];
        }
    }
}

// ------------------------------------------------------------------------------------------
// Packed-net forward over rows (evaluate(), learn()'s V(s) / V(s'), the value fix-up).
// Exact f32 (X3 = false): each wave walks 16*SUB-row groups (grid-stride, its own W2 ring); with a
// row predicate, groups without an active row are skipped wave-uniformly. f16x3 (X3 = true): the
// hidden layer on the rollout's split (mlp_x3_forward), the block's 4 waves sharing one W2 chunk
// ring, so the block walks 4 groups at a time (block-uniform trip count and skips).
// ------------------------------------------------------------------------------------------
template <int H, int SUB, int KS1, int NOUT, int MODE, bool X3>  // MODE 0: all rows; 1: done && !success
__global__ void __launch_bounds__(256, (SUB == 4 ? 1 : 2))
packed_forward_kernel(const float *__restrict__ P, MfmaNet net, const float *__restrict__ x,
                      float *__restrict__ y, int64_t rows, const uint8_t *__restrict__ done,
                      const uint8_t *__restrict__ success, int apply_out_act) {
    constexpr int WROWS = 16 * SUB;
    constexpr int SMALL = mlp_small_floats<H, KS1, NOUT>(), PF = mlp_phase_floats<H>();
    static_assert(4 * RING * PF == kX3RingFloats, "one LDS carve for both arithmetics");
    __shared__ __attribute__((aligned(16))) float lds[SMALL + 4 * RING * PF];
    float *small = lds, *ring = lds + SMALL + (X3 ? 0 : (threadIdx.x >> 6) * RING * PF);
    mlp_small_to_lds(P, net, small, X3);
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane >> 4, e = lane & 15;
    const int S = net.S;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    // X3: group (bg * 4 + wave) for block-uniform bg; else the wave's own grid-stride groups
    const int64_t g0 = X3 ? (int64_t)blockIdx.x * 4 : (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    for (int64_t gb = g0; gb * WROWS < rows; gb += nwaves) {
        const int64_t grp = X3 ? gb + (threadIdx.x >> 6) : gb;
        const int64_t r0 = grp * WROWS;
        bool act_row = false;
        if (lane < WROWS && r0 + lane < rows)
            act_row = MODE == 0 ? true : (done[r0 + lane] && !success[r0 + lane]);
        if constexpr (X3) {
            if (!__syncthreads_or(act_row)) continue;  // block-uniform
        } else {
            if (!__any(act_row)) continue;  // wave-uniform
        }
        float bobs[SUB][KS1];
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
            for (int kk = 0; kk < KS1; ++kk) {
                const int64_t row = r0 + 16 * sb + e;
                const int k = 4 * kk + g;
                bobs[sb][kk] = (row < rows && k < S) ? x[row * S + k] : 0.f;
            }
        float out[SUB][NOUT];
        if constexpr (X3)
            mlp_x3_forward<H, SUB, KS1, NOUT>(P, small, ring, net, net.A, bobs, out);
        else
            mlp_fused_forward<H, SUB, KS1, NOUT, RING>(P, small, ring, net, net.A, bobs, out);
        // lane (sub-block g, row e) owns out[g]; lanes 0..WROWS-1 store their row
        float sel[NOUT];
#pragma unroll
        for (int a = 0; a < NOUT; ++a) sel[a] = out[0][a];
#pragma unroll
        for (int sb = 1; sb < SUB; ++sb)
            if (g == sb) {
#pragma unroll
                for (int a = 0; a < NOUT; ++a) sel[a] = out[sb][a];
            }
        if (act_row) {
            const int64_t row = r0 + lane;
            for (int a = 0; a < net.A; ++a)
                y[row * net.A + a] = (apply_out_act && net.out_tanh) ? tanhf(sel[a]) : sel[a];
        }
    }
}

template <int MODE, int SUB, bool X3>
static int launch_packed_forward_sub(const MfmaNet &net, const float *P, const float *x, float *y,
                                     int64_t rows, const uint8_t *done, const uint8_t *success,
                                     int apply_out_act, hipStream_t s) {
    const int64_t groups = (rows + 16 * SUB - 1) / (16 * SUB);
    int64_t blocks = (groups + 3) / 4;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) return RLP_OK;
#define RLP_PF(KS1, NOUT)                                                                       \
    packed_forward_kernel<256, SUB, KS1, NOUT, MODE, X3><<<(int)blocks, 256, 0, s>>>(         \
        P, net, x, y, rows, done, success, apply_out_act)
    if (net.ks1 == 1) {
        if (net.A == 1) RLP_PF(1, 1); else if (net.A == 2) RLP_PF(1, 2); else if (net.A == 3) RLP_PF(1, 3); else RLP_PF(1, 4);
    } else if (net.ks1 == 2) {
        if (net.A == 1) RLP_PF(2, 1); else if (net.A == 2) RLP_PF(2, 2); else if (net.A == 3) RLP_PF(2, 3); else RLP_PF(2, 4);
    } else {  // 41-44 inputs (the lidar env's nets: actor A = 2, critic A = 1)
        if (net.A == 1) RLP_PF(11, 1); else if (net.A == 2) RLP_PF(11, 2);
        else return fail(RLP_EUNSUPPORTED, "packed forward: %d inputs with %d outputs", net.S, net.A);
    }
#undef RLP_PF
    RLP_CHECK_LAUNCH("packed forward");
    return RLP_OK;
}

// exact f32: 64 rows per wave for large batches (learn()'s V(s) over a whole segment), 16 when
// that would leave CUs idle (the value fix-up); f16x3: 32 rows per wave for large batches
template <int MODE>
static int launch_packed_forward(const MfmaNet &net, const float *P, const float *x, float *y,
                                 int64_t rows, const uint8_t *done, const uint8_t *success,
                                 int apply_out_act, int prec, hipStream_t s) {
    if (net.H != 256) return fail(RLP_EUNSUPPORTED, "packed forward: hidden width %d", net.H);
    const bool big = MODE == 0 && rows >= (int64_t)64 * 4 * 2 * device_cus();
    if (prec == RLP_MLP_F16X3) {
        if (big) return launch_packed_forward_sub<MODE, 2, true>(net, P, x, y, rows, done, success, apply_out_act, s);
        return launch_packed_forward_sub<MODE, 1, true>(net, P, x, y, rows, done, success, apply_out_act, s);
    }
    if (big) return launch_packed_forward_sub<MODE, 4, false>(net, P, x, y, rows, done, success, apply_out_act, s);
    return launch_packed_forward_sub<MODE, 1, false>(net, P, x, y, rows, done, success, apply_out_act, s);
}

static int g_rollout_shared_physics = -1;  // rlp_set_rollout_physics (-1: auto)

template <int KIND, int H, int SUB, bool X3>
static int launch_rollout(const void *params, double *state, uint8_t *need_reset,
                          const float *actor, const MfmaNet &an, const float *critic,
                          const MfmaNet &cn, const RolloutArgs &ra, const rlp_rollout_bufs &b,
                          int physics, hipStream_t stream) {
    const auto &p = *static_cast<const typename Env<KIND>::P *>(params);
    constexpr int threads = rollout_block<SUB, X3>();
    constexpr int envs_per_block = threads / 64 * 16 * SUB;
    const int blocks = (ra.n + envs_per_block - 1) / envs_per_block;
    if constexpr (X3 && SUB == 2 && rollout_sp_ring<KIND, 2, 8>() != 0) {
        if (physics == 3) {  // one 8-wave block per CU, 32 envs per wave
            const int blocks8 = (ra.n + 255) / 256;
            rollout_sp_kernel<KIND, H, 2, 8><<<blocks8, 512, 0, stream>>>(SpArgs<KIND>{p, state, need_reset, actor, an, critic, cn, ra, b});
            RLP_CHECK_LAUNCH("rlp_rollout");
            return RLP_OK;
        }
    }
    if constexpr (X3 && SUB == 2 && rollout_sp_ring<KIND, 2, 4, 1>() != 0) {
        if (physics == 5) {  // one 4-wave block of 32-env waves per CU (1 wave per SIMD, 512 registers)
            const int blocks4 = (ra.n + 127) / 128;
            rollout_sp_kernel<KIND, H, 2, 4, 1><<<blocks4, 256, 0, stream>>>(SpArgs<KIND>{p, state, need_reset, actor, an, critic, cn, ra, b});
            RLP_CHECK_LAUNCH("rlp_rollout");
            return RLP_OK;
        }
    }
    if constexpr (X3 && rollout_sp_fits<KIND, SUB>()) {
        if (physics)
            rollout_sp_kernel<KIND, H, SUB><<<blocks, threads, 0, stream>>>(SpArgs<KIND>{p, state, need_reset, actor, an, critic, cn, ra, b});
        else
            rollout_kernel<KIND, H, SUB, X3><<<blocks, threads, 0, stream>>>(p, state, need_reset, actor,
                                                                         an, critic, cn, ra, b);
    } else {
        rollout_kernel<KIND, H, SUB, X3><<<blocks, threads, 0, stream>>>(p, state, need_reset, actor,
                                                                     an, critic, cn, ra, b);
    }
    RLP_CHECK_LAUNCH("rlp_rollout");
    return RLP_OK;
}

template <int KIND>
static int rollout_kind(const void *params, double *state, uint8_t *need_reset, const float *actor,
                        const MfmaNet &an, const float *critic, const MfmaNet &cn,
                        const RolloutArgs &ra, const rlp_rollout_bufs &b, int sub, int prec,
                        int physics, hipStream_t stream) {
    using E = Env<KIND>;
    if (an.S != E::S || cn.S != E::S || an.A != E::A || cn.A != 1)
        return fail(RLP_EINVAL, "rlp_rollout: net dims (S=%d,A=%d / S=%d,A=%d) != env (S=%d,A=%d)",
                    an.S, an.A, cn.S, cn.A, E::S, E::A);
    if (an.H != 256 || cn.H != 256)
        return fail(RLP_EUNSUPPORTED, "rlp_rollout: hidden width %d/%d (built for 256)", an.H, cn.H);
    if (prec == RLP_MLP_F16X3) {
        const int cus = device_cus();
        // auto: one 8-wave block of 32-env waves per CU where the envs fill every CU; else one
        // 4-wave block of 32-env waves per CU (mode 5: 1 wave per SIMD with the VGPR + AGPR
        // budget). The UAV's physics spills at 256 registers (584 B per lane at 2 waves per SIMD,
        // 112 B in mode 5), so the UAV runs mode 5 at every n (measured: 32768 envs 3.77 ->
        // 2.93 ms, 65536 envs 7.23 -> 5.84 ms; CartPole at 32768 envs 5.16 -> 4.75 ms against
        // two 4-wave blocks of 16-env waves)
        if (physics < 0) {
            const bool fill256 = (ra.n + 255) / 256 >= cus;
            if (KIND != RLP_ENV_UAV_HOVER_OUTER_LOOP && (sub == 0 || sub == 2) && fill256 &&
                rollout_sp_ring<KIND, 2, 8>() != 0)
                physics = 3;
            else if ((sub == 0 || sub == 2) && rollout_sp_ring<KIND, 2, 4, 1>() != 0)
                physics = 5;
            else
                physics = 1;
        }
        if (physics == 3 || physics == 5) sub = 2;  // the one-block-per-CU variants of 32-env waves
        if (sub == 0)  // auto: 32-env waves unless that leaves fewer than 2 blocks per CU
            sub = (ra.n + 127) / 128 < 2 * cus ? 1 : 2;
        if (sub == 1)
            return launch_rollout<KIND, 256, 1, true>(params, state, need_reset, actor, an, critic,
                                                      cn, ra, b, physics, stream);
        if (sub == 4)
            return launch_rollout<KIND, 256, 4, true>(params, state, need_reset, actor, an, critic,
                                                      cn, ra, b, physics, stream);
        return launch_rollout<KIND, 256, 2, true>(params, state, need_reset, actor, an, critic, cn,
                                                  ra, b, physics, stream);
    }
    if (sub <= 2)
        return launch_rollout<KIND, 256, 2, false>(params, state, need_reset, actor, an, critic, cn,
                                                   ra, b, physics, stream);
    return launch_rollout<KIND, 256, 4, false>(params, state, need_reset, actor, an, critic, cn, ra,
                                               b, physics, stream);
}

// ------------------------------------------------------------------------------------------
// Nets in the plain layout (cfg->net_layout = 1): any Linear stack the fused kernels do not take
// — the PPO2-SecondOrderIntegration demo's 4 -> 128 -> 64 -> 32 -> 2 actor and 4 -> 64 -> 64 -> 1
// critic (demonstration/PPO2/PPO2-4-SecondOrderIntegration/train.py:37-125). The same driver
// loop, random draws and buffers as the fused kernel, as a sequence of launches per step on the
// caller's stream (no host round trip):
//   critic V(s_t), actor tanh(z_t)       rlp_mlp_forward's kernels (exact f32 MFMA)
//   plain_step_kernel                     mean = tanh(z) gain + off, Philox eps (the fused
//                                         kernel's stream), clamp, log-prob, V(s'_{t-1}) = V(s_t)
//                                         where the env did not end at t-1, env step, buffer
//                                         append, and s_{t+1}: obs_next, or the reset (counter
//                                         step0 + t + 1) and observation of an env that ended
// and after the segment the bootstrap V(s'_{T-1}) of the envs still running.
template <int KIND>
__global__ void __launch_bounds__(256) plain_begin_kernel(typename Env<KIND>::P p, double *state,
                                                          uint8_t *need_reset, RolloutArgs ra,
                                                          float *obs) {
    using E = Env<KIND>;
    const int i = blockIdx.x * 256 + threadIdx.x, n = ra.n;
    if (i >= n) return;
    const auto &pk = *(const typename E::P *)(const __attribute__((address_space(4))) typename E::P *)
        __builtin_amdgcn_kernarg_segment_ptr();
    double s[E::D];
#pragma unroll
    for (int d = 0; d < E::D; ++d) s[d] = state[(size_t)d * n + i];
    if (need_reset[i]) {
        E::reset(pk, s, ra.seed, ra.step0, ra.env_id0 + (uint64_t)i);
#pragma unroll
        for (int d = 0; d < E::D; ++d) state[(size_t)d * n + i] = s[d];
    }
    need_reset[i] = 0;
    float o[E::S];
    E::observe(pk, s, o);
#pragma unroll
    for (int j = 0; j < E::S; ++j) obs[(size_t)i * E::S + j] = o[j];
}

template <int KIND>
__global__ void __launch_bounds__(256) plain_step_kernel(typename Env<KIND>::P p, double *state,
                                                         uint8_t *need_reset, RolloutArgs ra, int t,
                                                         rlp_rollout_bufs b) {
    using E = Env<KIND>;
    constexpr int A = E::A, S = E::S;
    const int i = blockIdx.x * 256 + threadIdx.x, n = ra.n;
    if (i >= n) return;
    const auto &pk = *(const typename E::P *)(const __attribute__((address_space(4))) typename E::P *)
        __builtin_amdgcn_kernarg_segment_ptr();
    const int k = t * n + i;
    const uint64_t eid = ra.env_id0 + (uint64_t)i, gstep = ra.step0 + (uint64_t)t;
    float eps[A], act[A];
    philox_normal_f32<A>(ra.seed, gstep, eid, eps);
#pragma unroll
    for (int a = 0; a < A; ++a) {
        const float m = b.action[k * A + a] * ra.gain[a] + ra.off[a];  // actor output tanh(z)
        float x = m + ra.std_[a] * eps[a];
        x = fmaxf(fminf(x, ra.a_max[a]), ra.a_min[a]);
        act[a] = x;
        b.action[k * A + a] = x;
        b.logp[k * A + a] = normal_logp_c(x, m, ra.half_inv_var[a], ra.log_std[a]);
    }
    if (t > 0 && !b.done[k - n]) b.value_next[k - n] = b.value[k];  // V(s'_{t-1}) == V(s_t)
    double s[E::D];
#pragma unroll
    for (int d = 0; d < E::D; ++d) s[d] = state[(size_t)d * n + i];
    float on[S];
    double r;
    int f;
    bool dn;
    E::step(pk, s, act, on, r, f, dn);
#pragma unroll
    for (int j = 0; j < S; ++j) b.obs_next[(size_t)k * S + j] = on[j];
    b.reward[k] = (float)r;
    b.done[k] = dn;
    b.success[k] = success_of(ra.success_rule, ra.success_flag, dn, f);
    b.flag[k] = (int8_t)f;
    if (t + 1 < ra.T) {
        if (dn) {  // the next step's reset (as the fused kernel: right after the terminal step)
            E::reset(pk, s, ra.seed, gstep + 1, eid);
            E::observe(pk, s, on);
        }
#pragma unroll
        for (int j = 0; j < S; ++j) b.obs[(size_t)(k + n) * S + j] = on[j];
    } else {
        need_reset[i] = dn;
    }
#pragma unroll
    for (int d = 0; d < E::D; ++d) state[(size_t)d * n + i] = s[d];
}

__global__ void __launch_bounds__(256) oa_boot_kernel(int T, int n, const float *v, rlp_rollout_bufs b) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int k = (T - 1) * n + i;
    if (!b.done[k]) b.value_next[k] = v[i];
}

// the plain path's scratch: the bootstrap V, then rlp_mlp_forward's workspace (shared by the two
// nets' forwards, which run one after the other on the stream)
inline int64_t rollout_plain_ws_bytes(const rlp_mlp_desc &ad, const rlp_mlp_desc &cd, int n) {
    const int64_t wa = rlp_mlp_forward_workspace_bytes(&ad, n), wc = rlp_mlp_forward_workspace_bytes(&cd, n);
    if (wa < 0 || wc < 0) return RLP_EINVAL;
    return ((int64_t)n * 4 + 255) / 256 * 256 + (wa > wc ? wa : wc);
}

template <int KIND>
static int rollout_plain(const void *params, double *state, uint8_t *need_reset,
                         const rlp_mlp_desc &ad, const float *actor, const rlp_mlp_desc &cd,
                         const float *critic, const RolloutArgs &ra, const rlp_rollout_bufs &b,
                         void *ws, int64_t ws_bytes, hipStream_t s) {
    using E = Env<KIND>;
    const auto &p = *static_cast<const typename E::P *>(params);
    if (ad.dims[0] != E::S || cd.dims[0] != E::S || ad.dims[ad.n_layers] != E::A ||
        cd.dims[cd.n_layers] != 1)
        return fail(RLP_EINVAL, "rlp_rollout: net dims (S=%d,A=%d / S=%d,A=%d) != env (S=%d,A=%d)",
                    ad.dims[0], ad.dims[ad.n_layers], cd.dims[0], cd.dims[cd.n_layers], E::S, E::A);
    if (ad.act[ad.n_layers - 1] != RLP_ACT_TANH)
        return fail(RLP_EUNSUPPORTED, "rlp_rollout: the actor's last layer must be tanh");
    const int n = ra.n, T = ra.T, nb = (n + 255) / 256;
    float *vb = static_cast<float *>(ws);  // the bootstrap V
    void *mws = static_cast<char *>(ws) + ((int64_t)n * 4 + 255) / 256 * 256;
    const int64_t mwb = ws_bytes - ((int64_t)n * 4 + 255) / 256 * 256;
    plain_begin_kernel<KIND><<<nb, 256, 0, s>>>(p, state, need_reset, ra, b.obs);
    int rc = RLP_OK;
    for (int t = 0; t < T && rc == RLP_OK; ++t) {
        const size_t k0 = (size_t)t * n;
        const float *obs_t = b.obs + k0 * E::S;
        rc = rlp_mlp_forward(&cd, critic, obs_t, b.value + k0, n, nullptr, mws, mwb, s);
        if (rc == RLP_OK)
            rc = rlp_mlp_forward(&ad, actor, obs_t, b.action + k0 * E::A, n, nullptr, mws, mwb, s);
        if (rc == RLP_OK) plain_step_kernel<KIND><<<nb, 256, 0, s>>>(p, state, need_reset, ra, t, b);
    }
    if (rc == RLP_OK) {  // V(s'_{T-1}) of the envs still running
        rc = rlp_mlp_forward(&cd, critic, b.obs_next + (size_t)(T - 1) * n * E::S, vb, n, nullptr,
                             mws, mwb, s);
        if (rc == RLP_OK) oa_boot_kernel<<<nb, 256, 0, s>>>(T, n, vb, b);
    }
    if (rc != RLP_OK) return rc;
    RLP_CHECK_LAUNCH("rlp_rollout (plain-layout nets)");
    return RLP_OK;
}

static int g_rollout_sub = 0;  // 0: auto
static int g_mlp_precision = RLP_MLP_F16X3;

}  // namespace rlp

using namespace rlp;

extern "C" {

int rlp_set_mlp_precision(int mode) {
    if (mode != RLP_MLP_FP32 && mode != RLP_MLP_F16X3)
        return fail(RLP_EINVAL, "rlp_set_mlp_precision: %d", mode);
    g_mlp_precision = mode;
    return RLP_OK;
}

int rlp_get_mlp_precision(void) { return g_mlp_precision; }

// tuning knob (envs per wave = 16 * sub): 0 = auto (f16x3: 1 when 32-env waves would leave fewer
// than 2 blocks per CU, else 2; f32: 2), 1 (f16x3 only), 2, 4

// tuning knob (include/rlp.h): -1 (default) = auto (3 when the envs fill every CU with a 256-env
// block, else — and always for the UAV — 5), 0 / 1 / 3 / 5 the kernel variants listed there
int rlp_set_rollout_physics(int shared) {
    if (shared < -1 || shared > 5 || shared == 2 || shared == 4)
        return fail(RLP_EINVAL, "rlp_set_rollout_physics: %d", shared);
    g_rollout_shared_physics = shared;
    return RLP_OK;
}

int rlp_set_rollout_sub(int sub) {
    if (sub < 0 || sub > 4 || sub == 3) return fail(RLP_EINVAL, "rlp_set_rollout_sub: %d", sub);
    g_rollout_sub = sub;
    return RLP_OK;
}

// per-call arithmetic (include/rlp.h): 0 = the library-wide default (rlp_set_mlp_precision),
// else RLP_MLP_* + 1
static int call_precision(int mlp_precision, int *prec, const char *what) {
    if (mlp_precision < 0 || mlp_precision > 2)
        return fail(RLP_EINVAL, "%s: mlp_precision %d (0 default, 1 fp32, 2 f16x3)", what, mlp_precision);
    *prec = mlp_precision ? mlp_precision - 1 : g_mlp_precision;
    return RLP_OK;
}

int rlp_mfma_forward(const rlp_mlp_desc *desc, const float *packed, const float *x, float *y,
                     int64_t rows, int mlp_precision, rlp_stream_t stream) {
    RLP_REQUIRE(desc && packed && x && y, "rlp_mfma_forward: null argument");
    int prec;
    if (const int rc = call_precision(mlp_precision, &prec, "rlp_mfma_forward")) return rc;
    MfmaNet net;
    if (!mfma_net_from_desc(*desc, &net))
        return fail(RLP_EUNSUPPORTED, "rlp_mfma_forward: need a [S->H->H->A] tanh MLP");
    if (rows <= 0) return rows == 0 ? RLP_OK : RLP_EINVAL;
    return launch_packed_forward<0>(net, packed, x, y, rows, nullptr, nullptr, 1, prec, as_stream(stream));
}

int rlp_value_fixup(const rlp_mlp_desc *critic_desc, const float *critic_packed,
                    const float *obs_next, const uint8_t *done, const uint8_t *success,
                    float *value_next, int64_t rows, int mlp_precision, rlp_stream_t stream) {
    RLP_REQUIRE(critic_desc && critic_packed && obs_next && done && success && value_next,
                "rlp_value_fixup: null argument");
    int prec;
    if (const int rc = call_precision(mlp_precision, &prec, "rlp_value_fixup")) return rc;
    MfmaNet net;
    if (!mfma_net_from_desc(*critic_desc, &net) || net.A != 1)
        return fail(RLP_EUNSUPPORTED, "rlp_value_fixup: need a [S->H->H->1] critic");
    if (rows <= 0) return rows == 0 ? RLP_OK : RLP_EINVAL;
    return launch_packed_forward<1>(net, critic_packed, obs_next, value_next, rows, done, success,
                                    1, prec, as_stream(stream));
}

int64_t rlp_rollout_workspace_bytes(int kind, const rlp_mlp_desc *actor_desc,
                                    const rlp_mlp_desc *critic_desc, const rlp_rollout_cfg *cfg) {
    if (!actor_desc || !critic_desc || !cfg || cfg->n < 0 || cfg->T < 1) return RLP_EINVAL;
    if (cfg->net_layout == 1) return rollout_plain_ws_bytes(*actor_desc, *critic_desc, cfg->n);
    if (cfg->net_layout != 0) return RLP_EINVAL;
    // the lidar segment kernel's argument copy; the other fused kernels need no scratch
    return kind == RLP_ENV_UGV_OBSTACLE_AVOIDANCE ? rollout_oa_workspace_bytes() : 0;
}

int rlp_rollout(int kind, const void *env_params, double *state, uint8_t *need_reset,
                const rlp_mlp_desc *actor_desc, const float *actor_packed,
                const rlp_mlp_desc *critic_desc, const float *critic_packed,
                const rlp_rollout_cfg *cfg, const rlp_rollout_bufs *bufs, rlp_stream_t stream) {
    RLP_REQUIRE(env_params && state && need_reset && actor_desc && actor_packed && critic_desc &&
                    critic_packed && cfg && bufs,
                "rlp_rollout: null argument");
    const rlp_rollout_bufs &b = *bufs;
    RLP_REQUIRE(b.obs && b.obs_next && b.action && b.logp && b.reward && b.value && b.value_next &&
                    b.done && b.success && b.flag,
                "rlp_rollout: null buffer");
    RLP_REQUIRE(cfg->T >= 1 && cfg->n >= 0, "rlp_rollout: T=%d n=%d", cfg->T, cfg->n);
    RLP_REQUIRE((int64_t)cfg->T * cfg->n * 8 <= 2147483647 && (int64_t)cfg->n * 32 <= 2147483647,
                "rlp_rollout: T*n = %lld too large for one segment (32-bit buffer indices)",
                (long long)cfg->T * cfg->n);
    if (cfg->n == 0) return RLP_OK;
    RLP_REQUIRE(cfg->net_layout == 0 || cfg->net_layout == 1, "rlp_rollout: net_layout %d",
                cfg->net_layout);
    MfmaNet an, cn;
    if (cfg->net_layout == 0 &&
        (!mfma_net_from_desc(*actor_desc, &an) || !mfma_net_from_desc(*critic_desc, &cn)))
        return fail(RLP_EUNSUPPORTED, "rlp_rollout: packed nets must be [S->H->H->A] tanh MLPs "
                                      "(net_layout = 1 takes any Linear stack)");
    RolloutArgs ra;
    ra.T = cfg->T; ra.n = cfg->n;
    ra.seed = cfg->seed; ra.step0 = cfg->step0; ra.env_id0 = cfg->env_id0;
    ra.success_rule = cfg->success_rule; ra.success_flag = cfg->success_flag;
    for (int a = 0; a < 4; ++a) {
        ra.std_[a] = cfg->std[a];
        ra.a_min[a] = cfg->a_min[a];
        ra.a_max[a] = cfg->a_max[a];
        ra.off[a] = (cfg->a_min[a] + cfg->a_max[a]) / 2.0f;  // PPOActor_Gaussian: (a_min+a_max)/2
        ra.gain[a] = cfg->a_max[a] - ra.off[a];              //                   a_max - off
        ra.log_std[a] = logf(cfg->std[a]);
        ra.half_inv_var[a] = 0.5f / (cfg->std[a] * cfg->std[a]);
    }
    hipStream_t s = as_stream(stream);
    // per-call selections (cfg, 0 = the library-wide default of the rlp_set_* knobs)
    RLP_REQUIRE(cfg->mlp_precision >= 0 && cfg->mlp_precision <= 2 && cfg->physics >= 0 &&
                    cfg->physics <= 8 && cfg->physics != 3 && cfg->physics != 5 &&
                    cfg->physics != 7 && (cfg->sub == 0 || cfg->sub == 1 || cfg->sub == 2 ||
                                          cfg->sub == 4),
                "rlp_rollout: cfg mlp_precision=%d physics=%d sub=%d", cfg->mlp_precision,
                cfg->physics, cfg->sub);
    const int sub = cfg->sub ? cfg->sub : g_rollout_sub;
    const int prec = cfg->mlp_precision ? cfg->mlp_precision - 1 : g_mlp_precision;
    const int physics = cfg->physics == 8 ? -1 : cfg->physics ? cfg->physics - 1 : g_rollout_shared_physics;
    {  // the caller's workspace, checked before any launch
        const int64_t need = rlp_rollout_workspace_bytes(kind, actor_desc, critic_desc, cfg);
        RLP_REQUIRE(need >= 0, "rlp_rollout: workspace query failed (net descs)");
        RLP_REQUIRE(cfg->workspace_bytes >= need && (need == 0 || cfg->workspace),
                    "rlp_rollout: workspace of %lld bytes, need %lld (rlp_rollout_workspace_bytes)",
                    (long long)cfg->workspace_bytes, (long long)need);
    }
    if (cfg->net_layout == 1) {
        switch (kind) {
#define RLP_PLAIN(K)                                                                              \
    case K:                                                                                       \
        return rollout_plain<K>(env_params, state, need_reset, *actor_desc, actor_packed,        \
                                *critic_desc, critic_packed, ra, b, cfg->workspace,              \
                                cfg->workspace_bytes, s);
            RLP_PLAIN(RLP_ENV_CARTPOLE)
            RLP_PLAIN(RLP_ENV_CARTPOLE_ANGLEONLY)
            RLP_PLAIN(RLP_ENV_SOI)
            RLP_PLAIN(RLP_ENV_UGV_FORWARD)
            RLP_PLAIN(RLP_ENV_UGV_BIDIRECTIONAL)
            RLP_PLAIN(RLP_ENV_UAV_HOVER_OUTER_LOOP)
#undef RLP_PLAIN
        }
        return fail(RLP_EUNSUPPORTED, "rlp_rollout: plain-layout nets for env kind %d", kind);
    }
    switch (kind) {
    case RLP_ENV_CARTPOLE:
        return rollout_kind<RLP_ENV_CARTPOLE>(env_params, state, need_reset, actor_packed, an,
                                              critic_packed, cn, ra, b, sub, prec, physics, s);
    case RLP_ENV_CARTPOLE_ANGLEONLY:
        return rollout_kind<RLP_ENV_CARTPOLE_ANGLEONLY>(env_params, state, need_reset, actor_packed,
                                                        an, critic_packed, cn, ra, b, sub, prec, physics, s);
    case RLP_ENV_SOI:
        return rollout_kind<RLP_ENV_SOI>(env_params, state, need_reset, actor_packed, an,
                                         critic_packed, cn, ra, b, sub, prec, physics, s);
    case RLP_ENV_UGV_FORWARD:
        return rollout_kind<RLP_ENV_UGV_FORWARD>(env_params, state, need_reset, actor_packed, an,
                                                 critic_packed, cn, ra, b, sub, prec, physics, s);
    case RLP_ENV_UGV_BIDIRECTIONAL:
        return rollout_kind<RLP_ENV_UGV_BIDIRECTIONAL>(env_params, state, need_reset, actor_packed,
                                                       an, critic_packed, cn, ra, b, sub, prec, physics, s);
    case RLP_ENV_UAV_HOVER_OUTER_LOOP:
        return rollout_kind<RLP_ENV_UAV_HOVER_OUTER_LOOP>(env_params, state, need_reset,
                                                          actor_packed, an, critic_packed, cn, ra,
                                                          b, sub, prec, physics, s);
    case RLP_ENV_UGV_OBSTACLE_AVOIDANCE:
        return rollout_oa(env_params, state, need_reset, actor_packed, an, critic_packed, cn, ra, b,
                          prec, cfg->workspace, cfg->workspace_bytes, s);
    }
    return fail(RLP_EINVAL, "rlp_rollout: unknown env kind %d", kind);
}

}  // extern "C"
