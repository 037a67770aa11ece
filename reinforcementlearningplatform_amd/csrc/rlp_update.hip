// rlp_update.hip — gradients of one PPO2 optimiser step on MFMA (Proximal_Policy_Optimization2.learn,
// algorithm/policy_base/Proximal_Policy_Optimization2.py:102-163) for the drivers'
// [S -> 256 -> 256 -> A] tanh actor (PPOActor_Gaussian, demonstration/PPO2/PPO2-4-CartPole/
// train.py:39-88) and critic (PPOCritic, :91-125), plus clip_grad_norm_ and torch.optim.Adam.
//
// Two kernels per net and step:
//   ppo2_fd_kernel    per 64-row tile (4 waves x 16 rows, env-on-lane like the rollout): forward
//                     z2 = W2 h1 (f16x3 through the block's W2 chunk ring), h2, z3, the loss's
//                     gradient g3 = dL/dz3 per row, dW3/db3 partials (registers), g2 = W3^T g3 *
//                     (1 - h2^2), backward dh1 = W2^T g2 (f16x3 over the W2^T chunks, per-row
//                     power-of-two scaling of g2), g1 = dh1 * (1 - h1^2), dW1/db1 partials (the
//                     g1 tile transposed through LDS); G2 -> HBM in a [tile][neuron][64 rows]
//                     layout (rows contiguous: the reduction operand of the next kernel) and
//                     max|g2| (atomicMax) for its power-of-two scale.
//   ppo2_wgrad_kernel dW2 = sum_r g2 h1^T and db2 = sum_r g2 on f16x3 MFMA with K = 32 rows per
//                     instruction (g2 split under one power-of-two scale from max|g2|; h1
//                     recomputed bit-identically from s, once per block, as LDS fragments);
//                     per-block partials.
// A deterministic reduce assembles the flat gradient (torch parameter order).
#include "rlp_mfma_x3.hpp"

namespace rlp {

constexpr int kUpdRows = 64;          // rows per block tile (4 waves x 16)
constexpr int kUpdH = 256;
constexpr int kUpdTileFloats = kUpdH * kUpdRows;

struct Ppo2Args {
    const float *packed;
    MfmaNet net;
    const float *s, *a, *lp, *adv, *vt;
    const int64_t *index;
    int64_t rows;
    float inv_rows, eps_clip, ent_row;  // ent_row = entropy_coef * sum_a entropy_a (constant)
    float std_[4], gain[4], off[4];
    float log_std[4], inv_var[4];  // per-launch constants of the Normal log-prob and its gradient
    float *g2t;         // [tiles][256][64]
    unsigned *g2max;    // bits of max|g2| (atomicMax)
    float *part3;       // [FD waves][p3]: per-wave dW3 | db3 | dW1 | db1 (EXT: dW3 | db3)
    int p3;             // floats per wave partial: A*256 + A + 256*S + 256 (EXT: A*256 + A)
    double *lpart;      // [FD waves]: per-wave loss partials (summed in order by the reduce)
    const float *h1;    // EXT: [rows][256] tanh(W1 s + b1) (exact f32, rlp_dense.hip)
    float *g1;          // EXT: [rows][256] dL/dh1 (l1_wgrad_kernel applies 1 - h1^2: dL/dz1)
};

// block barrier for LDS hand-offs only: drains this wave's LDS ops, not its global loads (HIP's
// __syncthreads also waits for vmcnt(0), which would expose prefetched loads)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// wave-level 256x256 GEMM of 16 rows through the block's chunk ring (all 4 waves call it in step):
// acc[j] += A-chunks(Xw) x B(P), B(P) = bop(P) as f16 hi/lo (rlp_mfma_x3.hpp layout). The phase
// loop is fully unrolled, so bop may read register arrays at compile-time indices; the next
// phase's B operands are prepared inside the second chunk's MFMA region.
// SWAP: the chunk fragments are the B operand and bop's the A operand (C = [rows][chunk outputs]:
// "neuron on lane" instead of "row on lane"; the register contents of both operands are the same).
// pre(P) runs at the head of phase P - 1, so its results (the forward's layer-1 MFMAs) are ready
// when bop(P) needs them half a phase later (diag_fd.py: -1.2k cycles per tile; pinning bop's VALU
// between the second chunk's MFMAs with sched_group_barrier measured within noise).
// W: waves of the block sharing the ring (each DMAs 16 / W KiB of every chunk). CPB: 16-KiB
// chunks per ring slot and block barrier (the ring holds kX3Ring x CPB chunks).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <bool SWAP = false, int W = 4, int CPB = 1, int RG = kX3Ring, class BOp, class Pre>
__device__ __forceinline__ void x3_gemm16(const gptr<float> Xw, float *ring, float *my_part,
                                          floatx4 (&acc)[16], BOp &&bop, Pre &&pre) {
    constexpr int NC = 16, NPW = 16 / W, NS = NC / CPB;
    static_assert(RG >= 3 && RG <= 6, "ring slots");
    const int lane = threadIdx.x & 63;
    auto issue = [&](int sc) {  // chunks CPB sc .. CPB sc + CPB - 1
#pragma unroll
        for (int cc = 0; cc < CPB; ++cc) {
            float *slot = my_part + ((sc % RG) * CPB + cc) * kX3ChunkFloats;
            // scalar chunk base (opaque: the unrolled loop would otherwise materialise all 64 piece
            // addresses up front) + the lane's 16 B: saddr DMA, no per-piece VALU address math
#pragma unroll
            for (int q = 0; q < NPW; ++q) {
                gptr<float> src = Xw + (sc * CPB + cc) * kX3ChunkFloats + q * 256;
                asm volatile("" : "+s"(src));
                lds_dma_1k(src + lane * 4, slot + q * 256);
            }
        }
    };
    lds_barrier();  // every wave is done with the ring
#pragma unroll
    for (int q = 0; q < RG - 1; ++q) issue(q);
    // the B operands of phase P in buffer P & 1 (the loop is unrolled: no copies between phases)
    half8 bbh[2], bbl[2];
    pre(0);
    bop(0, bbh[0], bbl[0]);
#pragma unroll
    for (int P = 0; P < 8; ++P) {
        const half8 &bh = bbh[P & 1], &bl = bbl[P & 1];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int c = 2 * P + hf;
            if (c % CPB == 0) {
                const int sc = c / CPB;
                // own part of group sc landed; the groups issued after it (up to RG - 2 of them)
                // may still be in flight
                const int newer = (sc + RG - 2 < NS ? sc + RG - 2 : NS - 1) - sc;
                if (newer >= 4) wait_vmcnt<4 * NPW * CPB>();
                else if (newer == 3) wait_vmcnt<3 * NPW * CPB>();
                else if (newer == 2) wait_vmcnt<2 * NPW * CPB>();
                else if (newer == 1) wait_vmcnt<NPW * CPB>();
                else wait_vmcnt<0>();
                block_barrier_raw();
                if (sc + RG - 1 < NS) issue(sc + RG - 1);
            }
            const float *slot = ring + (((c / CPB) % RG) * CPB + c % CPB) * kX3ChunkFloats + lane * 4;
            if (hf == 0 && P + 1 < 8) pre(P + 1);
            if (hf == 1 && P + 1 < 8) bop(P + 1, bbh[(P + 1) & 1], bbl[(P + 1) & 1]);
            // the chunk's 8 output tiles in four pairs, each pair's 4 fragments read while the
            // previous pair's 6 MFMAs run (two register buffers: the same 32 fragment registers;
            // pinned with sched_group_barrier). Same-box rocprof A/B (profiles/r3/r3s_fd_ab.txt):
            // actor / critic FD 8.25 / 8.17 -> 8.02 / 7.99 ms against two groups of four tiles,
            // each read then multiplied (s_nop hazards and exposed LDS latency; removed)
            {
                half8 fh[2][2], fl[2][2];
                auto rd = [&](int grp, int buf) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        fh[buf][u] = *reinterpret_cast<const half8 *>(slot + (2 * (2 * grp + u)) * 256);
                        fl[buf][u] = *reinterpret_cast<const half8 *>(slot + (2 * (2 * grp + u) + 1) * 256);
                    }
                };
                rd(0, 0);
                // a group of its own for rd(0): without it the first pinned read group took rd(0)'s
                // reads and every group was read, waited on and multiplied in turn (the ISA's
                // ds_read -> first-use MFMA distance: 40 of ~130 groups pipelined -> 84; FD
                // -0.5 to -1.4 %, same box, two repetitions: profiles/r5/r5ab1_fd_sgb_ab.txt)
                __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
                for (int grp = 0; grp < 4; ++grp) {
                    if (grp + 1 < 4) {
                        rd(grp + 1, (grp + 1) & 1);
                        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    }
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const half8 ah = fh[grp & 1][u], al = fl[grp & 1][u];
                        floatx4 v = acc[8 * hf + 2 * grp + u];
                        if constexpr (SWAP) {
                            v = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, ah, v, 0, 0, 0);
                            v = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl, ah, v, 0, 0, 0);
                            v = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, al, v, 0, 0, 0);
                        } else {
                            v = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, v, 0, 0, 0);
                            v = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, v, 0, 0, 0);
                            v = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, v, 0, 0, 0);
                        }
                        acc[8 * hf + 2 * grp + u] = v;
                    }
                    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
                }
            }
        }
    }
}

// packed FP32 (v_pk_mul / v_pk_add / v_pk_fma_f32: two IEEE f32 results per instruction, each
// rounded exactly as the scalar op) for the FD kernel's elementwise work (layer-1 tanh, h2 tanh and
// z3, dW3 products, g2, the backward operand scale, the g1 recompute, dW1): 2745 -> 2226 VALU per
// 16-row wave tile in the ISA, FD -0.5 to -1.2 % (profiles/r6/r6b_fd_pk_lidar_ab.txt): the kernel is
// not VALU-issue bound
__device__ __forceinline__ float2v pk(float a, float b) { return (float2v){a, b}; }
__device__ __forceinline__ float2v pk_fma(float2v a, float2v b, float2v c) {
    return __builtin_elementwise_fma(a, b, c);
}
__device__ __forceinline__ float2v pk_exp2(float2v x) {
    return (float2v){__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
}
__device__ __forceinline__ float2v pk_rcp(float2v x) {
    return (float2v){__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)};
}

// wave-scope LDS fence + barrier (the staging buffer is private to the wave)
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void split8(const float (&x)[8], half8 &bh, half8 &bl) {
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        half2v hi, lo;
        split2_mix((float2v){x[i], x[i + 1]}, hi, lo);
        bh[i] = hi.x;
        bh[i + 1] = hi.y;
        bl[i] = lo.x;
        bl[i + 1] = lo.y;
    }
}

// Cross-lane sums without LDS (the weight gradients' row reductions):
// pair_sum_rows16: x + (x of the lane in the partner set), DPP within a 16-lane row; the lanes
// whose `bit` is set keep value b, the others a (a butterfly stage: the pair's two sums).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ float pair_sum_rows16(float a, float b, bool bit) {
    const float keep = bit ? b : a, send = bit ? a : b;
    return dpp_f<CTRL>(send) + keep;
}
// the same across 16-lane rows: lanes 0-31 (even rows) keep a, 32-63 (odd rows) keep b
__device__ __forceinline__ float pair_sum_x32(float a, float b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float pair_sum_x16(float a, float b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
constexpr int kDppRowMirror = 0x140, kDppHalfMirror = 0x141, kDppXor2 = 0x4E, kDppXor1 = 0xB1;

// LDS of one FD block (floats): [ W2 ring (3 x 16 KiB) | small weights | srw | dW1 partials ].
// One 8-wave block per CU (2 waves per SIMD; a block iteration covers 2 G2 tiles of 64 rows): half
// the W2 DMA per CU of two 4-wave blocks. The 8-wave block is ~2 % slower per wave tile
// (diag_fd.py: its barriers span 8 waves) but 4-5 % faster per launch: two co-resident 4-wave blocks
// do not get equal shares of the CU (oldest-first issue arbitration) and the launch waits for the
// slower half; a tile queue (atomic counter) instead of the static grid stride recovered only half
// of that. Measured and removed: 4-wave blocks (two per CU, or one per CU for the
// actor's and critic's FD on two streams), 2 chunks per ring slot (the actor's FD spilled 56 B),
// the second half of each block's waves at s_setprio 1.
constexpr int kFdWaves = 8;
constexpr int kFdRows = 16 * kFdWaves;
constexpr int kFdRing = 4;  // W2 chunk-ring slots (two chunks in flight while one is read; 3: the
                            // lidar nets' FD 2 % slower, the CartPole nets' the same, r5o_fd_ring_ab.txt)

// KS1 = 0 ("EXT", the lidar demos' 41-input nets): layer 1 lives outside the kernel — h1 =
// tanh(W1 s + b1) comes from g.h1 (one exact-f32 GEMM per step, rlp_dense.hip), g1 = dL/dz1 goes to
// g.g1 for the dense dW1 | db1 GEMM; the kernel keeps the 256 x 256 layer's f16x3 forward and
// backward, the loss head and dW3 | db3. (Eleven f32 K-steps of layer 1 in-kernel, twice per tile,
// would cost as much MFMA pipe as the f16 GEMMs, and dW1's 256 x 42 partials do not fit in registers.)
template <int KS1, int A, int LOSS>
__global__ void __launch_bounds__(64 * kFdWaves, 1) ppo2_fd_kernel(Ppo2Args g) {
    constexpr bool EXT = KS1 == 0;
    constexpr int KS = EXT ? 1 : KS1;
    constexpr int H = kUpdH, SMALL = EXT ? 2 * H + A * H + 8 : mlp_small_floats<H, KS1, A>();
    constexpr int NC = 4 * KS + 1;  // dW1 columns per neuron: s features | bias
    constexpr int kFdRegion = kFdRing * kX3ChunkFloats;
    __shared__ __attribute__((aligned(16))) float lds[kFdRegion + SMALL + (EXT ? 4 : kFdWaves * 16 * 8 + 4 * H)];
    float *ring = lds, *small = lds + kFdRegion;
    // b1 x 2/ln 2 four times per neuron: the g1 recompute's swapped layer-1 tiles take their C
    // operand {b1, b1, b1, b1} with one read (a broadcast from registers cost 4 v_mov per tile)
    float *const b1q = lds + kFdRegion + SMALL + kFdWaves * 16 * 8;
    // the wave index as a scalar (readfirstlane): every wave-derived offset, the G2 tile and its
    // store guard become SGPR values (no per-lane 64-bit address arithmetic, no exec-masked stores)
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float *const srw = lds + kFdRegion + SMALL + (EXT ? 0 : wv * 128);  // [16 rows][8]
    const MfmaNet &net = g.net;
    // small_r: W1, b1 x 2/ln 2, b2 x 2^(sw+SH) (EXT: from b1 on, W1 is not used)
    const int sb = EXT ? net.off_b1 : net.off_w1;
    {
        const gptr<float> src = as_global(g.packed) + net.off_small_r + (sb - net.off_w1);
        for (int i = threadIdx.x; i < net.small_count - (sb - net.off_w1); i += blockDim.x) small[i] = src[i];
        if constexpr (!EXT)
            for (int i = threadIdx.x; i < 4 * H; i += blockDim.x) b1q[i] = src[(net.off_b1 - sb) + i / 4];
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, gq = lane >> 4, e = lane & 15;
    const int S = net.S;
    const float *info = small + (net.off_info - sb);
    const float sw = info[0];
    const float k_out = 2.8853900817779268f * info[2];
    float *const my_part = ring + wv * (16 / kFdWaves) * 256;
    float dW3p[A][4];  // neurons 16 e + 4 gq + m (the row butterfly's result)
    float db3p[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
        db3p[a] = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) dW3p[a][c] = 0.f;
    }
    double lsum = 0.0;
    float dW1p[2][2 * NC];  // [h][i]: neuron 16 (8 h + 2 gq + i / NC) + e, column i % NC
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2 * NC; ++i) dW1p[h][i] = 0.f;
    float g2max = 0.f;
    floatx4 dh1[16];  // dh1 -> g1 of the wave's tile

    // the small weights are re-read from LDS per use, not hoisted into registers (an opaque offset
    // keeps the LDS address space; a pointer would go FLAT)
    auto small_at = [&](int off) {
        int smo = 0;
        asm volatile("" : "+s"(smo));
        return small + smo + off;
    };
    // layer 1 of neuron tile t "neuron on lane": C[row 4 gq + q][neuron 16 t + e] (operands swapped)
    auto layer1_t = [&](int t, const float (&bo)[KS]) {
        const float *W1c = small + 0;
        float w1[KS];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) w1[kk] = W1c[w1r_index(16 * t + e, 4 * kk + gq, KS)];
        floatx4 c = *reinterpret_cast<const floatx4 *>(b1q + 4 * (16 * t + e));
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
            c = __builtin_amdgcn_mfma_f32_16x16x4f32(bo[kk], w1[kk], c, 0, 0, 0);
        return c;
    };
    // dW1 | db1 += sum_rows g1 [s | 1]^T: the lane's 4 rows in registers (s rows from srw), then
    // the 4 lane groups by a 2-stage permlane butterfly, per half of the neuron tiles
    // (8 NC -> 2 NC values)
    auto dw1_acc = [&](const float *srw) {
        float sv[4][4 * KS];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) {
                const floatx4 v = *reinterpret_cast<const floatx4 *>(srw + (4 * gq + q) * 8 + 4 * kk);
#pragma unroll
                for (int u = 0; u < 4; ++u) sv[q][4 * kk + u] = v[u];
            }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float v[8 * NC];
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) {
                const floatx4 gt = dh1[8 * h + tt];
#pragma unroll
                for (int f = 0; f < 4 * KS; f += 2) {  // two features per packed op
                    float2v x = pk(gt[0], gt[0]) * pk(sv[0][f], sv[0][f + 1]);
#pragma unroll
                    for (int q = 1; q < 4; ++q) x = pk_fma(pk(gt[q], gt[q]), pk(sv[q][f], sv[q][f + 1]), x);
                    v[tt * NC + f] = x.x;
                    v[tt * NC + f + 1] = x.y;
                }
                v[tt * NC + 4 * KS] = (gt[0] + gt[1]) + (gt[2] + gt[3]);
            }
#pragma unroll
            for (int i = 0; i < 4 * NC; ++i) v[i] = pair_sum_x32(v[i], v[i + 4 * NC]);
#pragma unroll
            for (int i = 0; i < 2 * NC; ++i) dW1p[h][i] += pair_sum_x16(v[i], v[i + 2 * NC]);
        }
    };

    const int64_t nbt = (g.rows + kFdRows - 1) / kFdRows;  // block tiles of kFdRows rows
    for (int64_t bt = blockIdx.x; bt < nbt; bt += gridDim.x) {
        const int64_t tile = bt * (kFdWaves / 4) + (wv >> 2);  // this wave's 64-row G2 tile
        // opaque per iteration: keeps the 2 x 64 chunk addresses from being hoisted (and spilled)
        const float *Pg = g.packed;
        asm volatile("" : "+s"(Pg));
        const gptr<float> Xf = as_global(Pg) + net.off_x3 + wv * (16 / kFdWaves) * 256;
        const gptr<float> Xb = as_global(Pg) + net.off_x3t + wv * (16 / kFdWaves) * 256;
        auto *g2base = (__attribute__((address_space(1))) float *)g.g2t;
        asm volatile("" : "+s"(g2base));
        // the small weights are re-read from LDS per use, not hoisted into registers
        int smo = 0;  // (an opaque offset keeps the LDS address space; a pointer would go FLAT)
        asm volatile("" : "+s"(smo));
        const float *sm = small + smo;
        const float *W1c = sm;
        const float *B1c = sm + (net.off_b1 - sb);
        const float *B2c = sm + (net.off_b2 - sb);
        const float *W3c = sm + (net.off_w3 - sb);
        const float *b3c = sm + (net.off_b3 - sb);
        const int64_t r = bt * kFdRows + 16 * wv + e;
        const bool valid = r < g.rows;
        const int64_t src = valid ? (g.index ? g.index[r] : r) : 0;
        float bobs[KS];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            const int k = 4 * kk + gq;
            if constexpr (EXT) {
                bobs[kk] = 0.f;
            } else {
                bobs[kk] = (valid && k < S) ? g.s[src * S + k] : 0.f;
                srw[e * 8 + k] = bobs[kk];  // this wave's s rows, for dW1
            }
        }
        // EXT: this lane's h1 row (rows past the end read row 0: their g3 is zero)
        const float *h1r = EXT ? g.h1 + (size_t)src * H : nullptr;
        // the actor loss's row inputs, loaded now so that their latency hides under the forward
        // GEMM (the critic's one v_target stays at its use: held across the GEMMs it spilled)
        float in_a[A], in_lp[A], in_adv = 0.f;
#pragma unroll
        for (int a = 0; a < A; ++a) in_a[a] = in_lp[a] = 0.f;
        if constexpr (LOSS == RLP_LOSS_ACTOR) {
            if (valid) {
                in_adv = g.adv[src];
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    in_a[a] = g.a[src * A + a];
                    in_lp[a] = g.lp[src * A + a];
                }
            }
        }
        auto layer1 = [&](int t) {
            float w1[KS];
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) w1[kk] = W1c[w1r_index(16 * t + e, 4 * kk + gq, KS)];
            floatx4 c = *reinterpret_cast<const floatx4 *>(B1c + 16 * t + 4 * gq);
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
                c = __builtin_amdgcn_mfma_f32_16x16x4f32(w1[kk], bobs[kk], c, 0, 0, 0);
            return c;
        };

        // ---- forward: z2 (scaled by 2^(sw+SH)) = W2 h1 + b2
        floatx4 acc[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = *reinterpret_cast<const floatx4 *>(B2c + 16 * j + 4 * gq);
        floatx4 p0, p1;  // layer-1 tiles of the next phase (pre), consumed by its B operands (bop)
        // EXT: phase P's h1 quads in buffer P & 1, loaded two phases ahead (one phase ahead — half a
        // phase before bop — left the global load latency exposed)
        floatx4 q0[2], q1[2];
        x3_gemm16<false, kFdWaves, 1, kFdRing>(Xf, ring, my_part, acc, [&](int P, half8 &bh, half8 &bl) {
            if constexpr (EXT) {
                p0 = q0[P & 1];
                p1 = q1[P & 1];
            }
            float x[8];
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                const float2v pre = i < 4 ? pk(p0[i], p0[i + 1]) : pk(p1[i - 4], p1[i - 3]);
                float2v xv;
                if constexpr (EXT) {
                    xv = pre * kX3HScale;  // h1 itself (exact power-of-two scale)
                } else {  // pre = 2 h1 / ln 2 (small_r)
                    const float2v rc = pk_rcp(pk_exp2(pre) + 1.0f);
                    xv = pk_fma(rc, pk(-2.0f * kX3HScale, -2.0f * kX3HScale), pk(kX3HScale, kX3HScale));
                }
                x[i] = xv.x;
                x[i + 1] = xv.y;
            }
            split8(x, bh, bl);
        }, [&](int P) {
            if constexpr (EXT) {  // neurons 32 Q + 4 gq .. + 3 and 32 Q + 16 + 4 gq .. + 3 of the row
                auto ld = [&](int Q) {
                    q0[Q & 1] = *reinterpret_cast<const floatx4 *>(h1r + 32 * Q + 4 * gq);
                    q1[Q & 1] = *reinterpret_cast<const floatx4 *>(h1r + 32 * Q + 16 + 4 * gq);
                };
                if (P == 0) ld(0);   // (pre(0) runs just before bop(0))
                if (P + 1 < 8) ld(P + 1);
            } else {
                p0 = layer1(2 * P);
                p1 = layer1(2 * P + 1);
            }
        });
        // ---- h2 = tanh(z2), z3 = W3 h2 + b3 (every lane group ends with its row's z3)
        float z3[A];
        float2v z3p[A];  // two partial sums per output (even / odd neurons of each quad)
#pragma unroll
        for (int a = 0; a < A; ++a) z3p[a] = pk(0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            floatx4 w3[A];
#pragma unroll
            for (int a = 0; a < A; ++a) w3[a] = *reinterpret_cast<const floatx4 *>(W3c + a * H + 16 * j + 4 * gq);
#pragma unroll
            for (int q = 0; q < 4; q += 2) {
                const float2v rc = pk_rcp(pk_exp2(pk(acc[j][q], acc[j][q + 1]) * k_out) + 1.0f);
                const float2v h = pk_fma(pk(-2.0f, -2.0f), rc, pk(1.0f, 1.0f));
                acc[j][q] = h.x;
                acc[j][q + 1] = h.y;
#pragma unroll
                for (int a = 0; a < A; ++a) z3p[a] = pk_fma(pk(w3[a][q], w3[a][q + 1]), h, z3p[a]);
            }
        }
#pragma unroll
        for (int a = 0; a < A; ++a) z3[a] = z3p[a].x + z3p[a].y;
#pragma unroll
        for (int a = 0; a < A; ++a) {
            z3[a] += __shfl_xor(z3[a], 16);
            z3[a] += __shfl_xor(z3[a], 32);
            z3[a] += b3c[a];
        }
        // ---- head gradient g3 = dL/dz3 of this row (mean over rows folded in)
        float g3[A];
        float lrow = 0.f;
        if constexpr (LOSS == RLP_LOSS_ACTOR) {
            float t[A], d[A], lp_now = 0.f, lp_old = 0.f;
            const float adv = in_adv;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                t[a] = tanhf(z3[a]);
                const float mean = t[a] * g.gain[a] + g.off[a];
                const float act = valid ? in_a[a] : mean;
                d[a] = act - mean;
                // Normal(mean, std).log_prob(act) (torch's expression, the division by 2 var and
                // log(std) as launch constants)
                lp_now += -(d[a] * d[a]) * (0.5f * g.inv_var[a]) - g.log_std[a] - 0.91893853320467274178f;
                lp_old += in_lp[a];
            }
            const float ratio = expf(lp_now - lp_old);
            const float lo = 1.f - g.eps_clip, hi = 1.f + g.eps_clip;
            const float s1 = ratio * adv;
            const float rc = fminf(fmaxf(ratio, lo), hi);
            const float s2 = rc * adv;
            // torch.min backward: the smaller operand takes the gradient, a tie splits it
            const float w1 = s1 < s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
            const float w2 = s2 < s1 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
            const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;  // clamp backward
            const float dl_dratio = -adv * (w1 + w2 * inr);
            const float dl_dlp = dl_dratio * ratio * g.inv_rows;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                g3[a] = valid ? dl_dlp * (d[a] * g.inv_var[a]) * g.gain[a] * (1.f - t[a] * t[a]) : 0.f;
            }
            lrow = valid ? -fminf(s1, s2) - g.ent_row : 0.f;
        } else {
            const float v = z3[0];
            const float diff = valid ? v - g.vt[src] : 0.f;
            g3[0] = 2.f * diff * g.inv_rows;
            lrow = diff * diff;
        }
        if (gq == 0) {
            lsum += (double)lrow;
#pragma unroll
            for (int a = 0; a < A; ++a) db3p[a] += g3[a];
        }
        // ---- dW3 = sum_rows g3 h2^T: the 64 products g3 h2 of the lane's row, summed over the 16
        // rows of its lane group by a 4-stage DPP butterfly (64 -> 4 values: neurons 16 e + 4 gq + m)
        {
            const bool b3 = e & 8, b2 = e & 4, b1 = e & 2, b0 = e & 1;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                float pv[64];
#pragma unroll
                for (int i = 0; i < 64; i += 2) {
                    const float2v p2 = pk(g3[a], g3[a]) * pk(acc[i >> 2][i & 3], acc[i >> 2][(i & 3) + 1]);
                    pv[i] = p2.x;
                    pv[i + 1] = p2.y;
                }
#pragma unroll
                for (int i = 0; i < 32; ++i) pv[i] = pair_sum_rows16<kDppRowMirror>(pv[i], pv[i + 32], b3);
#pragma unroll
                for (int i = 0; i < 16; ++i) pv[i] = pair_sum_rows16<kDppHalfMirror>(pv[i], pv[i + 16], b2);
#pragma unroll
                for (int i = 0; i < 8; ++i) pv[i] = pair_sum_rows16<kDppXor2>(pv[i], pv[i + 8], b1);
#pragma unroll
                for (int i = 0; i < 4; ++i) dW3p[a][i] += pair_sum_rows16<kDppXor1>(pv[i], pv[i + 4], b0);
            }
        }
        // ---- g2 = (W3^T g3) * (1 - h2^2) in place, to HBM in G2's [tile][neuron][64 rows] layout
        // straight from the registers (lane (gq, e): rows 16 wv + e of neurons 16 j + 4 gq + q;
        // each store instruction writes four 64-B row runs)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            floatx4 w3[A];
#pragma unroll
            for (int a = 0; a < A; ++a) w3[a] = *reinterpret_cast<const floatx4 *>(W3c + a * H + 16 * j + 4 * gq);
#pragma unroll
            for (int q = 0; q < 4; q += 2) {
                const float2v h = pk(acc[j][q], acc[j][q + 1]);
                float2v dh = pk(w3[0][q], w3[0][q + 1]) * pk(g3[0], g3[0]);
#pragma unroll
                for (int a = 1; a < A; ++a) dh = pk_fma(pk(w3[a][q], w3[a][q + 1]), pk(g3[a], g3[a]), dh);
                const float2v v = dh * pk_fma(-h, h, pk(1.f, 1.f));  // tanh' = 1 - h^2, one rounding
                acc[j][q] = v.x;
                acc[j][q + 1] = v.y;
            }
        }
        // one wave-uniform guard (8-wave blocks: the last pair's 2nd tile); a scalar tile base
        // advanced per j plus the lane's 32-bit offset (saddr stores, no 64-bit VALU addresses)
        if (tile * kUpdRows < g.rows) {
            auto *tb = g2base + tile * kUpdTileFloats;
            const int lofs = (4 * gq) * kUpdRows + 16 * (wv & 3) + e;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                auto *tbj = tb + (16 * j) * kUpdRows;
                asm volatile("" : "+s"(tbj));  // keep the per-j base scalar
#pragma unroll
                for (int q = 0; q < 4; ++q) tbj[lofs + q * kUpdRows] = acc[j][q];
            }
        }

        // ---- backward: dh1 = W2^T g2, with g2 scaled per wave tile into f16 range; operands of phase
        // P straight from the g2 registers (neurons 32 P + 4 gq + i and 32 P + 16 + 4 gq + i)
        float m = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) m = fmaxf(m, fabsf(acc[j][q]));
        // one power-of-two scale per wave tile (the swapped GEMM's output rows are spread over the
        // lane groups, so a per-row scale would not be the lane's own)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
        g2max = fmaxf(g2max, m);
        const int ex = m > 0.f ? __builtin_amdgcn_frexp_expf(m) : 0;  // m in [2^(ex-1), 2^ex)
        const float sc = __builtin_amdgcn_ldexpf(1.f, 14 - ex);
        // exact powers of two; x 4: 1 - h1^2 = 4 r (1 - r) for h1 = 1 - 2 r
        const float unscale4 = 4.f * __builtin_amdgcn_ldexpf(1.f, ex - 14) / sw;
#pragma unroll
        for (int j = 0; j < 16; ++j) dh1[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        // (operands swapped: dh1 comes out "neuron on lane", dh1[t][q] = row 4 gq + q, neuron 16 t + e)
        x3_gemm16<true, kFdWaves, 1, kFdRing>(Xb, ring, my_part, dh1, [&](int P, half8 &bh, half8 &bl) {
            float x[8];
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
                const float2v u = pk(acc[2 * P][i], acc[2 * P][i + 1]) * sc;
                const float2v v = pk(acc[2 * P + 1][i], acc[2 * P + 1][i + 1]) * sc;
                x[i] = u.x; x[i + 1] = u.y;
                x[i + 4] = v.x; x[i + 5] = v.y;
            }
            split8(x, bh, bl);
        }, [](int) {});
        // ---- g1 = dh1 * (1 - h1^2) and dW1 | db1 of this tile: the 16 neuron tiles' layer-1
        // MFMAs first (their W1 / b1 reads in flight together), then the 64 independent tanh'
        // chains — tile by tile, each tile's LDS reads, MFMA latency and transcendental chain were
        // exposed in turn (r3x diag: g1 5.8k cycles per wave tile for ~2.5k of issue)
        if constexpr (EXT) {  // dL/dh1 to g.g1 (rows 4 gq + q, neuron 16 t + e); the tanh' factor
            // (1 - h1^2) is applied by l1_wgrad_kernel, whose coalesced row loads take h1 beside g1:
            // re-read here, the block's 128 KiB of h1 came in one burst with no MFMA work beside it
            // (13-18 % of this kernel, profiles/r5/r5ab11_ext_tail_noload_diag.txt)
            const float unscale = __builtin_amdgcn_ldexpf(1.f, ex - 14) / sw;
            const int64_t r0 = bt * kFdRows + 16 * wv + 4 * gq;
#pragma unroll
            for (int t = 0; t < 16; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float v = dh1[t][q] * unscale;
                    if (r0 + q < g.rows) g.g1[(size_t)(r0 + q) * H + 16 * t + e] = v;
                }
        } else {
            floatx4 pre[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) pre[t] = layer1_t(t, bobs);
#pragma unroll
            for (int t = 0; t < 16; ++t)
#pragma unroll
                for (int q = 0; q < 4; q += 2) {
                    const float2v r = pk_rcp(pk_exp2(pk(pre[t][q], pre[t][q + 1])) + 1.0f);
                    const float2v v = (pk(dh1[t][q], dh1[t][q + 1]) * unscale4) * pk_fma(-r, r, r);
                    dh1[t][q] = v.x;
                    dh1[t][q + 1] = v.y;
                }
            dw1_acc(srw);
        }
    }

    // ---- per-wave partials: dW3 (lane's neurons) | db3 summed over the 16 row lanes | dW1 | db1
    float *out = g.part3 + (size_t)(blockIdx.x * kFdWaves + wv) * g.p3;
    if constexpr (!EXT) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 2 * NC; ++i) {
                const int n = 16 * (8 * h + 2 * gq + i / NC) + e, f = i % NC;
                if (f < S) out[A * H + A + n * S + f] = dW1p[h][i];
                else if (f == 4 * KS1) out[A * H + A + H * S + n] = dW1p[h][i];
            }
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) g2max = fmaxf(g2max, __shfl_xor(g2max, o));
    if (lane == 0) atomicMax(g.g2max, __float_as_uint(g2max));  // non-negative: uint order
#pragma unroll
    for (int a = 0; a < A; ++a) {
#pragma unroll
        for (int m = 0; m < 4; ++m) out[a * H + 16 * e + 4 * gq + m] = dW3p[a][m];
        float b = db3p[a];
        b += __shfl_xor(b, 1);
        b += __shfl_xor(b, 2);
        b += __shfl_xor(b, 4);
        b += __shfl_xor(b, 8);
        if (lane == 0) out[A * H + a] = b;
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) lsum += __shfl_xor(lsum, o);
    if (lane == 0) g.lpart[blockIdx.x * kFdWaves + wv] = lsum;
}

struct WArgs {
    const float *packed;
    MfmaNet net;
    const float *s;
    const int64_t *index;
    int64_t rows;
    const float *g2t;
    const unsigned *g2max;
    float *part;  // [grid][H*H + H]: dW2 | db2
    const float *h1;  // EXT (KS1 = 0): [rows][256] tanh(W1 s + b1), read instead of recomputed
};

// B fragments of h1 for one 64-row tile: [ks 2][nt 16][hi, lo][64 lanes][8 halfs] (64 KiB):
// lane (g, e) of MFMA step ks holds h1(row, neuron 16 nt + e) * 2^SH for rows 32 ks + 4 g + i and
// 32 ks + 16 + 4 g + i (i < 4): the C layout of two layer-1 MFMA tiles (rows on the lane groups),
// with the A operands (g2 rows) loaded in the same K order.
// 8 waves per block (2 per SIMD, 256 registers), one block per CU; wave wv owns the JT = 2
// output-row tiles j in [32 wv, 32 wv + 32) of dW2 (128 accumulator registers); all waves share the
// tile's h1 fragments. Each fragment pair's LDS reads are pinned ahead of the MFMAs that precede
// their use (sched_group_barrier; without it the scheduler sinks them to just before their MFMAs,
// exposing LDS latency per column step), and each fragment build is fenced into a region of its
// own so the pinned groups only see the GEMM: wgrad 3.16-3.19 -> 3.04-3.07 ms (same box, three
// boxes -2.5 to -4 %, profiles/r3/r3v_wgrad_ab.txt). Measured and removed: 4-wave
// blocks with the VGPR + AGPR budget (half the LDS fragment reads per tile), the
// v_mfma_f32_32x32x16_f16 form (half the MFMA issue slots), the pinning without the fences (8 %
// slower), the build spread over four steps, the younger waves at s_setprio 1.
constexpr int kWgWaves = 8;
// KS1 = 0 (EXT, the 41-input nets): the fragments come from the stored h1 (g.h1 of the FD kernel)
// instead of a layer-1 recompute; each build's 8 values are loaded one build ahead.
template <int KS1>
__global__ void __launch_bounds__(64 * kWgWaves, 1) ppo2_wgrad_kernel(WArgs w) {
    constexpr bool EXT = KS1 == 0;
    constexpr int W = kWgWaves, H = kUpdH, SP = EXT ? 4 : 4 * KS1, NT = 64 * W, JT = 16 / W;
    constexpr int SV = (kUpdRows * SP + NT - 1) / NT;
    constexpr int FRAG = 2 * 16 * 2 * 64 * 8;  // halfs of one tile's h1 fragments (64 KiB)
    constexpr int FPW = 32 / W;                // fragments (ks, nt) built per wave and tile
    // double-buffered: tile i's MFMAs read hfrag[i & 1] while its waves build tile i + step's
    // fragments into hfrag[(i + 1) & 1] from srow[(i + 1) & 1]
    __shared__ float srow[2][EXT ? 1 : kUpdRows][SP];
    __shared__ float w1s[EXT ? 1 : H][SP + 1];
    // b1 four times per neuron: the swapped layer-1 tiles' C operand {b1, b1, b1, b1} in one read
    __shared__ __attribute__((aligned(16))) float b1s[EXT ? 4 : 4 * H];
    __shared__ __attribute__((aligned(16))) _Float16 hfrag[2][FRAG];
    const MfmaNet &net = w.net;
    const int S = net.S;
    const int lane = threadIdx.x & 63, gq = lane >> 4, e = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr (!EXT) {
        // small_r: W1, b1 x 2/ln 2 (h1 as in the FD forward)
        const float *W1c = w.packed + net.off_small_r;
        const float *B1c = w.packed + net.off_small_r + (net.off_b1 - net.off_w1);
        for (int i = threadIdx.x; i < H * SP; i += blockDim.x)
            w1s[i / SP][i % SP] = W1c[w1r_index(i / SP, i % SP, KS1)];
        for (int i = threadIdx.x; i < 4 * H; i += blockDim.x) b1s[i] = B1c[i / 4];
    }
    // g2 scale: max|g2| * 2^sg in [2^13, 2^14)
    const float gm = __uint_as_float(*w.g2max);
    const int gex = gm > 0.f ? __builtin_amdgcn_frexp_expf(gm) : 0;
    const float sg = __builtin_amdgcn_ldexpf(1.f, 14 - gex);
    const float un2 = __builtin_amdgcn_ldexpf(1.f, gex - 14) / kX3HScale;  // 1 / (2^sg 2^SH)
    const float unb = __builtin_amdgcn_ldexpf(1.f, gex - 14);
    half8 ones;
#pragma unroll
    for (int i = 0; i < 8; ++i) ones[i] = (_Float16)1.0f;
    floatx4 acc2[JT][16], accb[JT];
#pragma unroll
    for (int jt = 0; jt < JT; ++jt) {
        accb[jt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int nt = 0; nt < 16; ++nt) acc2[jt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    const int64_t ntiles = (w.rows + kUpdRows - 1) / kUpdRows;
    auto load_s = [&](int64_t tile, float (&sv)[SV]) {  // this thread's s values of a tile
        if constexpr (EXT) return;
#pragma unroll
        for (int u = 0; u < SV; ++u) {
            const int i = threadIdx.x + NT * u, rr = i / SP, k = i % SP;
            const int64_t r = tile * kUpdRows + rr;
            sv[u] = (tile < ntiles && i < kUpdRows * SP && r < w.rows && k < S)
                        ? w.s[(w.index ? w.index[r] : r) * S + k] : 0.f;
        }
    };
    auto store_s = [&](int buf, const float (&sv)[SV]) {
        if constexpr (EXT) return;
#pragma unroll
        for (int u = 0; u < SV; ++u) {
            const int i = threadIdx.x + NT * u;
            if (i < kUpdRows * SP) srow[buf][i / SP][i % SP] = sv[u];
        }
    };
    // fragment F = (ks, nt) of a tile by the wave: layer 1 of rows 32 ks .. 32 ks + 31 on two f32
    // MFMA tiles with the operands swapped (C = [rows][neurons 16 nt ..], the FD's layer1_t), so
    // h1 is the FD forward's (same products, same MFMA), then tanh, the f16 split, two b128 stores
    auto build_frag = [&](int buf, int F) {
        const int ks = F >> 4, nt = F & 15;
        float x[8];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            floatx4 c = *reinterpret_cast<const floatx4 *>(&b1s[4 * (16 * nt + e)]);
#pragma unroll
            for (int kk = 0; kk < KS1; ++kk)
                c = __builtin_amdgcn_mfma_f32_16x16x4f32(srow[buf][32 * ks + 16 * hh + e][4 * kk + gq],
                                                         w1s[16 * nt + e][4 * kk + gq], c, 0, 0, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                x[4 * hh + q] = __builtin_fmaf(-2.0f * kX3HScale,
                                               __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(c[q])),
                                               kX3HScale);
        }
        half8 hh8, hl8;
        split8(x, hh8, hl8);
        *reinterpret_cast<half8 *>(&hfrag[buf][(((ks * 16 + nt) * 2 + 0) * 64 + lane) * 8]) = hh8;
        *reinterpret_cast<half8 *>(&hfrag[buf][(((ks * 16 + nt) * 2 + 1) * 64 + lane) * 8]) = hl8;
    };
    // EXT: the 8 h1 values of fragment F of a tile (rows 32 ks + 16 hh + 4 gq + q, neuron 16 nt + e;
    // rows past the end 0: their g2 is zero), then the same split and stores
    auto load_hv = [&](int64_t tile, int F, float (&hv)[8]) {
        const int ks = F >> 4, nt = F & 15;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t r = tile * kUpdRows + 32 * ks + 16 * hh + 4 * gq + q;
                hv[4 * hh + q] = (tile < ntiles && r < w.rows) ? w.h1[(size_t)r * H + 16 * nt + e] : 0.f;
            }
    };
    auto build_frag_ext = [&](int buf, int F, const float (&hv)[8]) {
        float x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = hv[i] * kX3HScale;
        half8 hh8, hl8;
        split8(x, hh8, hl8);
        *reinterpret_cast<half8 *>(&hfrag[buf][((F * 2 + 0) * 64 + lane) * 8]) = hh8;
        *reinterpret_cast<half8 *>(&hfrag[buf][((F * 2 + 1) * 64 + lane) * 8]) = hl8;
    };
    const float *g2base = w.g2t;
    asm volatile("" : "+s"(g2base));
    // A operands of one K step: g2(rows 32 ks + 4 gq + i and 32 ks + 16 + 4 gq + i,
    // j = 16 JT wv + 16 jt + e) (the fragments' K order); loaded one K step ahead
    auto load_g2 = [&](int64_t tile, int ks, floatx4 (&gv)[JT][2]) {
        const int64_t t = tile < ntiles ? tile : ntiles - 1;
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            const gptr<float> src = as_global(g2base + t * kUpdTileFloats +
                                              (16 * JT * wv + 16 * jt + e) * kUpdRows + 32 * ks + 4 * gq);
            gv[jt][0] = *reinterpret_cast<const __attribute__((address_space(1))) floatx4 *>(src);
            gv[jt][1] = *reinterpret_cast<const __attribute__((address_space(1))) floatx4 *>(src + 16);
        }
    };
    auto frag = [&](int buf, int F, int hl) {
        return *reinterpret_cast<const half8 *>(&hfrag[buf][((F * 2 + hl) * 64 + lane) * 8]);
    };

    // prologue: the first tile's s rows and fragments
    int64_t tile = blockIdx.x;
    {
        float sv[SV];
        load_s(tile, sv);
        store_s(0, sv);
    }
    lds_barrier();
    float hvn[8];  // EXT: the next build's h1 values, in flight one build ahead
    if constexpr (EXT) {
#pragma unroll 1
        for (int u = 0; u < FPW; ++u) {
            load_hv(tile, FPW * wv + u, hvn);
            build_frag_ext(0, FPW * wv + u, hvn);
        }
        load_hv(tile + gridDim.x, FPW * wv, hvn);
    } else {
#pragma unroll 1
        for (int u = 0; u < FPW; ++u) build_frag(0, FPW * wv + u);
    }
    float svn[SV];
    load_s(tile + gridDim.x, svn);
    // the g2 A operands of K steps 0 and 1, each loaded a whole tile ahead (two steps): one step of
    // prefetch left 32 KiB in flight per CU, short of what hides an HBM miss under this load
    floatx4 gv0[JT][2], gv1[JT][2];
    load_g2(tile, 0, gv0);
    load_g2(tile, 1, gv1);
    lds_barrier();
    for (int i = 0; tile < ntiles; tile += gridDim.x, ++i) {
        const int cur = i & 1, nxt = cur ^ 1;
        // next tile's s rows (its fragments go into the other buffer during this tile's MFMAs;
        // the barrier at the end of the previous tile freed that buffer)
        store_s(nxt, svn);
        lds_barrier();
        load_s(tile + 2 * (int64_t)gridDim.x, svn);
        half8 bh = frag(cur, 0, 0), bl = frag(cur, 0, 1);
        // a pinned group of its own (as the FD's rd(0)): the tile's first steps then read one step
        // ahead too (exposed reads per tile 10 -> 3, EXT 24 -> 9; wgrad -0.5 %, EXT -1.4 %:
        // profiles/r5/r5ab3_wgrad_sgb_ab3.txt)
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            // A operands scaled by 2^sg and split
            half8 ah[JT], al[JT];
            floatx4 (&gv)[JT][2] = ks == 0 ? gv0 : gv1;
#pragma unroll
            for (int jt = 0; jt < JT; ++jt) {
                float x[8];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    x[u] = gv[jt][0][u] * sg;
                    x[u + 4] = gv[jt][1][u] * sg;
                }
                split8(x, ah[jt], al[jt]);
            }
            // the next tile's g2 of this K step, in flight under two steps of MFMAs
            load_g2(tile + gridDim.x, ks, gv);
#pragma unroll
            for (int nt = 0; nt < 16; ++nt) {
                const int F = ks * 16 + nt;
                half8 nbh, nbl;  // the next fragment pair, read one step ahead
                if (F + 1 < 32) {
                    nbh = frag(cur, F + 1, 0);
                    nbl = frag(cur, F + 1, 1);
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // (pinned ahead of the MFMAs)
                }
#pragma unroll
                for (int jt = 0; jt < JT; ++jt) {
                    floatx4 v = acc2[jt][nt];
                    v = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[jt], bh, v, 0, 0, 0);
                    v = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[jt], bl, v, 0, 0, 0);
                    v = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[jt], bh, v, 0, 0, 0);
                    acc2[jt][nt] = v;
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 3 * JT, 0);
                // the next tile's fragments, spread over this tile's MFMAs (FPW per wave); for the
                // recomputed h1 the two waves of a SIMD (w, w + 4) build half a spacing apart, so one's
                // build issues under the other's MFMAs (-2.5 %; the EXT loads +3 %, kept in step:
                // r5y_wgrad_stagger_ab.txt; the builds grouped 2 or 4 per point: no gain, r5x)
                constexpr int SP = 32 / FPW;
                static_assert(kWgWaves == 8, "the stagger pairs waves w and w + 4 (one SIMD)");
                if (F % SP == (!EXT && wv >= 4 ? SP / 2 - 1 : SP - 1)) {
                    __builtin_amdgcn_sched_barrier(0);  // (the build stays a region of its own)
                    const int u = F / SP;
                    if constexpr (EXT) {
                        build_frag_ext(nxt, FPW * wv + u, hvn);
                        if (u + 1 < FPW) load_hv(tile + gridDim.x, FPW * wv + u + 1, hvn);
                        else load_hv(tile + 2 * (int64_t)gridDim.x, FPW * wv, hvn);
                    } else {
                        build_frag(nxt, FPW * wv + u);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (F + 1 < 32) {
                    bh = nbh;
                    bl = nbl;
                }
            }
#pragma unroll
            for (int jt = 0; jt < JT; ++jt) {  // db2: g2 against a ones column
                accb[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[jt], ones, accb[jt], 0, 0, 0);
                accb[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[jt], ones, accb[jt], 0, 0, 0);
            }
        }
        lds_barrier();  // the next tile's fragments are complete; this tile's buffer is free
    }
    // C layout: lane holds rows m = 4 gq + q (j = 16 JT wv + 16 jt + m), column e (n = 16 nt + e)
    float *out = w.part + (size_t)blockIdx.x * (H * H + H);
#pragma unroll
    for (int jt = 0; jt < JT; ++jt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = 16 * JT * wv + 16 * jt + 4 * gq + q;
#pragma unroll
            for (int nt = 0; nt < 16; ++nt) out[j * H + 16 * nt + e] = acc2[jt][nt][q] * un2;
            if (e == 0) out[H * H + j] = accb[jt][q] * unb;
        }
}

// grad (torch order W1 b1 W2 b2 W3 b3) = sum over blocks / waves of the partials, in order
// 64 consecutive outputs per block x kRedSplit partial-slices: each thread sums every
// kRedSplit-th partial of its output (loads coalesced across the 64 outputs), then a fixed-order
// LDS combine — deterministic, and no thread walks all 2 x 4 x CUs FD partials serially
constexpr int kRedSplit = 16;
__global__ void __launch_bounds__(64 * kRedSplit)
ppo2_reduce_kernel(MfmaNet net, const float *__restrict__ part, int nw,
                   const float *__restrict__ part3, int n3, int p3, float *grad,
                   const double *__restrict__ lpart, double *loss_sum, int w1_ext) {
    const int H = net.H, S = net.S, A = net.A;
    const int64_t total = (int64_t)H * S + H + (int64_t)H * H + H + (int64_t)A * H + A;
    const int pw = H * H + H;
    const int o = threadIdx.x & 63, sl = threadIdx.x >> 6;
    // EXT nets: W1 | b1 come from the dense dW1 GEMM's own reduce (not in the FD partials)
    const int64_t i0 = w1_ext ? (int64_t)H * S + H : 0;
    const int64_t i = i0 + (int64_t)blockIdx.x * 64 + o;
    float acc = 0.f;
    if (i < total) {
        const float *src;
        int stride, cnt;
        int64_t off;
        if (i < H * S + H) { src = part3; off = A * H + A + i; stride = p3; cnt = n3; }       // W1, b1
        else if (i < H * S + H + H * H + H) { src = part; off = i - (H * S + H); stride = pw; cnt = nw; }  // W2, b2
        else { src = part3; off = i - (H * S + 2 * H + H * H); stride = p3; cnt = n3; }        // W3, b3
        // (unrolled: the loads of 8 partials in flight at once, the adds still in partial order —
        // the W1 / W3 outputs walk 2 048 / kRedSplit FD partials each, one exposed load latency
        // per partial without it)
#pragma unroll 8
        for (int b = sl; b < cnt; b += kRedSplit) acc += src[(size_t)b * stride + off];
    }
    __shared__ float red[kRedSplit][64];
    red[sl][o] = acc;
    __syncthreads();
    if (sl == 0 && i < total) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < kRedSplit; ++k) t += red[k][o];
        grad[i] = t;
    }
    // block 0 also sums the FD waves' loss partials in a fixed order (run-to-run identical loss)
    if (blockIdx.x == 0 && loss_sum) {
        double l = 0.0;
        for (int w = threadIdx.x; w < n3; w += 64 * kRedSplit) l += lpart[w];
        for (int k = 1; k < 64; k <<= 1) l += __shfl_xor(l, k);
        __shared__ double lred[kRedSplit];
        if ((threadIdx.x & 63) == 0) lred[threadIdx.x >> 6] = l;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int k = 0; k < kRedSplit; ++k) t += lred[k];
            *loss_sum += t;
        }
    }
}

// One block, fixed summation order (per-thread strided partials, then a fixed shuffle / LDS
// tree): the same bits on every run and every rank, so data-parallel replicas that each clip
// the all-reduced gradient compute the same clip coefficient. The learner's nets are <= a few
// 100K parameters: one 1024-thread block reads them in a few microseconds.
__global__ void __launch_bounds__(1024) sqnorm_kernel(const float *__restrict__ g, int64_t n,
                                                      double *out) {
    double acc = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) acc += (double)g[i] * (double)g[i];
    for (int o = 1; o < 64; o <<= 1) acc += __shfl_xor(acc, o);
    __shared__ double red[16];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
        out[0] += t;
    }
}

// clip_grad_norm_ applied in place (torch.nn.utils.clip_grad_norm_: coef = max_norm /
// (norm + 1e-6) in f32, clamped to <= 1, grads.mul_(coef)) — the DPPO2 Worker clips its
// persistent gradient buffer this way (DPPO2-4-CartPole/Distributed_PPO2.py:88-89, 99-100).
__global__ void grad_clip_kernel(float *__restrict__ g, int64_t n, const double *sqnorm,
                                 float max_norm) {
    const float norm = (float)sqrt(*sqnorm);
    const float scale = fminf(max_norm / (norm + 1e-6f), 1.f);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        g[i] = g[i] * scale;
}

__global__ void adam_kernel(float *__restrict__ p, const float *__restrict__ g,
                            float *__restrict__ m, float *__restrict__ v, int64_t n,
                            rlp_adam_cfg c, const double *clip_sqnorm) {
    float scale = 1.f;
    if (clip_sqnorm) {  // clip_grad_norm_: coef = max_norm / (norm + 1e-6), clamped to <= 1
        const float norm = (float)sqrt(*clip_sqnorm);
        scale = fminf(c.max_norm / (norm + 1e-6f), 1.f);
    }
    const float bc1 = 1.f - powf(c.beta1, (float)c.step);
    const float bc2 = 1.f - powf(c.beta2, (float)c.step);
    const float step_size = c.lr / bc1, bc2_sqrt = sqrtf(bc2);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float gi = clip_sqnorm ? g[i] * scale : g[i];
        float mi = m[i];
        mi = mi + (1.f - c.beta1) * (gi - mi);           // exp_avg.lerp_(grad, 1 - beta1)
        const float vi = v[i] * c.beta2 + (1.f - c.beta2) * gi * gi;  // mul_(b2).addcmul_(g, g, 1-b2)
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + c.eps;
        p[i] = p[i] + (-step_size) * (mi / denom);       // addcdiv_(exp_avg, denom, -step_size)
    }
}

static int ppo2_grid() { return device_cus(); }  // wgrad / FD: one block per CU

// the 41-input nets' layer 1 on the dense GEMM (rlp_dense.hip): h1 = tanh(s W1^T + b1) and
// dW1 | db1 = G1^T [s | 1] (fixed-order partials + reduce into gW / gb)
int64_t ppo2_ext_floats(int S, int H, int64_t rows);
void ppo2_ext_h1(const float *W1, int ldw, const float *b1, int S, int H, const float *s,
                 int64_t rows, float *h1, hipStream_t st);
void ppo2_ext_dw1(const float *g1, const float *h1, const float *s, int S, int H, int64_t rows,
                  float *part, float *gW, float *gb, hipStream_t st);

// floats of a net's rlp_ppo2_grad workspace, in this order: G2 tiles | wgrad partials | FD
// partials | g2max (16) | FD loss partials (f64) | EXT: h1 | g1 | dW1 partials
struct Ppo2Ws {
    int64_t g2t, partw, part3, g2max, lpart, h1, g1, dw1, total;
    int p3;
};
inline bool ppo2_ext(const MfmaNet &net) { return net.ks1 > 2; }
inline bool ppo2_net_ok(const MfmaNet &net) { return net.H == kUpdH && (net.ks1 <= 2 || net.ks1 == 11); }
inline Ppo2Ws ppo2_ws(const MfmaNet &net, int64_t rows) {
    const int64_t tiles = (rows + kUpdRows - 1) / kUpdRows;
    const int64_t grid = ppo2_grid();  // wgrad: one block per CU; FD: one 8-wave block per CU
    const bool ext = ppo2_ext(net);
    Ppo2Ws w{};
    w.p3 = ext ? net.A * kUpdH + net.A : net.A * kUpdH + net.A + kUpdH * net.S + kUpdH;
    int64_t o = 0;
    auto take = [&](int64_t k) { int64_t r = o; o += (k + 63) / 64 * 64; return r; };
    w.g2t = take(tiles * kUpdTileFloats);
    w.partw = take(grid * (kUpdH * kUpdH + kUpdH));
    w.part3 = take(grid * kFdWaves * (int64_t)w.p3);
    w.g2max = take(16);
    w.lpart = take(2 * grid * kFdWaves);
    if (ext) {
        w.h1 = take(rows * kUpdH);
        w.g1 = take(rows * kUpdH);
        w.dw1 = take(ppo2_ext_floats(net.S, kUpdH, rows));
    }
    w.total = o;
    return w;
}

}  // namespace rlp

using namespace rlp;

extern "C" {

int64_t rlp_ppo2_workspace_floats(const rlp_mlp_desc *desc, int64_t rows) {
    MfmaNet net;
    if (!desc || !mfma_net_from_desc(*desc, &net) || !ppo2_net_ok(net) || rows < 0) return RLP_EINVAL;
    return ppo2_ws(net, rows > 0 ? rows : 1).total;
}

int rlp_ppo2_grad(const rlp_mlp_desc *desc, const float *packed, const rlp_ppo2_loss_cfg *cfg,
                  const float *s, const float *a, const float *a_logprob, const float *adv,
                  const float *v_target, const int64_t *index, int64_t rows, float *grad,
                  double *loss_sum, float *workspace, rlp_stream_t stream) {
    RLP_REQUIRE(desc && packed && cfg && s && grad && workspace, "rlp_ppo2_grad: null argument");
    MfmaNet net;
    if (!mfma_net_from_desc(*desc, &net) || !ppo2_net_ok(net))
        return fail(RLP_EUNSUPPORTED, "rlp_ppo2_grad: need a [S<=8 or 41..44 -> 256 -> 256 -> A] tanh net");
    const bool ext = ppo2_ext(net);
    RLP_REQUIRE(!ext || !index, "rlp_ppo2_grad: %d-input nets take contiguous rows (gather the "
                "mini-batch first)", net.S);
    const bool actor = cfg->kind == RLP_LOSS_ACTOR;
    RLP_REQUIRE(actor || cfg->kind == RLP_LOSS_CRITIC, "rlp_ppo2_grad: loss kind %d", cfg->kind);
    if (actor) {
        RLP_REQUIRE(a && a_logprob && adv, "rlp_ppo2_grad: actor loss needs a, a_logprob, adv");
        RLP_REQUIRE(net.out_tanh, "rlp_ppo2_grad: actor net needs a tanh output layer");
    } else {
        RLP_REQUIRE(v_target && net.A == 1 && !net.out_tanh,
                    "rlp_ppo2_grad: critic loss needs v_target and a linear [..->1] net");
    }
    RLP_REQUIRE(rows > 0, "rlp_ppo2_grad: rows=%lld", (long long)rows);
    hipStream_t st = as_stream(stream);
    const int64_t tiles = (rows + kUpdRows - 1) / kUpdRows;
    const int grid = (int)(tiles < ppo2_grid() ? tiles : ppo2_grid());         // wgrad: 1 per CU
    const int64_t fd_tiles = (rows + kFdRows - 1) / kFdRows;  // FD: one 8-wave block per CU
    const int gfd = (int)(fd_tiles < ppo2_grid() ? fd_tiles : ppo2_grid());
    const int gfull = ppo2_grid();
    Ppo2Args g{};
    g.packed = packed; g.net = net;
    g.s = s; g.a = a; g.lp = a_logprob; g.adv = adv; g.vt = v_target; g.index = index;
    g.rows = rows; g.inv_rows = 1.f / (float)rows; g.eps_clip = cfg->eps_clip;
    float ent = 0.f;
    for (int k = 0; k < net.A && actor; ++k) {
        g.std_[k] = cfg->std[k];
        g.off[k] = (cfg->a_min[k] + cfg->a_max[k]) / 2.0f;
        g.gain[k] = cfg->a_max[k] - g.off[k];
        g.log_std[k] = logf(cfg->std[k]);
        g.inv_var[k] = 1.0f / (cfg->std[k] * cfg->std[k]);
        ent += 0.5f + 0.91893853320467274178f + logf(cfg->std[k]);  // Normal.entropy()
    }
    g.ent_row = cfg->entropy_coef * ent;
    const Ppo2Ws wl = ppo2_ws(net, rows);
    (void)gfull;
    g.g2t = workspace + wl.g2t;
    float *partw = workspace + wl.partw;
    g.part3 = workspace + wl.part3;
    g.p3 = wl.p3;
    g.g2max = reinterpret_cast<unsigned *>(workspace + wl.g2max);
    if (hipMemsetAsync(g.g2max, 0, sizeof(unsigned), st) != hipSuccess)
        return fail(RLP_EINVAL, "rlp_ppo2_grad: memset");
    g.lpart = reinterpret_cast<double *>(workspace + wl.lpart);
    if (ext) {  // h1 of every row for the FD forward, g1 back from it
        g.h1 = workspace + wl.h1;
        g.g1 = workspace + wl.g1;
        ppo2_ext_h1(packed + net.off_w1, 4 * net.ks1, packed + net.off_b1, net.S, kUpdH, s, rows,
                    workspace + wl.h1, st);
    }
#define RLP_FD(KS1, A_, L) ppo2_fd_kernel<KS1, A_, L><<<gfd, 64 * kFdWaves, 0, st>>>(g)
    if (ext) {
        if (!actor) RLP_FD(0, 1, 1);
        else if (net.A == 1) RLP_FD(0, 1, 0); else if (net.A == 2) RLP_FD(0, 2, 0); else if (net.A == 3) RLP_FD(0, 3, 0); else RLP_FD(0, 4, 0);
    } else if (actor) {
        if (net.ks1 == 1) {
            if (net.A == 1) RLP_FD(1, 1, 0); else if (net.A == 2) RLP_FD(1, 2, 0); else if (net.A == 3) RLP_FD(1, 3, 0); else RLP_FD(1, 4, 0);
        } else {
            if (net.A == 1) RLP_FD(2, 1, 0); else if (net.A == 2) RLP_FD(2, 2, 0); else if (net.A == 3) RLP_FD(2, 3, 0); else RLP_FD(2, 4, 0);
        }
    } else {
        if (net.ks1 == 1) RLP_FD(1, 1, 1); else RLP_FD(2, 1, 1);
    }
#undef RLP_FD
    RLP_CHECK_LAUNCH("rlp_ppo2_grad (fd)");
    WArgs w{};
    w.packed = packed; w.net = net; w.s = s; w.index = index; w.rows = rows;
    w.g2t = g.g2t; w.g2max = g.g2max; w.part = partw; w.h1 = g.h1;
    if (ext) ppo2_wgrad_kernel<0><<<grid, 64 * kWgWaves, 0, st>>>(w);
    else if (net.ks1 == 1) ppo2_wgrad_kernel<1><<<grid, 64 * kWgWaves, 0, st>>>(w);
    else ppo2_wgrad_kernel<2><<<grid, 64 * kWgWaves, 0, st>>>(w);
    RLP_CHECK_LAUNCH("rlp_ppo2_grad (wgrad)");
    if (ext)  // dW1 | db1 = G1^T [s | 1] on the dense GEMM, into grad's W1 / b1
        ppo2_ext_dw1(g.g1, g.h1, s, net.S, kUpdH, rows, workspace + wl.dw1, grad,
                     grad + (int64_t)kUpdH * net.S, st);
    const int64_t total = (int64_t)net.H * net.S + net.H + (int64_t)net.H * net.H + net.H +
                          (int64_t)net.A * net.H + net.A;
    const int64_t nred = ext ? total - ((int64_t)net.H * net.S + net.H) : total;
    ppo2_reduce_kernel<<<(int)((nred + 63) / 64), 64 * kRedSplit, 0, st>>>(
        net, partw, grid, g.part3, gfd * kFdWaves, g.p3, grad, g.lpart, loss_sum, ext ? 1 : 0);
    RLP_CHECK_LAUNCH("rlp_ppo2_grad (reduce)");
    return RLP_OK;
}

int rlp_grad_sqnorm(const float *grad, int64_t n, double *out, rlp_stream_t stream) {
    RLP_REQUIRE(grad && out && n >= 0, "rlp_grad_sqnorm: bad argument");
    if (n == 0) return RLP_OK;
    sqnorm_kernel<<<1, 1024, 0, as_stream(stream)>>>(grad, n, out);
    RLP_CHECK_LAUNCH("rlp_grad_sqnorm");
    return RLP_OK;
}

int rlp_grad_clip(float *grad, int64_t n, const double *sqnorm, float max_norm,
                  rlp_stream_t stream) {
    RLP_REQUIRE(grad && sqnorm && n >= 0 && max_norm > 0.f, "rlp_grad_clip: bad argument");
    if (n == 0) return RLP_OK;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    grad_clip_kernel<<<(int)blocks, 256, 0, as_stream(stream)>>>(grad, n, sqnorm, max_norm);
    RLP_CHECK_LAUNCH("rlp_grad_clip");
    return RLP_OK;
}

int rlp_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                  const rlp_adam_cfg *cfg, const double *clip_sqnorm, rlp_stream_t stream) {
    RLP_REQUIRE(param && grad && exp_avg && exp_avg_sq && cfg && n >= 0 && cfg->step >= 1,
                "rlp_adam_step: bad argument");
    if (n == 0) return RLP_OK;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    adam_kernel<<<(int)blocks, 256, 0, as_stream(stream)>>>(param, grad, exp_avg, exp_avg_sq, n,
                                                            *cfg, clip_sqnorm);
    RLP_CHECK_LAUNCH("rlp_adam_step");
    return RLP_OK;
}

}  // extern "C"
