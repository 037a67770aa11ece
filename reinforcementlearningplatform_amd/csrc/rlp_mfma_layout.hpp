// rlp_mfma_layout.hpp — MFMA-fragment weight layout of a [S -> H -> H -> A] tanh MLP (the
// PPO2 drivers' actor/critic, demonstration/PPO2/PPO2-4-CartPole/train.py:39-125) and the
// wave-level fused forward used by the rollout kernel.
//
// Per wave: SUB sub-blocks of 16 envs, "env on the lane" orientation (lane l <-> env l&15 of a
// sub-block, lane group g = l>>4). Layer 1 (H1^T = W1 obs^T) is one MFMA per 16-neuron tile; its
// C registers r = 0..3 (neurons 16t + 4g + r) ARE the B operand of layer 2 at k-phase (t, r) when
// layer 2's K dimension is permuted the same way — so H1 never leaves registers and only one
// 16-neuron tile of it is live at a time.
//
// Staging: layer 2's A operand (W2 fragments, 4 KiB per k-phase at H = 256) streams from L2 into a
// per-wave LDS ring by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave instruction, no VGPRs),
// RING-1 phases ahead, retired by counted vmcnt waits and read back with conflict-free
// ds_read_b128. The small weights (W1, b1, b2, W3, b3) live in LDS for the whole launch.
//
// Packed layout (floats), NT = H/16, NJQ = NT/4, KS1 = ceil(S/4):
//   W2p [t][r][jq][lane][4]   W2[16(4jq+q) + (l&15)][16t + 4(l>>4) + r]      (offset 0)
//   W1c [H][4*KS1]            W1[j][k] (0 for k >= S)                         (LDS-resident part:)
//   B1c [H], B2c [H], W3c [A][H], b3 [4], info [4] = {2^sw, 2^(sw+SH), 2^-(sw+SH), 0}
//   small_r                   the resident part in the f16x3 forward's form (same internal
//                             offsets; rlp_mfma_x3.hpp): W1, b1 times 2 / ln 2 (layer 1 yields
//                             tanh's exp2 argument), B2c times 2^(sw+SH), info {2^sw, 1,
//                             2^-(sw+SH), 0}; its W1 as [j / 16][k][j % 16] (w1r_index): a layer-1
//                             A operand (lane (g, e) reads W1[16 t + e][4 kk + g]) is then 64
//                             consecutive floats, conflict-free for ds_read_b32 (the [H][4 KS1]
//                             form put lanes e and e + 8 on one bank: 2-way at KS1 = 1, 4-way at
//                             KS1 = 2, the UAV's 6 inputs)
//   X3  (256-B aligned)       W2 * 2^sw split into f16 hi + lo, the f16x3 path's chunks
//                             (rlp_mfma_x3.hpp)
//   X3T                       the same for W2^T (the PPO2 update's backward GEMM, rlp_update.hip)
#pragma once
#include "rlp_common.hpp"

namespace rlp {

// f16x3 path: hidden activations h in [-1, 1] are scaled by 2^SH before the f16 split
constexpr float kX3HScale = 4096.f;

// offset of W1[j][k] in small_r's W1 block ([j / 16][k][j % 16], k < 4 KS1)
__host__ __device__ constexpr int w1r_index(int j, int k, int KS1) {
    return (j >> 4) * (64 * KS1) + k * 16 + (j & 15);
}

struct MfmaNet {
    int S, H, A, ks1;
    int out_tanh;  // last layer activation is tanh (actor) vs identity (critic)
    int off_w1, off_b1, off_b2, off_w3, off_b3, off_info;  // offsets of the LDS-resident part
    int small_count;                                         // floats from off_w1 to info's end
    int off_small_r;                                         // the f16x3 form of the same part
    int off_x3;                                              // f16 hi/lo W2 chunks (H*H floats)
    int off_x3t;                                             // the same for W2^T
    int64_t count;
};

inline bool mfma_net_from_desc(const rlp_mlp_desc &d, MfmaNet *net) {
    if (d.n_layers != 3) return false;
    const int S = d.dims[0], H = d.dims[1], A = d.dims[3];
    if (d.dims[2] != H || !(H == 64 || H == 128 || H == 256)) return false;
    // inputs: the drivers' 1-8 (CartPole, AngleOnly, SOI, UGV, UAV) or 41-44 (the UGV obstacle-
    // avoidance demos' 4 + 37 lidar beams: layer 1 as KS1 = 11 K-steps of the 16x16x4 MFMA)
    if (!((S >= 1 && S <= 8) || (S >= 41 && S <= 44)) || A < 1 || A > 4) return false;
    if (d.act[0] != RLP_ACT_TANH || d.act[1] != RLP_ACT_TANH) return false;
    if (d.act[2] != RLP_ACT_TANH && d.act[2] != RLP_ACT_NONE) return false;
    const int KS1 = (S + 3) / 4;
    net->S = S; net->H = H; net->A = A; net->ks1 = KS1;
    net->out_tanh = d.act[2] == RLP_ACT_TANH;
    net->off_w1 = H * H;
    net->off_b1 = net->off_w1 + H * 4 * KS1;
    net->off_b2 = net->off_b1 + H;
    net->off_w3 = net->off_b2 + H;
    net->off_b3 = net->off_w3 + A * H;
    net->off_info = net->off_b3 + 4;
    net->small_count = net->off_info + 4 - net->off_w1;
    net->off_small_r = net->off_info + 4;
    net->off_x3 = (net->off_small_r + net->small_count + 63) / 64 * 64;
    net->off_x3t = net->off_x3 + H * H;
    net->count = net->off_x3t + (int64_t)H * H;
    return true;
}

// LDS floats of one net's resident part (upper bound used for static carving)
template <int H, int KS1, int NOUT>
constexpr int mlp_small_floats() { return H * 4 * KS1 + 2 * H + NOUT * H + 8; }
template <int H>
constexpr int mlp_phase_floats() { return H / 64 * 256; }  // one k-phase of W2 fragments

// Cooperative copy of a net's resident part to LDS (all threads of the block; caller syncs);
// x3: its f16x3 form (small_r) for mlp_x3_forward.
__device__ __forceinline__ void mlp_small_to_lds(const float *P, const MfmaNet &net, float *dst,
                                                 bool x3 = false) {
    const gptr<float> src = as_global(P) + (x3 ? net.off_small_r : net.off_w1);
    for (int i = threadIdx.x; i < net.small_count; i += blockDim.x) dst[i] = src[i];
}

__device__ __forceinline__ void lds_dma_1k(gptr<float> src_lane, float *dst_wave_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src_lane,
                                     (__attribute__((address_space(3))) void *)dst_wave_base, 16,
                                     0, 0);
}

// Fused forward of one [S -> H -> H -> NOUT] net for the wave's SUB x 16 envs.
//   P      : packed net (global); W2 fragments are read from it by LDS-DMA
//   small  : the net's resident part in LDS (mlp_small_to_lds)
//   ring   : this wave's RING x phase LDS ring
//   bobs[sb][kk]: lane's layer-1 B operand = obs[env 16 sb + (l&15)][4 kk + (l>>4)]
//   out[sb][a]  : pre-activation output of the last layer for env 16 sb + (l&15) (all 4 lane
//                 groups hold the same value after the cross-group reduction); a < nout <= NOUT
// The counted waits assume the only VMEM ops this wave issues inside are the ring's LDS-DMA.
template <int H, int SUB, int KS1, int NOUT, int RING>
__device__ __forceinline__ void mlp_fused_forward(const float *__restrict__ P0, const float *small,
                                                  float *ring, const MfmaNet &net, const int nout,
                                                  const float (&bobs)[SUB][KS1],
                                                  float (&out)[SUB][NOUT]) {
    constexpr int NT = H / 16, NJQ = NT / 4, PH = NT * 4, PF = mlp_phase_floats<H>();
    static_assert(NJQ == 4, "counted waits below assume 4 LDS-DMA instructions per phase");
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, e = lane & 15;
    const float *Pg = P0;
    asm volatile("" : "+s"(Pg));
    const gptr<float> W2g = as_global(Pg) + lane * 4;
    const float *W1c = small;
    const float *B1c = small + (net.off_b1 - net.off_w1);
    const float *B2c = small + (net.off_b2 - net.off_w1);
    const float *W3c = small + (net.off_w3 - net.off_w1);
    const float *b3c = small + (net.off_b3 - net.off_w1);

    auto issue = [&](int p) {  // phase p -> ring slot p % RING (clamped: tail re-issues are unused)
        const int pc = p < PH ? p : PH - 1;
        float *slot = ring + (p % RING) * PF;
#pragma unroll
        for (int jq = 0; jq < NJQ; ++jq) lds_dma_1k(W2g + (pc * NJQ + jq) * 256, slot + jq * 256);
    };
#pragma unroll
    for (int p = 0; p < RING - 1; ++p) issue(p);

    floatx4 acc[SUB][NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const floatx4 b2 = *reinterpret_cast<const floatx4 *>(B2c + 16 * j + 4 * g);  // C-init
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb) acc[sb][j] = b2;
    }
    auto layer1 = [&](int t, floatx4(&c)[SUB]) {
        float w1[KS1];
#pragma unroll
        for (int kk = 0; kk < KS1; ++kk) w1[kk] = W1c[(16 * t + e) * (4 * KS1) + 4 * kk + g];
        const floatx4 b1 = *reinterpret_cast<const floatx4 *>(B1c + 16 * t + 4 * g);
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb) {
            c[sb] = b1;
#pragma unroll
            for (int kk = 0; kk < KS1; ++kk)
                c[sb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1[kk], bobs[sb][kk], c[sb], 0, 0, 0);
        }
    };
    floatx4 hpre[SUB];
    layer1(0, hpre);

#pragma unroll 1
    for (int t = 0; t < NT; ++t) {
        floatx4 h1[SUB];
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
            for (int r = 0; r < 4; ++r) h1[sb][r] = tanh_fast(hpre[sb][r]);
        layer1(t + 1 < NT ? t + 1 : NT - 1, hpre);  // next tile's layer 1, under this tile's MFMAs
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = 4 * t + r;
            issue(p + RING - 1);
            // retire phase p: all but the 4 * (RING - 1) youngest VMEM ops (the later phases)
            if constexpr (RING == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if constexpr (RING == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            const float *slot = ring + (p % RING) * PF;
            floatx4 w2[NJQ];
#pragma unroll
            for (int jq = 0; jq < NJQ; ++jq)
                w2[jq] = *reinterpret_cast<const floatx4 *>(slot + jq * 256 + lane * 4);
#pragma unroll
            for (int jq = 0; jq < NJQ; ++jq)
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int sb = 0; sb < SUB; ++sb)
                        acc[sb][4 * jq + q] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            w2[jq][q], h1[sb][r], acc[sb][4 * jq + q], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the clamped tail DMAs

    // ---- layer 3: out[a][env] = sum_n W3[a][n] tanh(H2^T[n][env]) + b3[a]
    float part[SUB][NOUT];
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
        for (int a = 0; a < NOUT; ++a) part[sb][a] = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        floatx4 w3[NOUT];
#pragma unroll
        for (int a = 0; a < NOUT; ++a)
            w3[a] = a < nout ? *reinterpret_cast<const floatx4 *>(W3c + a * H + 16 * j + 4 * g)
                             : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float h = tanh_fast(acc[sb][j][r]);
#pragma unroll
                for (int a = 0; a < NOUT; ++a) part[sb][a] = __builtin_fmaf(w3[a][r], h, part[sb][a]);
            }
    }
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
        for (int a = 0; a < NOUT; ++a) {
            float v = part[sb][a];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            out[sb][a] = v + (a < nout ? b3c[a] : 0.f);
        }
}

}  // namespace rlp
