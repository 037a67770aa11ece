// rlp_mfma_layout.hpp — MFMA-fragment weight layout of a [S -> H -> H -> A] tanh MLP (the
// PPO2 drivers' actor/critic, demonstration/PPO2/PPO2-4-CartPole/train.py:39-125) and the
// wave-level fused forward used by the rollout kernel.
//
// Per wave: SUB sub-blocks of 16 envs, "env on the lane" orientation (lane l <-> env l&15 of a
// sub-block, lane group g = l>>4). Layer 1 (H1^T = W1 obs^T) is one MFMA per 16-neuron tile;
// its C registers r = 0..3 (neurons 16t + 4g + r) ARE the B operand of layer 2 at k-step (t, r)
// when layer 2's K dimension is permuted the same way — so H1 never leaves registers and only
// one 16-neuron tile of it is live at a time. Layer 2's A operand (W2 fragments) is packed so that
// every load is one coalesced 1 KiB float4 wave access, shared by the SUB sub-blocks.
//
// Packed layout (floats), NT = H/16, KS1 = ceil(S/4):
//   W1p [t][kk][lane]          W1[16t + (l&15)][4kk + (l>>4)]      (0 for k >= S)
//   B1p [t][lane][4]           b1[16t + 4(l>>4) + r]
//   W2p [t][r][jq][lane][4]    W2[16(4jq+q) + (l&15)][16t + 4(l>>4) + r]
//   B2p [j][lane][4]           b2[16j + 4(l>>4) + r]
//   W3p [a][j][lane][4]        W3[a][16j + 4(l>>4) + r]
//   b3  [4]
#pragma once
#include "rlp_common.hpp"

namespace rlp {

struct MfmaNet {
    int S, H, A, ks1;
    int out_tanh;  // last layer activation is tanh (actor) vs identity (critic)
    int off_b1, off_w2, off_b2, off_w3, off_b3;
    int64_t count;
};

inline bool mfma_net_from_desc(const rlp_mlp_desc &d, MfmaNet *net) {
    if (d.n_layers != 3) return false;
    const int S = d.dims[0], H = d.dims[1], A = d.dims[3];
    if (d.dims[2] != H || !(H == 64 || H == 128 || H == 256)) return false;
    if (S < 1 || S > 8 || A < 1 || A > 4) return false;
    if (d.act[0] != RLP_ACT_TANH || d.act[1] != RLP_ACT_TANH) return false;
    if (d.act[2] != RLP_ACT_TANH && d.act[2] != RLP_ACT_NONE) return false;
    const int NT = H / 16, KS1 = (S + 3) / 4;
    net->S = S; net->H = H; net->A = A; net->ks1 = KS1;
    net->out_tanh = d.act[2] == RLP_ACT_TANH;
    net->off_b1 = NT * KS1 * 64;
    net->off_w2 = net->off_b1 + NT * 256;
    net->off_b2 = net->off_w2 + H * H;
    net->off_w3 = net->off_b2 + NT * 256;
    net->off_b3 = net->off_w3 + A * NT * 256;
    net->count = net->off_b3 + 4;
    return true;
}

// Fused forward of one [S -> H -> H -> NOUT] net for the wave's SUB x 16 envs.
//   bobs[sb][kk]: lane's layer-1 B operand = obs[env 16 sb + (l&15)][4 kk + (l>>4)]
//   out[sb][a]  : pre-activation output of the last layer for env 16 sb + (l&15) (all 4 lane
//                 groups hold the same value after the cross-group reduction); a < nout <= NOUT
template <int H, int SUB, int KS1, int NOUT>
__device__ __forceinline__ void mlp_fused_forward(const float *__restrict__ P0, const MfmaNet &net,
                                                  const int nout, const float (&bobs)[SUB][KS1],
                                                  float (&out)[SUB][NOUT]) {
    constexpr int NT = H / 16;
    const int lane = threadIdx.x & 63;
    // Opaque per call: stops the compiler from hoisting the (loop-invariant) bias / W3 fragment
    // loads out of the caller's T-step loop, which would pin ~256 VGPRs for the whole rollout.
    const float *P = P0;
    asm volatile("" : "+s"(P));
    const float *W1p = P;
    const floatx4 *B1p = reinterpret_cast<const floatx4 *>(P + net.off_b1);
    const floatx4 *W2p = reinterpret_cast<const floatx4 *>(P + net.off_w2);
    const floatx4 *B2p = reinterpret_cast<const floatx4 *>(P + net.off_b2);
    const floatx4 *W3p = reinterpret_cast<const floatx4 *>(P + net.off_w3);
    const float *b3 = P + net.off_b3;

    floatx4 acc[SUB][NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const floatx4 b2 = B2p[j * 64 + lane];  // layer-2 bias as the initial accumulator
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb) acc[sb][j] = b2;
    }

#pragma unroll 1
    for (int t = 0; t < NT; ++t) {
        // ---- layer 1, neuron tile t: H1^T[16t.., envs] = tanh(W1 obs^T + b1)
        float w1[KS1];
#pragma unroll
        for (int kk = 0; kk < KS1; ++kk) w1[kk] = W1p[(t * KS1 + kk) * 64 + lane];
        const floatx4 b1 = B1p[t * 64 + lane];
        floatx4 h1[SUB];
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb) {
            floatx4 c = b1;
#pragma unroll
            for (int kk = 0; kk < KS1; ++kk)
                c = __builtin_amdgcn_mfma_f32_16x16x4f32(w1[kk], bobs[sb][kk], c, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) h1[sb][r] = tanh_fast(c[r]);
        }
        // ---- layer 2, k-steps (t, r): acc[sb][j] += W2[16j.., k] * H1^T[k, envs]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            floatx4 w2[NT / 4];
#pragma unroll
            for (int jq = 0; jq < NT / 4; ++jq) w2[jq] = W2p[((t * 4 + r) * (NT / 4) + jq) * 64 + lane];
#pragma unroll
            for (int jq = 0; jq < NT / 4; ++jq)
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int sb = 0; sb < SUB; ++sb)
                        acc[sb][4 * jq + q] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            w2[jq][q], h1[sb][r], acc[sb][4 * jq + q], 0, 0, 0);
        }
    }

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
            w3[a] = a < nout ? W3p[(a * NT + j) * 64 + lane] : floatx4{0.f, 0.f, 0.f, 0.f};
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
            out[sb][a] = v + (a < nout ? b3[a] : 0.f);
        }
}

}  // namespace rlp
