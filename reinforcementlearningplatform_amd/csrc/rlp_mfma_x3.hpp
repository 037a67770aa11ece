// rlp_mfma_x3.hpp — f16x3 split-MFMA forward of the [S -> 256 -> 256 -> A] tanh MLP (the PPO2
// drivers' actor/critic, demonstration/PPO2/PPO2-4-CartPole/train.py:39-125): layer 2 (99 % of the
// FLOPs) on v_mfma_f32_16x16x32_f16 at 16x the f32-MFMA rate, with fp32-class accuracy.
//
// Split: w = 2^sw W2 and x = 2^SH h1 are each written as hi + lo with hi = f16(v), lo = f16(v - hi)
// (hi, lo normal f16 for every term that matters: 2^sw puts max|W2| in [2^13, 2^14), h1 is a tanh
// in [-1, 1]). w x = wh xh + wh xl + wl xh + wl xl; the three MFMAs keep the first three terms
// (f16 x f16 products are exact in the f32 accumulator), so the dropped wl xl and the rounding of
// lo leave ~3 * 2^-22 |w x| per product — the same order as the f32 MFMA's own accumulation
// rounding (MI355X_MICROARCH.md "FP32-input MFMA": 0.75-1.5e-7 sum|ab|). The accumulator carries
// 2^(sw + SH) (bias pre-scaled in small_r, removed inside the output tanh's exponent constant,
// exact powers of two); small_r's W1, b1 carry tanh's 2 / ln 2, so layer 1 yields the exp2
// argument directly. tests/test_gpu_rollout.py measures the error of both paths against float64.
// (Feeding layer 2 with 2^SH (1 - tanh) and a rowsum correction would save one more op per pair,
// but the accumulator then carries the rowsum's large offset: ~10x the error on the shipped
// PPO2-CartPole actor, outside the parity bound.)
//
// Operands ("env on lane", as rlp_mfma_layout.hpp): for phase P (K = 32 neurons), lane (g, e) of
// sub-block sb holds B[k = 8g + i][env e] = x(neuron 32P + 4g + i) for i < 4 (layer-1 tile 2P, its
// C registers) and x(32P + 16 + 4g + i - 4) for i >= 4 (tile 2P + 1); the packed A fragments
// (X3 region, mfma_pack_kernel) use the same k permutation.
//
// Staging: 16 chunks of 16 KiB per net (phase P, half hf: 8 output tiles x {hi, lo} x 64 lanes x
// 16 B). The kX3Waves waves of a block share one LDS ring of kX3Ring chunks: each wave DMAs a
// quarter of every chunk (global_load_lds_dwordx4, 4 x 1 KiB), waits for its own part with a
// counted vmcnt, and one s_barrier per chunk publishes the chunk and frees the slot the next DMA
// overwrites. Sharing divides the L2 -> CU weight stream by kX3Waves (at the f16 rate a per-wave
// stream would exceed the L2 bandwidth).
#pragma once
#include "rlp_mfma_layout.hpp"

namespace rlp {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));

// tanh(x) for two values on the packed FP32 pipe (v_pk_mul/add/fma_f32 around the two
// transcendentals), k = 2 / ln 2 times any exact scale of x
__device__ __forceinline__ float2v tanh2(float2v x, float k) {
    const float2v t = x * k;
    const float2v e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
    const float2v d = e + 1.0f;
    const float2v r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    return __builtin_elementwise_fma(r, (float2v){-2.0f, -2.0f}, (float2v){1.0f, 1.0f});
}

// f16 hi + lo of two values (packed RNE converts)
__device__ __forceinline__ void split2(float2v x, half2v &hi, half2v &lo) {
    hi = __builtin_convertvector(x, half2v);
    lo = __builtin_convertvector(x - __builtin_convertvector(hi, float2v), half2v);
}

// the same with lo = f16(x - hi) by v_fma_mix (the f16 hi read as a source operand, x - hi exact in
// f32, one rounding to f16 into the low / high half): bit-identical, 3 VALU ops instead of 5
// (tools/mix_split_probe.hip checks the identity on the GPU). The PPO2 update's B operands use it
// (-1.6 % FD cycles); in the rollout the opaque asm cost more in scheduling than it saved (+3 %).
__device__ __forceinline__ void split2_mix(float2v x, half2v &hi, half2v &lo) {
    hi = __builtin_convertvector(x, half2v);
    const unsigned h = __builtin_bit_cast(unsigned, hi);
    // both halves of l are written, so its prior value is not an input (an early-clobber output:
    // a "+v" operand initialised to 0 cost one v_mov per pair, 32 per 16-row GEMM operand build)
    unsigned l;
    asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %0, -%1, 1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(l) : "v"(h), "v"(x.x), "v"(x.y));
    lo = __builtin_bit_cast(half2v, l);
}


constexpr int kX3Waves = 4;             // waves per block sharing the W2 ring
constexpr int kX3Ring = 3;              // chunks resident in the ring
constexpr int kX3ChunkFloats = 4096;    // 16 KiB
constexpr int kX3RingFloats = kX3Ring * kX3ChunkFloats;

__device__ __forceinline__ void block_barrier_raw() {
    // s_barrier without the compiler's vmcnt(0) drain: the counted waits above it already cover
    // exactly the DMA this barrier publishes, and later chunks stay in flight.
    asm volatile("s_barrier" ::: "memory");
}

// Every wave of the block must call this the same number of times (it contains block barriers).
// RG: chunks in the ring (RG - 1 in flight while one is read: 3 for two blocks per CU, 2 where the
// other LDS leaves no room for a third 16-KiB slot, 4 for one block per CU).
// W: waves of the block sharing the ring (4 or 8); each DMAs 16 / W of the 16 KiB of every chunk.
// CPB: 16-KiB chunks per ring slot and block barrier (2: one barrier per k-phase instead of per
// half-phase; the ring then holds RG x CPB chunks).
// (Pipelining the next phase's B operands between the current phase's MFMAs, for the lone wave of
// the one-wave-per-SIMD variants, measured 7 % slower on the UAV: DESIGN.md §4, removed.)
template <int H, int SUB, int KS1, int NOUT, int RG = kX3Ring, int W = kX3Waves, int CPB = 1>
__device__ __forceinline__ void mlp_x3_forward(const float *__restrict__ P0, const float *small,
                                               float *ring, const MfmaNet &net, const int nout,
                                               const float (&bobs)[SUB][KS1],
                                               float (&out)[SUB][NOUT]) {
    static_assert(H == 256, "chunking assumes H = 256 (2 chunks of 8 output tiles per phase)");
    constexpr int NT = H / 16, NPH = H / 32, NC = 2 * NPH;
    static_assert(W == 4 || W == 8, "4 or 8 waves share the ring");
    constexpr int NPW = 16 / W;  // 1-KiB DMA pieces per wave and chunk
    const int lane = threadIdx.x & 63, wv = (threadIdx.x >> 6) & (W - 1);
    const int g = lane >> 4, e = lane & 15;
    const float *Pg = P0;
    asm volatile("" : "+s"(Pg));
    const gptr<float> X = as_global(Pg) + net.off_x3 + wv * NPW * 256 + lane * 4;
    float *const my_part = ring + wv * NPW * 256;
    const float *W1c = small;
    const float *B1c = small + (net.off_b1 - net.off_w1);
    const float *B2c = small + (net.off_b2 - net.off_w1);
    const float *W3c = small + (net.off_w3 - net.off_w1);
    const float *b3c = small + (net.off_b3 - net.off_w1);
    const float *info = small + (net.off_info - net.off_w1);
    const float k_out = 2.8853900817779268f * info[2];  // exp(2x) constant with 2^-(sw+SH) folded

    static_assert(RG >= 2 && RG <= 4, "ring of 2 to 4 slots");
    static_assert(CPB == 1 || CPB == 2, "1 or 2 chunks per slot");
    constexpr int NS = NC / CPB;  // ring slots' worth of chunks per pass
    auto issue = [&](int sc) {    // slot-sized group sc (chunks CPB sc .. CPB sc + CPB - 1)
#pragma unroll
        for (int cc = 0; cc < CPB; ++cc) {
            float *slot = my_part + ((sc % RG) * CPB + cc) * kX3ChunkFloats;
            const gptr<float> src = X + (sc * CPB + cc) * kX3ChunkFloats;
#pragma unroll
            for (int q = 0; q < NPW; ++q) {
                lds_dma_1k(src + q * 256, slot + q * 256);
            }
        }
    };
    block_barrier_raw();  // every wave is done reading the ring (previous call)
#pragma unroll
    for (int sc = 0; sc < RG - 1; ++sc) issue(sc);

    floatx4 acc[SUB][NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const floatx4 b2 = *reinterpret_cast<const floatx4 *>(B2c + 16 * j + 4 * g);
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb) acc[sb][j] = b2;
    }
    auto layer1 = [&](int t, floatx4(&c)[SUB]) {
        float w1[KS1];
#pragma unroll
        for (int kk = 0; kk < KS1; ++kk) w1[kk] = W1c[w1r_index(16 * t + e, 4 * kk + g, KS1)];
        const floatx4 b1 = *reinterpret_cast<const floatx4 *>(B1c + 16 * t + 4 * g);
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb) {
            c[sb] = b1;
#pragma unroll
            for (int kk = 0; kk < KS1; ++kk)
                c[sb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1[kk], bobs[sb][kk], c[sb], 0, 0, 0);
        }
    };
    floatx4 hp0[SUB], hp1[SUB];
    layer1(0, hp0);
    layer1(1, hp1);
    // B operands of one neuron pair (values i, i + 1 of sub-block sb) from the layer-1 tiles
    auto bop_pair = [&](int sb, int i, half8 (&dh)[SUB], half8 (&dl)[SUB]) {
        const float2v pre = i < 4 ? (float2v){hp0[sb][i], hp0[sb][i + 1]}
                                  : (float2v){hp1[sb][i - 4], hp1[sb][i - 3]};
        // 2^SH tanh(h1) = 2^SH - 2^(SH+1) / (1 + exp2(pre)), pre = 2 h1 / ln 2 (small_r)
        const float2v ex = {__builtin_amdgcn_exp2f(pre.x), __builtin_amdgcn_exp2f(pre.y)};
        const float2v dn = ex + 1.0f;
        const float2v rc = {__builtin_amdgcn_rcpf(dn.x), __builtin_amdgcn_rcpf(dn.y)};
        const float2v x = __builtin_elementwise_fma(
            rc, (float2v){-2.0f * kX3HScale, -2.0f * kX3HScale}, (float2v){kX3HScale, kX3HScale});
        half2v hi, lo;
        split2(x, hi, lo);
        dh[sb][i] = hi.x;
        dh[sb][i + 1] = hi.y;
        dl[sb][i] = lo.x;
        dl[sb][i + 1] = lo.y;
    };
    half8 bh[SUB], bl[SUB];

#pragma unroll 1
    for (int P = 0; P < NPH; ++P) {
#pragma unroll
        for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
            for (int i = 0; i < 8; i += 2) bop_pair(sb, i, bh, bl);
        if (P + 1 < NPH) {  // next phase's layer-1 tiles, under this phase's MFMAs
            layer1(2 * P + 2, hp0);
            layer1(2 * P + 3, hp1);
        }
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int c = 2 * P + hf;
            if (c % CPB == 0) {
                const int sc = c / CPB;
                // own part of slot group sc landed; the younger groups' pieces (up to RG - 2) may not
                const int ahead = (RG - 2 < NS - 1 - sc ? RG - 2 : NS - 1 - sc) * NPW * CPB;
                if (ahead >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                else if (ahead >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else if (ahead >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                block_barrier_raw();  // all parts of sc landed; everyone is done with group sc - 1
                if (sc + RG - 1 < NS) issue(sc + RG - 1);  // into group sc - 1's slot
            }
            const float *slot = ring + (((c / CPB) % RG) * CPB + c % CPB) * kX3ChunkFloats + lane * 4;
            // fragments one output tile ahead: tile jj + 1's two reads are issued before tile
            // jj's MFMAs, so an LDS round trip is not exposed per tile (the default schedule
            // reads each pair right before its MFMAs and waits for it)
            half8 ahn = *reinterpret_cast<const half8 *>(slot);
            half8 aln = *reinterpret_cast<const half8 *>(slot + 256);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const half8 ah = ahn, al = aln;
                if (jj + 1 < 8) {
                    ahn = *reinterpret_cast<const half8 *>(slot + (2 * jj + 2) * 256);
                    aln = *reinterpret_cast<const half8 *>(slot + (2 * jj + 3) * 256);
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                }
#pragma unroll
                for (int sb = 0; sb < SUB; ++sb) {
                    floatx4 a = acc[sb][8 * hf + jj];
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[sb], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[sb], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[sb], a, 0, 0, 0);
                    acc[sb][8 * hf + jj] = a;
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 3 * SUB, 0);
            }
        }
    }

    // ---- layer 3: out[a][env] = sum_n W3[a][n] tanh(H2^T[n][env]) + b3[a] (pairs of neurons on
    // the packed FP32 pipe: two partial sums per output)
    float2v part[SUB][NOUT];
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
        for (int a = 0; a < NOUT; ++a) part[sb][a] = (float2v){0.f, 0.f};
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
            for (int r = 0; r < 4; r += 2) {
                const float2v h = tanh2((float2v){acc[sb][j][r], acc[sb][j][r + 1]}, k_out);
#pragma unroll
                for (int a = 0; a < NOUT; ++a)
                    part[sb][a] = __builtin_elementwise_fma((float2v){w3[a][r], w3[a][r + 1]}, h,
                                                            part[sb][a]);
            }
    }
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
        for (int a = 0; a < NOUT; ++a) {
            float v = part[sb][a].x + part[sb][a].y;
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            out[sb][a] = v + (a < nout ? b3c[a] : 0.f);
        }
}

}  // namespace rlp
