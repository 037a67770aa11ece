// mfma_issue_bench.hip — how much VALU a wave can issue between its own f16 MFMAs on gfx950:
// cycles per MFMA (s_memtime ticks) for v_mfma_f32_16x16x32_f16 vs v_mfma_f32_32x32x16_f16 with
// K independent VALU fillers (v_fma_f32 or v_exp_f32) pinned after every MFMA by
// sched_group_barrier, at 1 and 2 waves per SIMD. Evidence for DESIGN.md's round-2 plan (the
// rollout's layer 2 on 32x32x16). Build: hipcc -O3 --offload-arch=gfx950 -o mfma_issue_bench
// mfma_issue_bench.hip; run on one MI355X.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kIters = 256, kUnroll = 8;

template <int SHAPE, int K, int TRANS>
__global__ void __launch_bounds__(512) issue_kernel(float *out, long long *cyc) {
    const int lane = threadIdx.x & 63;
    half8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = (_Float16)(0.001f * (lane + i));
        b[i] = (_Float16)(0.002f * (lane - i));
    }
    floatx4 c4[4] = {};
    floatx16 c16[4] = {};
    float x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = 0.01f * (lane + k);
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            if constexpr (SHAPE == 0)
                c4[u & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c4[u & 3], 0, 0, 0);
            else
                c16[u & 3] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c16[u & 3], 0, 0, 0);
#pragma unroll
            for (int k = 0; k < K; ++k)
                x[k] = TRANS ? __builtin_amdgcn_exp2f(x[k]) : __builtin_fmaf(x[k], 0.999f, 0.001f);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (K) __builtin_amdgcn_sched_group_barrier(0x002, K, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        s += c4[j][0];
        s += c16[j][0];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int SHAPE, int K, int TRANS>
static void run(int waves, float *out, long long *cyc) {
    long long h[8];
    issue_kernel<SHAPE, K, TRANS><<<1, 64 * waves>>>(out, cyc);  // warm-up
    issue_kernel<SHAPE, K, TRANS><<<1, 64 * waves>>>(out, cyc);
    hipDeviceSynchronize();
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    long long m = 0;
    for (int w = 0; w < waves; ++w) m = h[w] > m ? h[w] : m;
    printf("%-10s waves/SIMD=%d fillers=%d x %-4s : %.1f ticks per MFMA\n",
           SHAPE ? "32x32x16" : "16x16x32", waves / 4, K, TRANS ? "exp" : "fma",
           (double)m / (kIters * kUnroll));
}

template <int SHAPE, int TRANS>
static void sweep(int waves, float *out, long long *cyc) {
    run<SHAPE, 0, TRANS>(waves, out, cyc);
    run<SHAPE, 1, TRANS>(waves, out, cyc);
    run<SHAPE, 2, TRANS>(waves, out, cyc);
    run<SHAPE, 3, TRANS>(waves, out, cyc);
    run<SHAPE, 4, TRANS>(waves, out, cyc);
    run<SHAPE, 6, TRANS>(waves, out, cyc);
    run<SHAPE, 8, TRANS>(waves, out, cyc);
}

int main() {
    float *out;
    long long *cyc;
    hipMalloc(&out, 512 * sizeof(float));
    hipMalloc(&cyc, 8 * sizeof(long long));
    for (int waves : {4, 8}) {
        sweep<0, 0>(waves, out, cyc);
        sweep<1, 0>(waves, out, cyc);
        sweep<0, 1>(waves, out, cyc);
        sweep<1, 1>(waves, out, cyc);
    }
    hipFree(out);
    hipFree(cyc);
    return 0;
}
