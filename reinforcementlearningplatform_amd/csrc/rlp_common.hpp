// rlp_common.hpp — shared device/host helpers for librlp (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rlp.h"

namespace rlp {

// ------------------------------------------------------------------------------------------
// error plumbing (never throw across the C-ABI)
// ------------------------------------------------------------------------------------------
void set_error(const char *fmt, ...);
int fail(int code, const char *fmt, ...);
// Launch helpers that refuse a launch without a return path to the entry point (e.g. the dense
// GEMM's gemm_multi, called from deep inside a chain) record their status here as well as in the
// error string; RLP_CHECK_LAUNCH hands the first such status back through the C-ABI, so a refused
// launch never reads as RLP_OK with unwritten outputs. take_pending() returns and clears it (entry
// points call it first, so a status never leaks from one call into the next).
int fail_pending(int code, const char *fmt, ...);
int take_pending();

#define RLP_CHECK_LAUNCH(what)                                                            \
    do {                                                                                  \
        const int p_ = ::rlp::take_pending();                                             \
        if (p_ != RLP_OK) return p_;                                                      \
        hipError_t e_ = hipGetLastError();                                                \
        if (e_ != hipSuccess) return ::rlp::fail(-(int)e_, "%s: %s", what, hipGetErrorString(e_)); \
    } while (0)

#define RLP_REQUIRE(cond, ...)                                          \
    do {                                                                \
        if (!(cond)) return ::rlp::fail(RLP_EINVAL, __VA_ARGS__);      \
    } while (0)

inline hipStream_t as_stream(rlp_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// CUs of the current device, read once per process (device properties are slow; a magic static,
// so the first calls from several host threads initialise it once). Grid sizes and the workspace
// sizes derived from them all read this one value, so they always agree. 256 (MI355X) if the
// query fails.
inline int device_cus() {
    static const int cus = [] {
        int dev = 0, n = 0;
        return (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
                   ? n : 256;
    }();
    return cus;
}

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// Global-address-space views: loads through them are global_load_* (counted, in-order vmcnt
// waits) rather than flat_load_*, which the compiler emits when it cannot prove the address space
// and which force vmcnt(0)+lgkmcnt(0) waits that serialise a prefetch pipeline.
template <typename T>
using gptr = const __attribute__((address_space(1))) T *;
template <typename T>
__device__ __forceinline__ gptr<T> as_global(const T *p) {
    return (gptr<T>)p;
}

// ------------------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG: (seed, counter, env_id, tag) -> 4 x u32. Identical stream on
// every rank, so sharding envs over GPUs never changes any env's trajectory.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox_block(uint64_t seed, uint64_t counter, uint64_t env_id,
                                             uint32_t tag, uint32_t out[4]) {
    uint32_t c0 = (uint32_t)counter;
    uint32_t c1 = (uint32_t)(counter >> 32) ^ ((uint32_t)(env_id >> 32) << 16);
    uint32_t c2 = (uint32_t)env_id;
    uint32_t c3 = tag;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// two doubles in [0,1) with 53 random bits each (bit-identical to the CPU oracle)
__device__ __forceinline__ void philox_u01_f64x2(uint64_t seed, uint64_t counter, uint64_t env_id,
                                                 uint32_t tag, double u[2]) {
    uint32_t r[4];
    philox_block(seed, counter, env_id, tag, r);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        uint64_t bits = ((uint64_t)r[2 * k] << 21) ^ (uint64_t)(r[2 * k + 1] >> 11);
        bits &= ((uint64_t)1 << 53) - 1;
        u[k] = (double)bits * (1.0 / 9007199254740992.0);
    }
}

// standard normals (Box-Muller, fp32), block j = 0,1 gives eps[2j], eps[2j+1]
template <int A>
__device__ __forceinline__ void philox_normal_f32(uint64_t seed, uint64_t counter, uint64_t env_id,
                                                  float *eps) {
#pragma unroll
    for (int j = 0; 2 * j < A; ++j) {
        uint32_t r[4];
        philox_block(seed, counter, env_id, 0x100u + (uint32_t)j, r);
        float u1 = (float)(r[0] >> 8) * 5.9604644775390625e-08f + 2.98023223876953125e-08f;
        float u2 = (float)(r[1] >> 8) * 5.9604644775390625e-08f;
        float rad = sqrtf(-2.0f * logf(u1));
        float th = 6.28318530717958647692f * u2;
        eps[2 * j] = rad * cosf(th);
        if (2 * j + 1 < A) eps[2 * j + 1] = rad * sinf(th);
    }
}

// ------------------------------------------------------------------------------------------
// fp32 activations
// ------------------------------------------------------------------------------------------
// Hidden-layer tanh: 1 - 2 / (1 + exp(2x)) on v_exp_f32 / v_rcp_f32 (5 VALU ops, saturates
// correctly at +-inf). Absolute error <= ~1.5e-7, below the fp32 rounding noise of the 256-term
// dot products it feeds.
__device__ __forceinline__ float tanh_fast(float x) {
    const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // exp(2x)
    return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + e), 1.0f);
}

// torch.distributions.Normal(mean, std).log_prob(a) in its fp32 expression order
__device__ __forceinline__ float normal_logp(float a, float mean, float std) {
    float var = std * std;
    float d = a - mean;
    return -(d * d) / (2.0f * var) - logf(std) - 0.91893853320467274178f;
}

__device__ __forceinline__ float mfma16(float a, float b, floatx4 &c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    return 0.f;
}

}  // namespace rlp
