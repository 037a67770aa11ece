// rlp_mlp.hip — actor/critic MLP forward on fp32 MFMA (v_mfma_f32_16x16x4_f32), the packer for
// the fused-rollout weight layout, and Gaussian policy sampling.
//
// Orientation used everywhere ("env on the lane"): a layer computes H_out^T = W · H_in^T, so the
// MFMA A operand is a weight fragment (lane l: W[16 j + (l&15)][k]) and the B operand an activation
// fragment (lane l: H_in[env l&15][k]); the 16x16 C tile lands as lane l: H_out[env l&15]
// [neuron 16 j + 4 (l>>4) + r], r = 0..3. MFMA numerics are an exact k-ordered fp32 fma chain.
#include "rlp_mfma_layout.hpp"

namespace rlp {

// ------------------------------------------------------------------------------------------
// Generic forward: any Linear(+act) stack, one wave per 16 rows, activations in LDS.
// ------------------------------------------------------------------------------------------
constexpr int kMlpMaxW = 512;

struct MlpArgs {
    rlp_mlp_desc d;
};

__device__ __forceinline__ float act_apply(int act, float v) {
    return act == RLP_ACT_TANH ? tanhf(v) : (act == RLP_ACT_RELU ? fmaxf(v, 0.f) : v);
}

__global__ void __launch_bounds__(64) mlp_forward_kernel(MlpArgs args, const float *__restrict__ P,
                                                         const float *__restrict__ x, float *y, int n,
                                                         const uint8_t *mask, int ldw) {
    extern __shared__ float lds[];  // [2][16][ldw]
    const rlp_mlp_desc &d = args.d;
    const int lane = threadIdx.x;
    const int g = lane >> 4, e = lane & 15;
    const int row0 = blockIdx.x * 16;
    const int row = row0 + e;
    bool active = row < n && (!mask || mask[row]);
    if (!__any(active)) return;  // wave-uniform skip of fully masked 16-row groups
    float *buf0 = lds, *buf1 = lds + 16 * ldw;
    // stage input rows (zero padded)
    const int in0 = d.dims[0];
    for (int idx = lane; idx < 16 * ldw; idx += 64) {
        const int r = idx / ldw, k = idx % ldw;
        const int gr = row0 + r;
        buf0[idx] = (gr < n && k < in0) ? x[(size_t)gr * in0 + k] : 0.f;
    }
    __syncthreads();
    const float *pw = P;
    float *cur = buf0, *nxt = buf1;
    for (int l = 0; l < d.n_layers; ++l) {
        const int in = d.dims[l], out = d.dims[l + 1];
        const float *W = pw, *b = pw + (size_t)in * out;
        const int ks_n = (in + 3) / 4, jt_n = (out + 15) / 16;
        for (int jt = 0; jt < jt_n; ++jt) {
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
            const int wrow = 16 * jt + e;
            for (int ks = 0; ks < ks_n; ++ks) {
                const int k = 4 * ks + g;
                const float a = (wrow < out && k < in) ? W[(size_t)wrow * in + k] : 0.f;
                const float bv = cur[e * ldw + k];
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int nr = 16 * jt + 4 * g + r;
                float v = 0.f;
                if (nr < out) v = act_apply(d.act[l], acc[r] + b[nr]);
                nxt[e * ldw + nr] = v;
            }
        }
        // zero the k-padding of the next layer's input
        const int pad_to = ((out + 3) / 4) * 4;
        for (int k = jt_n * 16; k < pad_to; ++k) nxt[e * ldw + k] = 0.f;
        __syncthreads();
        pw += (size_t)in * out + out;
        float *t = cur; cur = nxt; nxt = t;
    }
    const int outn = d.dims[d.n_layers];
    if (active) {
        for (int j = g; j < outn; j += 4) y[(size_t)row * outn + j] = cur[e * ldw + j];
    }
}

// ------------------------------------------------------------------------------------------
// Fused-layout packer (see rlp_mfma_layout.hpp for the layout)
// ------------------------------------------------------------------------------------------
// info[] = {2^sw, 2^sw * 2^SH, 2^-(sw + SH), 0}: 2^sw puts max|W2| in [2^13, 2^14), far inside f16
// range, so the hi and lo f16 halves of every weight that matters stay normal (rlp_mfma_x3.hpp).
// (one 1024-thread block; each thread keeps 8 independent loads in flight, so the 256 KB of W2
// stream at once instead of one dependent load per thread and step: 83 -> a few us per call)
__global__ void __launch_bounds__(1024) mfma_scale_kernel(MfmaNet net, const float *__restrict__ P,
                                                          float *out) {
    const int S = net.S, H = net.H;
    const float *W2 = P + S * H + H;
    float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if ((((uintptr_t)W2) & 15) == 0) {  // 16-byte loads, all of a thread's in flight at once
        const float4 *W4 = reinterpret_cast<const float4 *>(W2);  // (H * H % 4 == 0: H even)
        for (int i0 = threadIdx.x; i0 < H * H / 4; i0 += 16 * 1024) {
            float4 q[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int i = i0 + u * 1024;
                q[u] = i < H * H / 4 ? W4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < 16; ++u)
                m[u & 7] = fmaxf(m[u & 7], fmaxf(fmaxf(fabsf(q[u].x), fabsf(q[u].y)),
                                                 fmaxf(fabsf(q[u].z), fabsf(q[u].w))));
        }
    } else {
        for (int i0 = threadIdx.x; i0 < H * H; i0 += 8 * 1024) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u * 1024;
                if (i < H * H) m[u] = fmaxf(m[u], fabsf(W2[i]));
            }
        }
    }
    float mm = fmaxf(fmaxf(fmaxf(m[0], m[1]), fmaxf(m[2], m[3])), fmaxf(fmaxf(m[4], m[5]), fmaxf(m[6], m[7])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mm = fmaxf(mm, __shfl_xor(mm, o));
    __shared__ float red[16];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mm;
    __syncthreads();
    if (threadIdx.x == 0)
        for (int w = 1; w < 16; ++w) red[0] = fmaxf(red[0], red[w]);
    if (threadIdx.x == 0) {
        int e = 0;
        if (red[0] > 0.f) frexpf(red[0], &e);  // max = f * 2^e, f in [0.5, 1)
        e = e < -60 ? -60 : (e > 60 ? 60 : e);
        const float sw = ldexpf(1.f, 14 - e);
        float *info = out + net.off_info;
        info[0] = sw;
        info[1] = sw * kX3HScale;
        info[2] = 1.f / (sw * kX3HScale);
        info[3] = 0.f;
    }
}

__global__ void mfma_pack_kernel(MfmaNet net, const float *__restrict__ P, float *out) {
    const int total = (int)net.count;
    const int S = net.S, H = net.H, A = net.A, NT = H / 16, KS1 = net.ks1;
    const float *W1 = P, *b1 = W1 + S * H, *W2 = b1 + H, *b2 = W2 + H * H, *W3 = b2 + H,
                *b3 = W3 + H * A;
    const float sw = out[net.off_info];  // written by mfma_scale_kernel (same stream)
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += gridDim.x * blockDim.x) {
        float v = 0.f;
        if (idx < net.off_w1) {  // W2p [t][r][jq][lane][4]
            const int q = idx;
            const int qq = q & 3, lane = (q >> 2) & 63, jq = (q >> 8) % (NT / 4);
            const int r = ((q >> 8) / (NT / 4)) & 3, t = ((q >> 8) / (NT / 4)) >> 2;
            const int j = 16 * (4 * jq + qq) + (lane & 15);
            const int k = 16 * t + 4 * (lane >> 4) + r;
            v = W2[j * H + k];
        } else if (idx < net.off_b1) {  // W1c [H][4*KS1]
            const int q = idx - net.off_w1;
            const int j = q / (4 * KS1), k = q % (4 * KS1);
            v = k < S ? W1[j * S + k] : 0.f;
        } else if (idx < net.off_b2) {  // B1c [H]
            v = b1[idx - net.off_b1];
        } else if (idx < net.off_w3) {  // B2c [H]
            v = b2[idx - net.off_b2];
        } else if (idx < net.off_b3) {  // W3c [A][H]
            v = W3[idx - net.off_w3];
        } else if (idx < net.off_info) {  // b3 [4]
            const int a = idx - net.off_b3;
            v = a < A ? b3[a] : 0.f;
        } else if (idx < net.off_small_r) {  // info (mfma_scale_kernel)
            continue;
        } else if (idx < net.off_x3) {  // small_r + alignment pad
            const int q = idx - net.off_small_r + net.off_w1;
            constexpr float k2 = 2.8853900817779268f;  // 2 / ln 2: tanh's exp(2x) as exp2
            if (q < net.off_b1) {  // W1 as [j / 16][k][j % 16] (w1r_index)
                const int o = q - net.off_w1;
                const int j = 16 * (o / (64 * KS1)) + (o & 15), k = (o % (64 * KS1)) >> 4;
                v = k < S ? W1[j * S + k] * k2 : 0.f;
            } else if (q < net.off_b2) {
                v = b1[q - net.off_b1] * k2;
            } else if (q < net.off_w3) {
                v = b2[q - net.off_b2] * (sw * kX3HScale);
            } else if (q < net.off_b3) {
                v = W3[q - net.off_w3];
            } else if (q < net.off_info) {
                const int a = q - net.off_b3;
                v = a < A ? b3[a] : 0.f;
            } else if (q < net.off_info + 4) {
                const int i = q - net.off_info;
                v = i == 0 ? sw : (i == 1 ? 1.f : (i == 2 ? 1.f / (sw * kX3HScale) : 0.f));
            }
        } else {  // X3 / X3T [P][j][part][lane][8 halfs]: two halfs per float slot
            const bool tr = idx >= net.off_x3t;
            const int q = idx - (tr ? net.off_x3t : net.off_x3);
            const int i = 2 * (q & 3), lane = (q >> 2) & 63, part = (q >> 8) & 1;
            const int j = (q >> 9) % NT, Pp = (q >> 9) / NT;
            const int row = 16 * j + (lane & 15), g = lane >> 4;
            _Float16 h2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int ii = i + u;
                const int k = 32 * Pp + (ii < 4 ? 4 * g + ii : 16 + 4 * g + ii - 4);
                const float w = (tr ? W2[k * H + row] : W2[row * H + k]) * sw;
                const _Float16 hi = (_Float16)w;
                h2[u] = part == 0 ? hi : (_Float16)(w - (float)hi);
            }
            __builtin_memcpy(&v, h2, 4);
        }
        out[idx] = v;
    }
}

// ------------------------------------------------------------------------------------------
// Gaussian policy sample (Proximal_Policy_Optimization2.choose_action :69-76)
// ------------------------------------------------------------------------------------------
struct SampleArgs {
    float std[8], a_min[8], a_max[8];
};

template <int A>
__global__ void __launch_bounds__(256) policy_sample_kernel(const float *__restrict__ mean, int n,
                                                            SampleArgs sa, const float *noise,
                                                            uint64_t seed, uint64_t counter,
                                                            uint64_t env_id0, float *action,
                                                            float *logp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float eps[A];
    if (noise) {
#pragma unroll
        for (int j = 0; j < A; ++j) eps[j] = noise[(size_t)i * A + j];
    } else {
        philox_normal_f32<A>(seed, counter, env_id0 + (uint64_t)i, eps);
    }
#pragma unroll
    for (int j = 0; j < A; ++j) {
        const float m = mean[(size_t)i * A + j];
        float a = m + sa.std[j] * eps[j];
        a = fmaxf(fminf(a, sa.a_max[j]), sa.a_min[j]);
        action[(size_t)i * A + j] = a;
        logp[(size_t)i * A + j] = normal_logp(a, m, sa.std[j]);
    }
}

struct SacArgs {
    float ls_lo[4], ls_hi[4], gain[4], off[4], a_min[4], a_max[4];
    int clamp_action, deterministic;
};

// softplus with torch's default threshold (beta 1, threshold 20)
__device__ __forceinline__ float softplus_f(float x) { return x > 20.f ? x : log1pf(expf(x)); }

template <int A>
__global__ void __launch_bounds__(256) sac_sample_kernel(const float *__restrict__ head, int n,
                                                         SacArgs sa, const float *noise,
                                                         uint64_t seed, uint64_t counter,
                                                         uint64_t env_id0, float *action,
                                                         float *log_pi) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float eps[A];
    if (sa.deterministic) {
#pragma unroll
        for (int j = 0; j < A; ++j) eps[j] = 0.f;
    } else if (noise) {
#pragma unroll
        for (int j = 0; j < A; ++j) eps[j] = noise[(size_t)i * A + j];
    } else {
        philox_normal_f32<A>(seed, counter, env_id0 + (uint64_t)i, eps);
    }
    float lp = 0.f, corr = 0.f;
    const float kHalfLog2Pi = 0.918938533204672742f;  // math.log(math.sqrt(2 * math.pi)) in f32
    const float kLog2 = 0.693147180559945309f;         // np.log(2) in f32
#pragma unroll
    for (int j = 0; j < A; ++j) {
        const float mean = head[(size_t)i * 2 * A + j];
        float ls = head[(size_t)i * 2 * A + A + j];
        ls = fminf(fmaxf(ls, sa.ls_lo[j]), sa.ls_hi[j]);  // torch.clamp
        const float sd = expf(ls);
        const float u = sa.deterministic ? mean : mean + eps[j] * sd;  // loc + eps * scale
        // Normal.log_prob: -((u - loc) ** 2) / (2 * var) - log(scale) - log(sqrt(2 pi))
        const float d = u - mean;
        const float lpj = -(d * d) / (2.f * (sd * sd)) - logf(sd) - kHalfLog2Pi;
        lp = j == 0 ? lpj : lp + lpj;
        const float cj = 2.f * ((kLog2 - u) - softplus_f(-2.f * u));
        corr = j == 0 ? cj : corr + cj;
        float a = tanhf(u) * sa.gain[j] + sa.off[j];
        if (sa.clamp_action) a = fmaxf(fminf(a, sa.a_max[j]), sa.a_min[j]);
        action[(size_t)i * A + j] = a;
    }
    if (log_pi) log_pi[i] = lp - corr;
}

}  // namespace rlp

using namespace rlp;

namespace rlp {
int dense_mlp_forward(const rlp_mlp_desc &d, const float *params, const float *x, float *y, int n,
                      float *scratch, hipStream_t s);  // rlp_dense.hip
int64_t dense_mlp_scratch_floats(const rlp_mlp_desc &d, int n);  // rlp_dense.hip (0: chain path)
constexpr int kMlpDenseRows = 2048;

// the path rlp_mlp_forward takes for (desc, n, masked): true = rlp_dense.hip's tiled GEMM / chain
bool mlp_dense_path(const rlp_mlp_desc &d, int n, bool masked) {
    int maxw = 0;
    bool acts_ok = true;
    for (int l = 0; l <= d.n_layers; ++l) maxw = d.dims[l] > maxw ? d.dims[l] : maxw;
    for (int l = 0; l < d.n_layers; ++l)
        acts_ok &= d.act[l] == RLP_ACT_RELU || d.act[l] == RLP_ACT_TANH || d.act[l] == RLP_ACT_NONE;
    // (the GEMM's element offsets are 32-bit: rows x width < 2^31)
    return !masked && n >= kMlpDenseRows && acts_ok && (int64_t)n * maxw < (int64_t(1) << 31);
}
bool mlp_desc_ok(const rlp_mlp_desc *d) {
    if (!d || d->n_layers < 1 || d->n_layers > RLP_MLP_MAX_LAYERS) return false;
    for (int l = 0; l <= d->n_layers; ++l)
        if (d->dims[l] < 1 || d->dims[l] > kMlpMaxW) return false;
    return true;
}
}  // namespace rlp

extern "C" {

int64_t rlp_mlp_param_count(const rlp_mlp_desc *desc) {
    if (!desc || desc->n_layers < 1 || desc->n_layers > RLP_MLP_MAX_LAYERS) return RLP_EINVAL;
    int64_t c = 0;
    for (int l = 0; l < desc->n_layers; ++l)
        c += (int64_t)desc->dims[l] * desc->dims[l + 1] + desc->dims[l + 1];
    return c;
}

int64_t rlp_mlp_forward_workspace_bytes(const rlp_mlp_desc *desc, int n) {
    if (!mlp_desc_ok(desc) || n < 0) return RLP_EINVAL;
    return mlp_dense_path(*desc, n, false) ? 4 * dense_mlp_scratch_floats(*desc, n) : 0;
}

int rlp_mlp_forward(const rlp_mlp_desc *desc, const float *params, const float *x, float *y,
                    int n, const uint8_t *mask, void *workspace, int64_t workspace_bytes,
                    rlp_stream_t stream) {
    RLP_REQUIRE(desc && params && x && y, "rlp_mlp_forward: null argument");
    RLP_REQUIRE(desc->n_layers >= 1 && desc->n_layers <= RLP_MLP_MAX_LAYERS,
                "rlp_mlp_forward: n_layers %d", desc->n_layers);
    int maxw = 0;
    for (int l = 0; l <= desc->n_layers; ++l) {
        RLP_REQUIRE(desc->dims[l] >= 1 && desc->dims[l] <= kMlpMaxW,
                    "rlp_mlp_forward: width %d not in [1, %d]", desc->dims[l], kMlpMaxW);
        maxw = desc->dims[l] > maxw ? desc->dims[l] : maxw;
    }
    if (n <= 0) return n == 0 ? RLP_OK : RLP_EINVAL;
    // large unmasked batches (the off-policy drivers' acting forward over every env) on the tiled
    // GEMM of rlp_dense.hip: one launch per layer, weights staged once per 64-row tile
    if (mlp_dense_path(*desc, n, mask != nullptr)) {
        const int64_t need = 4 * dense_mlp_scratch_floats(*desc, n);
        RLP_REQUIRE(workspace_bytes >= need && (need == 0 || workspace),
                    "rlp_mlp_forward: workspace of %lld bytes, need %lld "
                    "(rlp_mlp_forward_workspace_bytes)", (long long)workspace_bytes, (long long)need);
        return dense_mlp_forward(*desc, params, x, y, n, static_cast<float *>(workspace),
                                 as_stream(stream));
    }
    // row stride: multiple of 32 (+2) so the B-operand reads (16 rows x 2 k per half-wave) hit
    // 32 distinct banks
    const int ldw = ((maxw + 31) / 32) * 32 + 2;
    const size_t lds = sizeof(float) * 2 * 16 * ldw;
    MlpArgs args{*desc};
    mlp_forward_kernel<<<(n + 15) / 16, 64, lds, as_stream(stream)>>>(args, params, x, y, n, mask,
                                                                      ldw);
    RLP_CHECK_LAUNCH("rlp_mlp_forward");
    return RLP_OK;
}

int64_t rlp_mfma_packed_count(const rlp_mlp_desc *desc) {
    MfmaNet net;
    if (!desc || !mfma_net_from_desc(*desc, &net))
        return fail(RLP_EUNSUPPORTED,
                    "rlp_mfma_packed_count: need [S<=8 or 41<=S<=44 -> H -> H -> A<=4], H in {64,128,256}");
    return net.count;
}

int rlp_mfma_pack(const rlp_mlp_desc *desc, const float *params, float *packed,
                  rlp_stream_t stream) {
    RLP_REQUIRE(desc && params && packed, "rlp_mfma_pack: null argument");
    MfmaNet net;
    if (!mfma_net_from_desc(*desc, &net))
        return fail(RLP_EUNSUPPORTED,
                    "rlp_mfma_pack: need [S<=8 or 41<=S<=44 -> H -> H -> A<=4], H in {64,128,256}");
    const int blocks = (int)((net.count + 255) / 256);
    mfma_scale_kernel<<<1, 1024, 0, as_stream(stream)>>>(net, params, packed);
    mfma_pack_kernel<<<blocks < 1024 ? blocks : 1024, 256, 0, as_stream(stream)>>>(net, params,
                                                                                  packed);
    RLP_CHECK_LAUNCH("rlp_mfma_pack");
    return RLP_OK;
}

int rlp_policy_sample(const float *mean, int n, int A, const float *std, const float *a_min,
                      const float *a_max, const float *noise, uint64_t seed, uint64_t counter,
                      uint64_t env_id0, float *action, float *logp, rlp_stream_t stream) {
    RLP_REQUIRE(mean && std && a_min && a_max && action && logp, "rlp_policy_sample: null argument");
    RLP_REQUIRE(A >= 1 && A <= 4, "rlp_policy_sample: A = %d not in [1, 4]", A);
    if (n <= 0) return n == 0 ? RLP_OK : RLP_EINVAL;
    SampleArgs sa;
    for (int j = 0; j < 8; ++j) {
        sa.std[j] = j < A ? std[j] : 1.f;
        sa.a_min[j] = j < A ? a_min[j] : 0.f;
        sa.a_max[j] = j < A ? a_max[j] : 0.f;
    }
    const dim3 grid((n + 255) / 256), block(256);
    hipStream_t s = as_stream(stream);
    switch (A) {
    case 1: policy_sample_kernel<1><<<grid, block, 0, s>>>(mean, n, sa, noise, seed, counter, env_id0, action, logp); break;
    case 2: policy_sample_kernel<2><<<grid, block, 0, s>>>(mean, n, sa, noise, seed, counter, env_id0, action, logp); break;
    case 3: policy_sample_kernel<3><<<grid, block, 0, s>>>(mean, n, sa, noise, seed, counter, env_id0, action, logp); break;
    case 4: policy_sample_kernel<4><<<grid, block, 0, s>>>(mean, n, sa, noise, seed, counter, env_id0, action, logp); break;
    }
    RLP_CHECK_LAUNCH("rlp_policy_sample");
    return RLP_OK;
}

int rlp_sac_sample(const float *head, int n, int A, const float *ls_lo, const float *ls_hi,
                   const float *gain, const float *off, const float *a_min, const float *a_max,
                   int deterministic, const float *noise, uint64_t seed, uint64_t counter,
                   uint64_t env_id0, float *action, float *log_pi, rlp_stream_t stream) {
    RLP_REQUIRE(head && ls_lo && ls_hi && gain && off && action, "rlp_sac_sample: null argument");
    RLP_REQUIRE((a_min == nullptr) == (a_max == nullptr), "rlp_sac_sample: a_min/a_max both or neither");
    RLP_REQUIRE(A >= 1 && A <= 4, "rlp_sac_sample: A = %d not in [1, 4]", A);
    if (n <= 0) return n == 0 ? RLP_OK : RLP_EINVAL;
    SacArgs sa;
    for (int j = 0; j < 4; ++j) {
        const bool on = j < A;
        sa.ls_lo[j] = on ? ls_lo[j] : 0.f;
        sa.ls_hi[j] = on ? ls_hi[j] : 0.f;
        sa.gain[j] = on ? gain[j] : 0.f;
        sa.off[j] = on ? off[j] : 0.f;
        sa.a_min[j] = on && a_min ? a_min[j] : 0.f;
        sa.a_max[j] = on && a_max ? a_max[j] : 0.f;
    }
    sa.clamp_action = a_min != nullptr;
    sa.deterministic = deterministic != 0;
    const dim3 grid((n + 255) / 256), block(256);
    hipStream_t s = as_stream(stream);
    switch (A) {
    case 1: sac_sample_kernel<1><<<grid, block, 0, s>>>(head, n, sa, noise, seed, counter, env_id0, action, log_pi); break;
    case 2: sac_sample_kernel<2><<<grid, block, 0, s>>>(head, n, sa, noise, seed, counter, env_id0, action, log_pi); break;
    case 3: sac_sample_kernel<3><<<grid, block, 0, s>>>(head, n, sa, noise, seed, counter, env_id0, action, log_pi); break;
    case 4: sac_sample_kernel<4><<<grid, block, 0, s>>>(head, n, sa, noise, seed, counter, env_id0, action, log_pi); break;
    }
    RLP_CHECK_LAUNCH("rlp_sac_sample");
    return RLP_OK;
}

}  // extern "C"

