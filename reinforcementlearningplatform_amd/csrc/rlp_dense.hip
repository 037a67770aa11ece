// rlp_dense.hip — batched dense layers and the native DDPG update (algorithm/actor_critic/
// DDPG.py:72-109 learn, :111-118 update_network_parameters) for the drivers' ReLU nets
// (demonstration/DDPG/DDPG-4-*/train.py:26-100: actor S -> 256 -> 256 -> A, relu, relu,
// gain * tanh + off; critic cat(s, a) -> 256 -> 256 -> 1, relu, relu, identity).
//
// Every matrix product of the update — the forward passes (x W^T + b), the backward data passes
// (dY W, masked by the activation's derivative) and the weight gradients (dY^T X, the bias as an
// extra all-ones column of X) — runs through ONE tiled GEMM on v_mfma_f32_16x16x4_f32 (exact f32
// products, f32 accumulation, like torch's f32 GEMMs): 64 x 64 output tiles per 4-wave block,
// each wave a 32 x 32 quarter (2 x 2 MFMA tiles), the reduction staged through LDS 16 deep. The
// operands are strided views (row / column strides, an optional column split for torch.cat and
// an all-ones column), so transposes and concatenations are never materialised. Weight
// gradients split the batch over gridDim.z into partials summed in fixed order (deterministic,
// no atomics) by the optimizer kernel itself: per net one launch sums every layer's partials,
// takes the Adam step (torch.optim.Adam's non-capturable arithmetic, step count read from device
// memory so a captured HIP graph can be replayed) and the soft target update. Fused epilogues:
// + bias, relu, gain * tanh + off (keeping tanh for the backward), relu' mask,
// (. * gain) * (1 - t^2).
#include "rlp_common.hpp"

#include <mutex>

namespace rlp {

// element (i, j) of a rows x cols matrix: columns (rows, with split_rows) [0, split) from p0, the
// rest from p1 (indexed from the split); column `ones` reads 1 (the bias column of a weight
// gradient); out of range reads 0
struct Opnd {
    const float *p0, *p1;
    int rs0, cs0, rs1, cs1;  // element strides (every operand here has < 2^31 elements)
    int rows, cols, split, ones, split_rows;
};

// branch-free: one unconditional load (index 0 of the chosen source when out of range), then
// selects — so a thread's many staged loads issue back to back instead of one per branch
__device__ __forceinline__ float opnd_ld(const Opnd &o, int i, int j) {
    const bool in = i < o.rows && j < o.cols;
    const bool ld = in && j != o.ones;
    const bool second = o.split_rows ? i >= o.split : j >= o.split;
    const int ii = (o.split_rows && second) ? i - o.split : i;
    const int jj = (!o.split_rows && second) ? j - o.split : j;
    const int idx = second ? ii * o.rs1 + jj * o.cs1 : ii * o.rs0 + jj * o.cs0;
    const float v = (second ? o.p1 : o.p0)[ld ? idx : 0];
    // arithmetic, not a select on the loaded value: the backend turns "c ? load : k" into a branch
    // around the load, which serialises the staged loads (v is finite operand data)
    return __builtin_fmaf(v, ld ? 1.f : 0.f, (in && j == o.ones) ? 1.f : 0.f);
}

enum : int { kEpiNone = 0, kEpiRelu, kEpiTanhAff, kEpiReluBack, kEpiTanhAffBack, kEpiPartial, kEpiTanh };

struct Epi {
    float *y;
    int64_t ldy;
    const float *bias;                 // + bias[n] (forward kinds)
    const float *gain, *off;           // kEpiTanhAff: y = gain * tanh(z) + off; kEpiTanhAffBack: gain
    float *aux;                        // kEpiTanhAff: tanh(z) stored here (ldaux)
    int64_t ldaux;
    const float *mask;                 // kEpiReluBack: y = acc where mask > 0 (relu output), else 0
    int64_t ldm;                       // kEpiTanhAffBack: mask holds t = tanh(z)
    int kind, M, N;
};

constexpr int kDT = 64;            // output tile (M and N)
constexpr int kDRc = 128;          // reduction rows one block stages at once (one LDS stage)
constexpr int kDLd = kDRc + 4;     // LDS row: operand row-major along r, 4 banks apart per row
constexpr int kDSlice = 256;       // reduction rows per slice of make_prob (two stages)
constexpr int kDPf = kDT * kDRc / 4 / 256;  // float4 loads per thread of one panel's fast path (8)

// extent of the panel's outer index u (A: rows m; B: columns n)
__device__ __forceinline__ int e_rows(const Opnd &o, bool is_a) { return is_a ? o.rows : o.cols; }

// LDS column of reduction index r in a stage of Q MFMA steps per lane group (Q a multiple of 4,
// <= 32; r < 4 Q): lane group g reads the Q consecutive indices [g Q, g Q + Q) as columns
// [32 g, 32 g + Q), and rows u with bit 3 set swap the 32-column halves (XOR 32). Then every
// 16-lane group of a ds_read_b128 fragment read (rows c = 0..15 at 4 banks apart, two lane groups
// g) hits 64 distinct banks for any Q: with the plain g Q offsets a 128-row stage (Q = 32) put
// lane groups g and g + 1 on the same banks (2-way), and the transposing stores below were 8-way
// (profiles/r5/r5d_pmc_shapes.txt: SQ_LDS_BANK_CONFLICT 0.74-0.78 of the LDS cycles).
__device__ __forceinline__ int lds_col(int r, int Q) {
    const int g = (r >= Q) + (r >= 2 * Q) + (r >= 3 * Q);  // r / Q (r < 4 Q) without a division
    return 32 * g + (r - g * Q);
}
__device__ __forceinline__ int lds_swz(int u) { return (u & 8) << 2; }

// A block's panel of an operand for one stage, as L[u][r] (row stride kDLd): u in [0, 64) the
// outer index (A: m0 + u; B: n0 + u), r in [0, kDRc) the reduction index (r_lo + r; zero past rc).
// Fast path (the panel lies inside one source, off the ones column, fully in range, and is
// contiguous along r or along u with 16-byte alignment): kDPf float4 loads per thread into
// registers (panel_load, issued one stage ahead so they fly under the current stage's MFMAs),
// written to LDS by panel_store. Otherwise the generic element loader, straight to LDS.
struct PanelFast {
    const float *base;
    int u_stride, r_stride;
    bool fast, rfast;
};
__device__ __forceinline__ PanelFast panel_plan(const Opnd &o, bool is_a, int u0, int ubound, int r_lo,
                                                int rc) {
    const int i_lo = is_a ? u0 : r_lo, i_hi = is_a ? u0 + 64 : r_lo + rc;  // [lo, hi)
    const int j_lo = is_a ? r_lo : u0, j_hi = is_a ? r_lo + rc : u0 + 64;
    const int s_lo = o.split_rows ? i_lo : j_lo, s_hi = o.split_rows ? i_hi : j_hi;
    const bool one_src = s_hi <= o.split || s_lo >= o.split;
    const bool second = s_lo >= o.split;
    const bool no_ones = o.ones < j_lo || o.ones >= j_hi;
    const bool inrange = u0 + 64 <= ubound && (rc & 3) == 0;
    const float *p = second ? o.p1 : o.p0;
    const int rs = second ? o.rs1 : o.rs0, cs = second ? o.cs1 : o.cs0;
    const int ioff = (o.split_rows && second) ? o.split : 0, joff = (!o.split_rows && second) ? o.split : 0;
    // contiguity along r or u
    const int r_stride = is_a ? cs : rs, u_stride = is_a ? rs : cs;
    const bool rfast = r_stride == 1 && (u_stride & 3) == 0;
    const bool ufast = u_stride == 1 && (r_stride & 3) == 0;
    const bool aligned = ((uintptr_t)p & 15) == 0 &&
                         (((is_a ? (u0 - ioff) * rs + (r_lo - joff) * cs : (r_lo - ioff) * rs + (u0 - joff) * cs)) & 3) == 0;
    PanelFast f;
    f.fast = one_src && no_ones && inrange && aligned && (rfast || ufast);
    f.rfast = rfast;
    f.base = p + (int64_t)((is_a ? u0 : r_lo) - ioff) * rs + (int64_t)((is_a ? r_lo : u0) - joff) * cs;
    f.u_stride = u_stride;
    f.r_stride = r_stride;
    return f;
}
// rfast thread: r4 = 4 (t & 31), u = (t >> 5) + 8 q; ufast thread: u4 = 4 (t >> 4), r = (t & 15) + 16 q
// (a half-wave of the transposing store then writes two u quads x 16 r: 32 distinct banks; the
// former u4 = 4 (t & 15) mapping wrote 16 u quads x 2 r, 8-way conflicts)
__device__ __forceinline__ void panel_load(const PanelFast &f, int rc, floatx4 (&v)[kDPf]) {
    const int t = threadIdx.x;
    if (f.rfast) {
        const int r4 = 4 * (t & 31);
#pragma unroll
        for (int q = 0; q < kDPf; ++q) {
            const int u = (t >> 5) + 8 * q;
            v[q] = r4 < rc ? *(const floatx4 *)(f.base + (int64_t)u * f.u_stride + r4) : floatx4{0.f, 0.f, 0.f, 0.f};
        }
    } else {
        const int u4 = 4 * (t >> 4);
#pragma unroll
        for (int q = 0; q < kDPf; ++q) {
            const int r = (t & 15) + 16 * q;
            v[q] = r < rc ? *(const floatx4 *)(f.base + (int64_t)r * f.r_stride + u4) : floatx4{0.f, 0.f, 0.f, 0.f};
        }
    }
}
// the stage's panel into L (columns lds_col; reduction indices past 4 Q are never read: skipped)
__device__ __forceinline__ void panel_store(const PanelFast &f, const floatx4 (&v)[kDPf], float *L, int Q) {
    const int t = threadIdx.x;
    if (f.rfast) {
        const int r4 = 4 * (t & 31);
        const int col = r4 < 4 * Q ? lds_col(r4, Q) : -1;
        if (col >= 0) {
#pragma unroll
            for (int q = 0; q < kDPf; ++q) {
                const int u = (t >> 5) + 8 * q;
                *(floatx4 *)&L[u * kDLd + (col ^ lds_swz(u))] = v[q];
            }
        }
    } else {
        const int u4 = 4 * (t >> 4), sw = lds_swz(u4);
#pragma unroll
        for (int q = 0; q < kDPf; ++q) {
            const int r = (t & 15) + 16 * q;
            if (r < 4 * Q) {
                const int col = lds_col(r, Q) ^ sw;
#pragma unroll
                for (int k = 0; k < 4; ++k) L[(u4 + k) * kDLd + col] = v[q][k];
            }
        }
    }
}
// generic element loader (the panel is not on the fast path). Rows u past ubound are left as they
// are (their outputs are never stored); columns r in [rc, nr) are zeroed (they meet valid outputs
// in the MFMAs).
__device__ __forceinline__ void panel_generic(const Opnd &o, bool is_a, int u0, int ubound, int r_lo,
                                              int rc, int nr, float *L) {
    const int t = threadIdx.x;
    // (i, j) of panel element (u, r)
    auto ij = [&](int u, int r, int &i, int &j) {
        i = is_a ? u0 + u : r_lo + r;
        j = is_a ? r_lo + r : u0 + u;
    };
    const int nu = ubound - u0 < 64 ? ubound - u0 : 64;
    if (nu <= 16) {  // few valid u (a last layer's W, an edge tile): thread = r, loop over u
        const int r = t;
        if (r < nr) {
            float v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                int i, j;
                ij(u, r, i, j);
                const bool ok = u < nu && r < rc;
                v[u] = opnd_ld(o, ok ? i : 0x7fffffff, ok ? j : 0x7fffffff);
            }
            const int col = lds_col(r, nr / 4);
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (u < nu) L[u * kDLd + (col ^ lds_swz(u))] = v[u];
        }
        return;
    }
    // thread = u (t & 63) and every 4th r from t >> 6, 8 loads in flight per step
    const int u = t & 63;
    if (u >= nu) return;
#pragma unroll 1
    for (int r0 = t >> 6; r0 < nr; r0 += 32) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int r = r0 + 4 * k;
            int i, j;
            ij(u, r, i, j);
            const bool ok = r < rc;
            v[k] = opnd_ld(o, ok ? i : 0x7fffffff, ok ? j : 0x7fffffff);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (r0 + 4 * k < nr) L[u * kDLd + (lds_col(r0 + 4 * k, nr / 4) ^ lds_swz(u))] = v[k];
    }
}

// C[M x N] = sum_r A(m, r) B(r, n) over r in [z * rchunk, min(R, (z + 1) * rchunk)), rchunk <= 256
// (make_prob; make_prob_long: longer). The block stages its slice 128 rows at a time: both
// operands' panels of a stage in one burst of 16-byte loads (64 registers per lane), the next
// stage's burst issued right after the current stage lands in LDS so that it flies under the
// current stage's MFMAs. 67.6 KB of LDS per block: two blocks per CU, so a launch of more blocks
// than CUs (a weight gradient beside its backward data pass, the twin critic's two chains)
// overlaps one block's loads with the other's MFMAs instead of running in rounds of one block per
// CU (DDPG learn(): the layer-1 weight-gradient + backward launch was 42 us in three rounds,
// profiles/r4/r4e_ddpg_learn_timeline.txt). LDS holds A as [m][r] and B as [n][r] (row stride
// 132 floats, columns lds_col / lds_swz: conflict-free fragment reads and stores); the reduction
// order is permuted so that each lane's operands for four consecutive MFMA steps are contiguous
// (one 16-byte LDS read): step s, lane group g reads r = g * Q + s.
struct Prob {
    Opnd A, B;
    Epi e;
    int R, rchunk;   // reduction length, rows per slice
    int nx, ny, nz;  // column tiles, row tiles, reduction slices
};

// Up to kMaxProbs independent problems in one launch (the twin critic's chains, a layer's weight
// gradient beside its backward data pass, every layer's weight gradient of a net after the fused
// data chain): the 1-D grid's blocks [start[i], start[i + 1]) run problem i.
constexpr int kMaxProbs = 6;
struct ProbSet {
    Prob p[kMaxProbs];
    int start[kMaxProbs + 1];
    int n;
};
__global__ void __launch_bounds__(256) dense_gemm_kernel(ProbSet ps) {
    extern __shared__ float lds[];
    float *As = lds, *Bs = lds + kDT * kDLd;
    int pi = 0;  // block-uniform
#pragma unroll
    for (int k = 1; k < kMaxProbs; ++k)
        if (k < ps.n && (int)blockIdx.x >= ps.start[k]) pi = k;
    const Prob &q = ps.p[pi];
    const Opnd A = q.A, B = q.B;
    const Epi e = q.e;
    const int R = q.R, rchunk = q.rchunk, nx = q.nx, ny = q.ny;
    const int bid = (int)blockIdx.x - ps.start[pi];
    const int bx = bid % nx, by = (bid / nx) % ny, bz = bid / (nx * ny);
    const int m0 = by * kDT, n0 = bx * kDT;
    // the block's reduction slice [r_lo, r_end), staged kDRc rows at a time; the next stage's
    // fast-path panels are loaded into registers while the current stage's MFMAs run
    const int r_lo = bz * rchunk, r_end = min(R, r_lo + rchunk);
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
    floatx4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int g = l >> 4, c = l & 15;
    const int ua = e_rows(A, true), ub = e_rows(B, false);
    floatx4 va[kDPf], vb[kDPf];
    int rc = min(r_end, r_lo + kDRc) - r_lo;
    PanelFast fa = panel_plan(A, true, m0, ua, r_lo, rc), fb = panel_plan(B, false, n0, ub, r_lo, rc);
    if (fa.fast) panel_load(fa, rc, va);
    if (fb.fast) panel_load(fb, rc, vb);
    for (int rs = r_lo; rs < r_end || rs == r_lo; rs += kDRc) {
        const int Q = (rc + 15) / 16 * 4;  // MFMA steps (multiple of 4); rows g * Q + s, s < Q
        if (rs != r_lo) __syncthreads();   // the previous stage's fragments are read
        if (fa.fast) panel_store(fa, va, As, Q); else panel_generic(A, true, m0, ua, rs, rc, 4 * Q, As);
        if (fb.fast) panel_store(fb, vb, Bs, Q); else panel_generic(B, false, n0, ub, rs, rc, 4 * Q, Bs);
        __syncthreads();
        const int rn = rs + kDRc, rcn = min(r_end, rn + kDRc) - rn;
        if (rn < r_end) {  // next stage's loads, in flight under this stage's MFMAs
            fa = panel_plan(A, true, m0, ua, rn, rcn);
            fb = panel_plan(B, false, n0, ub, rn, rcn);
            if (fa.fast) panel_load(fa, rcn, va);
            if (fb.fast) panel_load(fb, rcn, vb);
        }
        const int fcol = (32 * g) ^ lds_swz(c);  // lane group g's columns (rows wm + 16 i + c: c's bit 3)
        for (int s = 0; s < Q; s += 4) {
            floatx4 af[2], bf[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = *(const floatx4 *)&As[(wm + 16 * i + c) * kDLd + fcol + s];
#pragma unroll
            for (int j = 0; j < 2; ++j) bf[j] = *(const floatx4 *)&Bs[(wn + 16 * j + c) * kDLd + fcol + s];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][u], bf[j][u], acc[i][j], 0, 0, 0);
        }
        if (rc <= 0) break;
        rc = rcn;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int m = m0 + wm + 16 * i + 4 * (l >> 4) + q, n = n0 + wn + 16 * j + (l & 15);
                if (m >= e.M || n >= e.N) continue;
                float v = acc[i][j][q];
                switch (e.kind) {
                case kEpiPartial:
                    e.y[(size_t)bz * e.M * e.N + (size_t)m * e.N + n] = v;
                    continue;
                case kEpiReluBack:
                    v = e.mask[m * e.ldm + n] > 0.f ? v : 0.f;
                    break;
                case kEpiTanhAffBack: {  // torch: grad_t = da * gain; grad_z = grad_t * (1 - t*t)
                    const float tt = e.mask[m * e.ldm + n];
                    v = (v * e.gain[n]) * (1.f - tt * tt);
                    break;
                }
                default:
                    if (e.bias) v = v + e.bias[n];
                    if (e.kind == kEpiRelu) {
                        v = fmaxf(v, 0.f);
                    } else if (e.kind == kEpiTanh) {
                        v = tanhf(v);
                    } else if (e.kind == kEpiTanhAff) {
                        const float tt = tanhf(v);
                        e.aux[m * e.ldaux + n] = tt;
                        v = e.gain[n] * tt + e.off[n];
                    }
                }
                e.y[m * e.ldy + n] = v;
            }
}

// grad[m][n] = sum over the splits of the partials; column N-1 is the bias. 64 outputs per block
// x kWrSlices slices: each thread sums every kWrSlices-th split (8 loads in flight), then a
// fixed-order LDS combine — deterministic; the PPO2 dense update's long reductions leave up to
// 512 partials per element, which one thread per element walked with one latency each.
// blockIdx.y = 1: the second problem of a twin launch (part1 -> gW1, gb1)
constexpr int kWrSlices = 16;
__global__ void __launch_bounds__(64 * kWrSlices) wgrad_reduce_kernel(const float *__restrict__ part0,
                                                                      int splits, int M, int N,
                                                                      float *__restrict__ gW0,
                                                                      float *__restrict__ gb0,
                                                                      const float *__restrict__ part1,
                                                                      float *__restrict__ gW1,
                                                                      float *__restrict__ gb1) {
    const float *part = blockIdx.y ? part1 : part0;
    float *gW = blockIdx.y ? gW1 : gW0, *gb = blockIdx.y ? gb1 : gb0;
    const int o = threadIdx.x & 63, sl = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + o;
    float s = 0.f;
    if (i < M * N) {
#pragma unroll 8
        for (int z = sl; z < splits; z += kWrSlices) s += part[(size_t)z * M * N + i];
    }
    __shared__ float red[kWrSlices][64];
    red[sl][o] = s;
    __syncthreads();
    if (sl != 0 || i >= M * N) return;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kWrSlices; ++k) t += red[k][o];
    const int m = i / N, n = i - m * N;
    if (n < N - 1)
        gW[(size_t)m * (N - 1) + n] = t;
    else
        gb[m] = t;
}

// NetParts is declared below; the multi-layer reduce takes its fields directly
constexpr int kMaxRegions = 8;
struct PartRegions {
    const float *part[kMaxRegions];
    int64_t off[kMaxRegions];  // the layer's W in g (its bias follows)
    int z[kMaxRegions], in[kMaxRegions], out[kMaxRegions];
    int n;
};
// every layer's weight gradient of one net from its partials in one launch: wgrad_reduce_kernel's
// sliced sum (the same order: the same bits) over the concatenated outputs of the regions; g
// elements outside every region are left alone
__global__ void __launch_bounds__(64 * kWrSlices) parts_reduce_kernel(float *__restrict__ g, int64_t n,
                                                                       PartRegions pr) {
    const int o = threadIdx.x & 63, sl = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 64 + o;
    int l = -1;
    int64_t idx = 0, stride = 0;
    for (int k = 0; k < pr.n; ++k) {
        const int64_t r = i - pr.off[k], in = pr.in[k], out = pr.out[k];
        if (i < n && r >= 0 && r < out * (in + 1)) {
            l = k;
            idx = r < in * out ? (r / in) * (in + 1) + r % in : (r - in * out) * (in + 1) + in;
            stride = out * (in + 1);
        }
    }
    float s = 0.f;
    if (l >= 0) {
        const float *part = pr.part[l];
        const int z = pr.z[l];
#pragma unroll 8
        for (int zz = sl; zz < z; zz += kWrSlices) s += part[(size_t)zz * stride + idx];
    }
    __shared__ float red[kWrSlices][64];
    red[sl][o] = s;
    __syncthreads();
    if (sl != 0 || l < 0) return;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kWrSlices; ++k) t += red[k][o];
    g[i] = t;
}

// TD target + critic MSE gradient (DDPG.py:83-89): y = r + (gamma * end) * Q'; dQ = d/dQ of
// mse_loss(y, Q) = -((2 / B) * (y - Q)); loss = mean((y - Q)^2). One block; also advances the
// two Adam step counters (actor, critic) the update's optimizer steps read.
__global__ void __launch_bounds__(1024) ddpg_td_kernel(const float *__restrict__ r,
                                                       const float *__restrict__ end,
                                                       const float *__restrict__ q_next,
                                                       const float *__restrict__ q, int B, float gamma,
                                                       float *__restrict__ dq, float *loss,
                                                       int32_t *steps) {
    __shared__ double red[16];
    double s = 0;
    const float two_b = 2.f / (float)B;
    for (int i = threadIdx.x; i < B; i += 1024) {
        const float y = r[i] + (gamma * end[i]) * q_next[i];
        const float d = y - q[i];
        dq[i] = -(two_b * d);
        s += (double)d * (double)d;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0;
        for (int k = 0; k < 16; ++k) tot += red[k];
        loss[0] = (float)(tot / B);
        steps[0] += 1;
        steps[1] += 1;
    }
}

// actor loss -mean(Q(s, mu(s))) and its gradient dQ = -(1 / B) per row (DDPG.py:97)
__global__ void __launch_bounds__(1024) ddpg_actor_loss_kernel(const float *__restrict__ q, int B,
                                                               float *__restrict__ dq, float *loss) {
    __shared__ double red[16];
    double s = 0;
    const float g = -(1.f / (float)B);
    for (int i = threadIdx.x; i < B; i += 1024) {
        s += (double)q[i];
        dq[i] = g;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0;
        for (int k = 0; k < 16; ++k) tot += red[k];
        loss[1] = (float)(-(tot / B));
    }
}

// torch.optim.Adam step (non-capturable arithmetic) with the step count read from the device
__global__ void __launch_bounds__(256) adam_dev_kernel(float *__restrict__ p, const float *__restrict__ g,
                                                       float *__restrict__ m, float *__restrict__ v,
                                                       int64_t n, float lr, float beta1, float beta2,
                                                       float eps, const int32_t *step) {
    const float st = (float)*step;
    const float bc1 = 1.f - powf(beta1, st);
    const float bc2 = 1.f - powf(beta2, st);
    const float step_size = lr / bc1, bc2_sqrt = sqrtf(bc2);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float gi = g[i];
        float mi = m[i];
        mi = mi + (1.f - beta1) * (gi - mi);
        const float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = p[i] + (-step_size) * (mi / denom);
    }
}

// The weight-gradient partials of the layers of one parameter buffer ([z][out][in + 1] each, the
// bias as the last column), left unreduced by the backward pass for adam_reduce_kernel
constexpr int kMaxParts = 8;  // a net's layers (SAC: both critic chains, the actor's two heads)
struct NetParts {
    const float *part[kMaxParts];
    int64_t off[kMaxParts];  // the layer's W in the flat parameters (b follows)
    int z[kMaxParts], in[kMaxParts], out[kMaxParts];
    int n;
};

// One launch for what wgrad_reduce (per layer), Adam and the soft target update did in five: the
// gradient element summed over its layer's partials in split order (DDPG / SAC: 16 splits of 256
// batch rows), stored to g, the Adam step on it, and — when tp is set — the soft target update
// with the new parameter, tp (1 - tau) + p tau (DDPG.py:113-118, Soft_Actor_Critic.py:126-127;
// the target is not read again in the update).
// Elements outside every layer (a module's unused parameters) keep the gradient in g.
__global__ void __launch_bounds__(256) adam_reduce_kernel(float *__restrict__ p, float *__restrict__ g,
                                                          float *__restrict__ m, float *__restrict__ v,
                                                          int64_t n, NetParts np, float lr, float beta1,
                                                          float beta2, float eps, const int32_t *step,
                                                          float *__restrict__ tp, float keep, float take) {
    const float st = (float)*step;
    const float bc1 = 1.f - powf(beta1, st);
    const float bc2 = 1.f - powf(beta2, st);
    const float step_size = lr / bc1, bc2_sqrt = sqrtf(bc2);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float gi = g[i];
        for (int l = 0; l < np.n; ++l) {
            const int64_t r = i - np.off[l], in = np.in[l], out = np.out[l];
            if (r < 0 || r >= out * (in + 1)) continue;
            const int64_t idx = r < in * out ? (r / in) * (in + 1) + r % in : (r - in * out) * (in + 1) + in;
            const int64_t stride = out * (in + 1);
            float s = 0.f;
#pragma unroll 8
            for (int zz = 0; zz < np.z[l]; ++zz) s += np.part[l][zz * stride + idx];
            gi = s;
            g[i] = s;
        }
        float mi = m[i];
        mi = mi + (1.f - beta1) * (gi - mi);
        const float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        const float pi = p[i] + (-step_size) * (mi / denom);
        p[i] = pi;
        if (tp) tp[i] = tp[i] * keep + pi * take;
    }
}

// ---- SAC (algorithm/actor_critic/Soft_Actor_Critic.py:70-129) --------------------------------
__device__ __forceinline__ float softplus_t(float x) {  // torch softplus(beta=1, threshold=20)
    return x > 20.f ? x : log1pf(expf(x));
}

// the actor's squashed-Gaussian head on z = [mean | log_std] pre-bias (utils/classes.py SACActor
// forward): ls = clamp(z + b, lo, hi), std = exp(ls), u = mean + eps * std (Normal.rsample),
// log_pi = sum log_prob(u) - sum 2 (log 2 - u - softplus(-2u)), a = tanh(u) * gain + off. TRAIN
// keeps u, std, eps, tanh(u) and the clamp's pass mask for the backward.
template <int A, bool TRAIN>
__global__ void __launch_bounds__(256) sac_head_kernel(const float *__restrict__ z, int B,
                                                       const float *bm, const float *bl,
                                                       const float *ls_lo, const float *ls_hi,
                                                       const float *gain, const float *off,
                                                       const float *noise, uint64_t seed,
                                                       const uint64_t *counter, uint64_t draw,
                                                       float *__restrict__ act, float *__restrict__ lp,
                                                       float *__restrict__ save) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= B) return;
    float eps[A];
    if (noise) {
#pragma unroll
        for (int j = 0; j < A; ++j) eps[j] = noise[(size_t)i * A + j];
    } else {
        // draw + 1 in the high bits: the update's stream never meets rlp_sac_sample's exploration
        // draws, which key (seed, counter, env id) with env ids below 2^40
        philox_normal_f32<A>(seed, *counter, (uint64_t)i + ((draw + 1) << 40), eps);
    }
    const float kHalfLog2Pi = 0.918938533204672742f, kLog2 = 0.693147180559945309f;
    float l = 0.f, corr = 0.f;
#pragma unroll
    for (int j = 0; j < A; ++j) {
        const float mean = z[(size_t)i * 2 * A + j] + bm[j];
        const float x = z[(size_t)i * 2 * A + A + j] + bl[j];
        const float ls = fminf(fmaxf(x, ls_lo[j]), ls_hi[j]);
        const float sd = expf(ls);
        const float u = mean + eps[j] * sd;
        const float d = u - mean;
        const float lpj = -(d * d) / (2.f * (sd * sd)) - logf(sd) - kHalfLog2Pi;
        l = j == 0 ? lpj : l + lpj;
        const float cj = 2.f * ((kLog2 - u) - softplus_t(-2.f * u));
        corr = j == 0 ? cj : corr + cj;
        const float t = tanhf(u);
        act[(size_t)i * A + j] = t * gain[j] + off[j];
        if (TRAIN) {  // [6][B][A]: u, std, eps, tanh(u), clamp pass, u - mean
            const size_t o = (size_t)i * A + j, st = (size_t)B * A;
            save[o] = u;
            save[st + o] = sd;
            save[2 * st + o] = eps[j];
            save[3 * st + o] = t;
            save[4 * st + o] = (x >= ls_lo[j] && x <= ls_hi[j]) ? 1.f : 0.f;
            save[5 * st + o] = d;
        }
    }
    lp[i] = l - corr;
}

__device__ __forceinline__ float sac_alpha(const float *log_alpha, int adaptive, float alpha) {
    return adaptive ? expf(*log_alpha) : alpha;
}

// target_Q = r + (gamma * (1 - dw)) * (min(Q1', Q2') - alpha * log_pi')  (:75-78)
__global__ void __launch_bounds__(256) sac_target_kernel(const float *__restrict__ r,
                                                         const float *__restrict__ dw,
                                                         const float *__restrict__ q1,
                                                         const float *__restrict__ q2,
                                                         const float *__restrict__ lp, int B,
                                                         float gamma, const float *log_alpha,
                                                         int adaptive, float alpha_fixed,
                                                         float *__restrict__ tq) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= B) return;
    const float al = sac_alpha(log_alpha, adaptive, alpha_fixed);
    const float m = fminf(q1[i], q2[i]) - al * lp[i];
    tq[i] = r[i] + (gamma * (1.f - dw[i])) * m;
}

// actor loss mean(alpha * log_pi - min(Q1, Q2)) and d/dQ1, d/dQ2 (torch.minimum's backward: ties
// split the gradient in half); the temperature's gradient exp(log_alpha) * sum(-(log_pi + H)/B);
// advances the Adam step counts and the noise counter (both samples of this update are drawn).
__global__ void __launch_bounds__(1024) sac_actor_loss_kernel(const float *__restrict__ q1,
                                                              const float *__restrict__ q2,
                                                              const float *__restrict__ lp, int B,
                                                              const float *log_alpha, int adaptive,
                                                              float alpha_fixed, float target_entropy,
                                                              float *__restrict__ g1,
                                                              float *__restrict__ g2, float *losses,
                                                              float *alpha_grad, int32_t *steps,
                                                              uint64_t *counter) {
    __shared__ double red[2][16];
    const float al = sac_alpha(log_alpha, adaptive, alpha_fixed);
    const float g = -(1.f / (float)B), h = g / 2.f;
    double sl = 0, sa = 0;
    for (int i = threadIdx.x; i < B; i += 1024) {
        const float a = q1[i], b = q2[i];
        g1[i] = a == b ? h : a < b ? g : 0.f;
        g2[i] = a == b ? h : a > b ? g : 0.f;
        sl += (double)(al * lp[i] - fminf(a, b));
        sa += (double)(g * (lp[i] + target_entropy));
    }
    for (int o = 32; o > 0; o >>= 1) {
        sl += __shfl_xor(sl, o);
        sa += __shfl_xor(sa, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = sl;
        red[1][threadIdx.x >> 6] = sa;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double tl = 0, ta = 0;
        for (int k = 0; k < 16; ++k) {
            tl += red[0][k];
            ta += red[1][k];
        }
        losses[1] = (float)(tl / B);
        if (adaptive) alpha_grad[0] = (float)ta * expf(*log_alpha);
        steps[0] += 1;
        steps[1] += 1;
        steps[2] += 1;
        counter[0] += 1;
    }
}

// d(actor loss)/d[mean | log_std pre-clamp] per row from da (both critic chains' input
// gradients at a) and the log-prob terms (G = alpha / B per row's log_pi)
template <int A>
__global__ void __launch_bounds__(256) sac_head_back_kernel(const float *__restrict__ save,
                                                            const float *__restrict__ da1,
                                                            const float *__restrict__ da2, int B,
                                                            const float *gain, const float *log_alpha,
                                                            int adaptive, float alpha_fixed,
                                                            float *__restrict__ gz) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= B) return;
    const float G = (1.f / (float)B) * sac_alpha(log_alpha, adaptive, alpha_fixed);
    const size_t st = (size_t)B * A;
#pragma unroll
    for (int j = 0; j < A; ++j) {
        const size_t o = (size_t)i * A + j;
        const float u = save[o], sd = save[st + o], eps = save[2 * st + o], t = save[3 * st + o];
        const float pass = save[4 * st + o];
        const float da = da1[o] + da2[o];
        const float d = save[5 * st + o];  // u - mean
        const float var = sd * sd;
        const float sig = 1.f / (1.f + expf(2.f * u));  // sigmoid(-2u) (softplus' at -2u)
        const float dsq = -2.f * u > 20.f ? 1.f : sig;
        const float gu = (da * gain[j]) * (1.f - t * t) + G * (-(d / var) + (2.f - 4.f * dsq));
        const float gmean = gu + G * (d / var);
        const float gsd = gu * eps + G * ((d * d) / (var * sd) - 1.f / sd);
        gz[(size_t)i * 2 * A + j] = gmean;
        gz[(size_t)i * 2 * A + A + j] = pass != 0.f ? gsd * sd : 0.f;
    }
}

// critic loss MSE(Q1, y) + MSE(Q2, y) and its gradients (2 / B) (Qk - y)  (:110-113)
__global__ void __launch_bounds__(1024) sac_critic_loss_kernel(const float *__restrict__ q1,
                                                               const float *__restrict__ q2,
                                                               const float *__restrict__ tq, int B,
                                                               float *__restrict__ g1,
                                                               float *__restrict__ g2, float *losses) {
    __shared__ double red[2][16];
    const float nb = 2.f / (float)B;
    double s1 = 0, s2 = 0;
    for (int i = threadIdx.x; i < B; i += 1024) {
        const float d1 = q1[i] - tq[i], d2 = q2[i] - tq[i];
        g1[i] = nb * d1;
        g2[i] = nb * d2;
        s1 += (double)d1 * d1;
        s2 += (double)d2 * d2;
    }
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o);
        s2 += __shfl_xor(s2, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = s1;
        red[1][threadIdx.x >> 6] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t1 = 0, t2 = 0;
        for (int k = 0; k < 16; ++k) {
            t1 += red[0][k];
            t2 += red[1][k];
        }
        losses[0] = (float)(t1 / B) + (float)(t2 / B);
    }
}

// ---- fused forward of a three- or four-layer chain ----------------------------------------------
// [K0 -> H1 -> H2 (-> Hm) -> NO] with relu or tanh hidden layers (the DDPG demo nets, the SAC
// critics and actor trunk + heads, the PPO2 demo nets), 16 or 32 rows per block, all layers in one
// launch instead of one GEMM launch per layer: the block's input rows and the hidden activations
// stay in LDS between the layers (and go to HBM once, for the backward's masks and weight
// gradients; not at all for batched inference). Exact f32 products
// (v_mfma_f32_16x16x4_f32). Eight waves per block (two per SIMD: one wave's loads and VALU under
// the other's MFMAs). Layer 1 / 2: wave w owns the 16-column tiles t = w + 8 j, j < NT1 / NT2
// (compile-time: every MFMA and load unconditional — a guarded tile made each MFMA a branch with a
// vmcnt(0) in front, which serialised the weight loads: 43 us per DDPG chain at batch 4096); lane
// (g, c) feeds A = the activation row c at k = kb + 4 g + u and B = W[16 t + c][kb + 4 g + u] for
// the four steps u of a 16-deep k block, so both operands are 16-byte reads (LDS / the L2-resident
// weights; the packed parameter buffers leave some W unaligned — global loads take that). The
// weights of a 16-deep block load one 32-deep pass ahead of its MFMAs (two register sets, unrolled
// by two: a register copy of an in-flight load would wait for it). Tiles past the width
// read a clamped row and are not stored. Layer 3 (NO <= 8 outputs): the 64 lanes of a wave split
// k, one wave per 2 rows, a shuffle tree per output.
// a 16-byte weight read at 4-byte alignment: the packed parameter buffers put some layers' W at
// offsets that are not multiples of 4 floats (the SAC critic's Q2 chain); gfx950's global loads
// take unaligned addresses, and this type tells the compiler so instead of promising 16
typedef float floatx4_a4 __attribute__((ext_vector_type(4), aligned(4)));
struct ChainArgs {
    const float *x0, *x1;  // input columns [0, split) from x0 (row stride ld0), the rest from x1
    int ld0, ld1, split, K0;
    const float *W1, *b1, *W2, *b2, *W3, *b3;
    const float *W3b;      // output rows [split3, NO) of layer 3 from W3b (the SAC actor's two heads)
    int split3;            // (b3 may be null: no layer-3 bias)
    int H1, H2, NO, B;
    float *h1, *h2, *y;    // [B][H1], [B][H2], [B][NO]
    int head;              // 0: y = z; 1: t = tanh(z) into aux, y = gain t + off; 2: y = tanh(z)
                           // (h1 / h2 null: the hidden activations are not stored — inference)
    const float *gain, *off;
    float *aux;
    int hact;              // hidden activation: 0 relu, 1 tanh (the PPO2 nets)
    const float *Wm, *bm;  // optional fourth layer between layer 2 and the head: H2 -> Hm (Hm <= 128;
    int Hm;                // Hm = 0: none), activations to hm [B][Hm]; the head then reads Hm inputs
    float *hm;
};
constexpr int kChRows = 16, kChK0 = 64, kChH = 256, kChLd = kChH + 4;
__device__ __forceinline__ float chain_act(float x, int hact) { return hact ? tanhf(x) : fmaxf(x, 0.f); }
constexpr int kChWaves = 8, kChThreads = 64 * kChWaves, kChRpw = kChRows / kChWaves;  // rows per wave (layer 3)
constexpr int kChMaxNt = kChH / 16 / kChWaves;  // 16-column tiles per wave at the widest layer

// acc[j] += A (16 x 16, fragments f) x B (16 x 16 of tile j, fragments b[j]) over one 16-deep block
template <int NT>
__device__ __forceinline__ void chain_block(const floatx4 &f, const floatx4 (&b)[NT], floatx4 (&acc)[NT]) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[u], b[j][u], acc[j], 0, 0, 0);
}

template <int NT1, int NT2, int RT, int NTM, int LD = kChLd, int KX = kChK0>
__global__ void __launch_bounds__(kChThreads) chain3_fwd_kernel(ChainArgs a0, ChainArgs a1) {
    constexpr int ROWS = kChRows * RT, RPW = ROWS / kChWaves;  // block rows, layer-3 rows per wave
    const ChainArgs &a = blockIdx.y ? a1 : a0;
    __shared__ __attribute__((aligned(16))) float xs[ROWS][KX + 4];
    __shared__ __attribute__((aligned(16))) float hs1[ROWS][LD];
    __shared__ __attribute__((aligned(16))) float hs2[ROWS][LD];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, g = lane >> 4, c = lane & 15;
    const int r0 = blockIdx.x * ROWS;
    const int K8 = (a.K0 + 7) & ~7;  // zero-padded input columns: two 4-deep steps per pass
    // both layers' first weight fragments are in flight before the input rows land (they do not
    // depend on them: one L2 / HBM latency less on the chain's critical path)
    int row1[NT1], row2[NT2];
#pragma unroll
    for (int j = 0; j < NT1; ++j) {
        const int n = 16 * (w + kChWaves * j) + c;
        row1[j] = n < a.H1 ? n : a.H1 - 1;
    }
#pragma unroll
    for (int j = 0; j < NT2; ++j) {
        const int n = 16 * (w + kChWaves * j) + c;
        row2[j] = n < a.H2 ? n : a.H2 - 1;
    }
    auto ld1 = [&](int k, float (&v)[NT1]) {  // k past K0: a clamped column (its x is 0)
        const int kk = k < a.K0 ? k : a.K0 - 1;
#pragma unroll
        for (int j = 0; j < NT1; ++j) v[j] = a.W1[(int64_t)row1[j] * a.K0 + kk];
    };
    auto ld2 = [&](int kb, floatx4 (&v)[NT2]) {  // kb past H1: a clamped reload, unused
        const int k = (kb < a.H1 ? kb : a.H1 - 16) + 4 * g;
#pragma unroll
        for (int j = 0; j < NT2; ++j) v[j] = *reinterpret_cast<const floatx4_a4 *>(a.W2 + (int64_t)row2[j] * a.H1 + k);
    };
    float wa[NT1], wb[NT1];
    floatx4 ba[NT2], bb[NT2];
    ld1(g, wa);
    ld2(0, ba);
    ld2(16, bb);
    for (int i = t; i < ROWS * K8; i += kChThreads) {
        const int rr = i / K8, k = i % K8, r = r0 + rr;
        float v = 0.f;
        if (r < a.B && k < a.K0) v = k < a.split ? a.x0[(int64_t)r * a.ld0 + k] : a.x1[(int64_t)r * a.ld1 + k - a.split];
        xs[rr][k] = v;
    }
    __syncthreads();
    // layer 1: k outer (one W1 element per tile and step, the next step's in flight)
    {
        floatx4 acc[RT][NT1];
#pragma unroll
        for (int j = 0; j < NT1; ++j) {
            const float b1 = a.b1[row1[j]];
#pragma unroll
            for (int q = 0; q < RT; ++q) acc[q][j] = floatx4{b1, b1, b1, b1};
        }
        for (int k4 = 0; k4 < K8; k4 += 8) {
            ld1(k4 + 4 + g, wb);
#pragma unroll
            for (int q = 0; q < RT; ++q) {
                const float x0 = xs[16 * q + c][k4 + g];
#pragma unroll
                for (int j = 0; j < NT1; ++j) acc[q][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(x0, wa[j], acc[q][j], 0, 0, 0);
            }
            ld1(k4 + 8 + g, wa);
#pragma unroll
            for (int q = 0; q < RT; ++q) {
                const float x1 = xs[16 * q + c][k4 + 4 + g];
#pragma unroll
                for (int j = 0; j < NT1; ++j) acc[q][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(x1, wb[j], acc[q][j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < NT1; ++j) {
            const int n = 16 * (w + kChWaves * j) + c;
            if (n >= a.H1) continue;
#pragma unroll
            for (int q = 0; q < RT; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rr = 16 * q + 4 * g + i;
                    const float v = chain_act(acc[q][j][i], a.hact);
                    hs1[rr][n] = v;
                    if (a.h1 && r0 + rr < a.B) a.h1[(int64_t)(r0 + rr) * a.H1 + n] = v;
                }
        }
    }
    __syncthreads();
    // layer 2 (H1 a multiple of 32); each B fragment feeds the RT row tiles
    {
        floatx4 acc[RT][NT2];
#pragma unroll
        for (int j = 0; j < NT2; ++j) {
            const float b2 = a.b2[row2[j]];
#pragma unroll
            for (int q = 0; q < RT; ++q) acc[q][j] = floatx4{b2, b2, b2, b2};
        }
        for (int kb = 0; kb < a.H1; kb += 32) {  // (sched barriers: the scheduler sinks the loads)
            floatx4 f0[RT], f1[RT];
#pragma unroll
            for (int q = 0; q < RT; ++q) {
                f0[q] = *reinterpret_cast<const floatx4 *>(&hs1[16 * q + c][kb + 4 * g]);
                f1[q] = *reinterpret_cast<const floatx4 *>(&hs1[16 * q + c][kb + 16 + 4 * g]);
            }
#pragma unroll
            for (int q = 0; q < RT; ++q) chain_block<NT2>(f0[q], ba, acc[q]);
            __builtin_amdgcn_sched_barrier(0);
            ld2(kb + 32, ba);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < RT; ++q) chain_block<NT2>(f1[q], bb, acc[q]);
            __builtin_amdgcn_sched_barrier(0);
            ld2(kb + 48, bb);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < NT2; ++j) {
            const int n = 16 * (w + kChWaves * j) + c;
            if (n >= a.H2) continue;
#pragma unroll
            for (int q = 0; q < RT; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rr = 16 * q + 4 * g + i;
                    const float v = chain_act(acc[q][j][i], a.hact);
                    hs2[rr][n] = v;
                    if (a.h2 && r0 + rr < a.B) a.h2[(int64_t)(r0 + rr) * a.H2 + n] = v;
                }
        }
    }
    __syncthreads();
    if constexpr (NTM > 0) {  // the fourth layer (H2 a multiple of 32): hs2 -> hs1 (layer 2 has read hs1)
        int rowm[NTM];
        floatx4 acc[RT][NTM], ma[NTM], mb[NTM];
#pragma unroll
        for (int j = 0; j < NTM; ++j) {
            const int n = 16 * (w + kChWaves * j) + c;
            rowm[j] = n < a.Hm ? n : a.Hm - 1;
            const float bv = a.bm[rowm[j]];
#pragma unroll
            for (int q = 0; q < RT; ++q) acc[q][j] = floatx4{bv, bv, bv, bv};
        }
        auto ldm = [&](int kb, floatx4 (&v)[NTM]) {
            const int k = (kb < a.H2 ? kb : a.H2 - 16) + 4 * g;
#pragma unroll
            for (int j = 0; j < NTM; ++j) v[j] = *reinterpret_cast<const floatx4_a4 *>(a.Wm + (int64_t)rowm[j] * a.H2 + k);
        };
        ldm(0, ma);
        ldm(16, mb);
        for (int kb = 0; kb < a.H2; kb += 32) {
            floatx4 f0[RT], f1[RT];
#pragma unroll
            for (int q = 0; q < RT; ++q) {
                f0[q] = *reinterpret_cast<const floatx4 *>(&hs2[16 * q + c][kb + 4 * g]);
                f1[q] = *reinterpret_cast<const floatx4 *>(&hs2[16 * q + c][kb + 16 + 4 * g]);
            }
#pragma unroll
            for (int q = 0; q < RT; ++q) chain_block<NTM>(f0[q], ma, acc[q]);
            __builtin_amdgcn_sched_barrier(0);
            ldm(kb + 32, ma);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < RT; ++q) chain_block<NTM>(f1[q], mb, acc[q]);
            __builtin_amdgcn_sched_barrier(0);
            ldm(kb + 48, mb);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < NTM; ++j) {
            const int n = 16 * (w + kChWaves * j) + c;
            if (n >= a.Hm) continue;
#pragma unroll
            for (int q = 0; q < RT; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rr = 16 * q + 4 * g + i;
                    const float v = chain_act(acc[q][j][i], a.hact);
                    hs1[rr][n] = v;
                    if (a.hm && r0 + rr < a.B) a.hm[(int64_t)(r0 + rr) * a.Hm + n] = v;
                }
        }
        __syncthreads();
    }
    // the head: wave w, rows RPW w .. (over hs2, or hs1 after the fourth layer)
    const int KL = NTM > 0 ? a.Hm : a.H2;
    float (*hl)[LD] = NTM > 0 ? hs1 : hs2;
    for (int o = 0; o < a.NO; ++o) {
        const float *w3 = o < a.split3 ? a.W3 + (int64_t)o * KL : a.W3b + (int64_t)(o - a.split3) * KL;
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int rr = RPW * w + i;
            float z = 0.f;
            for (int k = lane; k < KL; k += 64) z = __builtin_fmaf(hl[rr][k], w3[k], z);
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) z += __shfl_xor(z, m);
            const int r = r0 + rr;
            if (lane == 0 && r < a.B) {
                if (a.b3) z = z + a.b3[o];
                if (a.head == 2) {
                    z = tanhf(z);
                } else if (a.head) {
                    const float th = tanhf(z);
                    a.aux[(int64_t)r * a.NO + o] = th;
                    z = a.gain[o] * th + a.off[o];
                }
                a.y[(int64_t)r * a.NO + o] = z;
            }
        }
    }
}

// The backward data pass of the same chains: dH2 = (dY W3) act'(h2) and dH1 = (dH2 W2) act'(h1)
// (with a fourth layer dHm = (dY W3) act'(hm) first, then dH2 = (dHm Wm) act'(h2)) stay in LDS
// and, when asked (d2 / d1 / dm), go to HBM as the weight gradients' dY operands; dX[:, c0:c0+nc]
// = dH1 W1[:, c0:c0+nc] with the tanh-affine backward of the actor's head when t is given (the
// critic's input gradient of DDPG / SAC's actor pass). One launch instead of one or two GEMMs per
// layer. Layer 2: as chain3_fwd_kernel's (NT tiles of dH1 per wave, H2 a multiple of 32,
// the next block's weights in flight), with B(k, n) = W2[k][n] (four 64-byte row segments per lane
// instead of one 16-byte column read); the dX columns: the lane-split dot products of
// chain3_fwd_kernel's layer 3.
struct ChainBwdArgs {
    const float *dy, *W1, *W2, *W3;  // dY [B][NO]; the layers' weights ([out][in])
    const float *h1, *h2;            // relu outputs [B][H1], [B][H2] (the masks)
    int K0, H1, H2, NO, B, c0, nc;
    const float *t, *gain;           // t: tanh(z) of the actor's head [B][nc] (or null), gain [nc]
    float *dx;                       // [B][nc] (nc = 0: none)
    float *d2, *d1;                  // dH2 [B][H2], dH1 [B][H1] to HBM when set (the weight
                                     // gradients' dY operands)
    const float *W3b;                // rows [split3, NO) of W3 from W3b (the SAC actor's heads)
    int split3;
    int hact;                        // hidden activation: 0 relu, 1 tanh (the PPO2 nets)
    const float *Wm, *hm;            // optional fourth layer (H2 -> Hm, Hm a multiple of 32, W3 then
    int Hm;                          // [NO][Hm]): its weights [Hm][H2], its outputs [B][Hm], and
    float *dm;                       // dHm [B][Hm] to HBM when set
};

template <int NT, int NTB>
__global__ void __launch_bounds__(kChThreads) chain3_bwd_kernel(ChainBwdArgs a0, ChainBwdArgs a1) {
    const ChainBwdArgs &a = blockIdx.y ? a1 : a0;
    __shared__ __attribute__((aligned(16))) float gs2[kChRows][kChLd];
    __shared__ __attribute__((aligned(16))) float gs1[kChRows][kChLd];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, g = lane >> 4, c = lane & 15;
    const int r0 = blockIdx.x * kChRows;
    // the derivative of the hidden activation from its output h: relu (h > 0) or tanh (1 - h^2,
    // the GEMM path's kEpiTanhAffBack with gain 1)
    auto dact = [&](float v, float h) { return a.hact ? (v * 1.f) * (1.f - h * h) : (h > 0.f ? v : 0.f); };
    int col[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int n = 16 * (w + kChWaves * j) + c;
        col[j] = n < a.H1 ? n : a.H1 - 1;
    }
    auto ld = [&](int kb, floatx4 (&v)[NT]) {  // kb past H2: a clamped reload, unused
        const int k = (kb < a.H2 ? kb : a.H2 - 16) + 4 * g;
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int u = 0; u < 4; ++u) v[j][u] = a.W2[(int64_t)(k + u) * a.H1 + col[j]];
    };
    floatx4 ba[NT], bb[NT];  // the first weight fragments in flight under the dH2 fill
    ld(0, ba);
    ld(16, bb);
    // the first gradient: dY W3 through the top hidden layer (an outer product for NO = 1: the GEMM
    // path's single product per element) — dH2, or with the fourth layer dHm (into gs1, free until
    // the dH1 stage)
    const int KT = NTB > 0 ? a.Hm : a.H2;
    const float *htop = NTB > 0 ? a.hm : a.h2;
    float *dtop = NTB > 0 ? a.dm : a.d2;
    float (*gtop)[kChLd] = NTB > 0 ? gs1 : gs2;
    for (int i = t; i < kChRows * KT; i += kChThreads) {
        const int rr = i / KT, o = i % KT, r = r0 + rr;
        float v = 0.f;
        if (r < a.B) {
            v = a.dy[(int64_t)r * a.NO] * a.W3[o];
            for (int j = 1; j < a.NO; ++j) {
                const float *w3 = j < a.split3 ? a.W3 + (int64_t)j * KT : a.W3b + (int64_t)(j - a.split3) * KT;
                v = __builtin_fmaf(a.dy[(int64_t)r * a.NO + j], w3[o], v);
            }
            v = dact(v, htop[(int64_t)r * KT + o]);
        }
        gtop[rr][o] = v;
        if (dtop && r < a.B) dtop[(int64_t)r * KT + o] = v;
    }
    __syncthreads();
    if constexpr (NTB > 0) {  // dH2 = (dHm Wm) act'(h2): gs1 -> gs2 (Hm a multiple of 32)
        int colb[NTB];
        floatx4 acc[NTB], ma[NTB], mb[NTB];
#pragma unroll
        for (int j = 0; j < NTB; ++j) {
            const int n = 16 * (w + kChWaves * j) + c;
            colb[j] = n < a.H2 ? n : a.H2 - 1;
            acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        auto ldm = [&](int kb, floatx4 (&v)[NTB]) {
            const int k = (kb < a.Hm ? kb : a.Hm - 16) + 4 * g;
#pragma unroll
            for (int j = 0; j < NTB; ++j)
#pragma unroll
                for (int u = 0; u < 4; ++u) v[j][u] = a.Wm[(int64_t)(k + u) * a.H2 + colb[j]];
        };
        ldm(0, ma);
        ldm(16, mb);
        for (int kb = 0; kb < a.Hm; kb += 32) {
            const floatx4 f0 = *reinterpret_cast<const floatx4 *>(&gs1[c][kb + 4 * g]);
            const floatx4 f1 = *reinterpret_cast<const floatx4 *>(&gs1[c][kb + 16 + 4 * g]);
            chain_block<NTB>(f0, ma, acc);
            __builtin_amdgcn_sched_barrier(0);
            ldm(kb + 32, ma);
            __builtin_amdgcn_sched_barrier(0);
            chain_block<NTB>(f1, mb, acc);
            __builtin_amdgcn_sched_barrier(0);
            ldm(kb + 48, mb);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < NTB; ++j) {
            const int n = 16 * (w + kChWaves * j) + c;
            if (n >= a.H2) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = r0 + 4 * g + i;
                const float v = r < a.B ? dact(acc[j][i], a.h2[(int64_t)r * a.H2 + n]) : 0.f;
                gs2[4 * g + i][n] = v;
                if (a.d2 && r < a.B) a.d2[(int64_t)r * a.H2 + n] = v;
            }
        }
        __syncthreads();
    }
    {
        floatx4 acc[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int kb = 0; kb < a.H2; kb += 32) {  // (sched barriers: the scheduler sinks the loads)
            const floatx4 f0 = *reinterpret_cast<const floatx4 *>(&gs2[c][kb + 4 * g]);
            const floatx4 f1 = *reinterpret_cast<const floatx4 *>(&gs2[c][kb + 16 + 4 * g]);
            chain_block<NT>(f0, ba, acc);
            __builtin_amdgcn_sched_barrier(0);
            ld(kb + 32, ba);
            __builtin_amdgcn_sched_barrier(0);
            chain_block<NT>(f1, bb, acc);
            __builtin_amdgcn_sched_barrier(0);
            ld(kb + 48, bb);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = 16 * (w + kChWaves * j) + c;
            if (n >= a.H1) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = r0 + 4 * g + i;
                const float v = r < a.B ? dact(acc[j][i], a.h1[(int64_t)r * a.H1 + n]) : 0.f;
                gs1[4 * g + i][n] = v;
                if (a.d1 && r < a.B) a.d1[(int64_t)r * a.H1 + n] = v;
            }
        }
    }
    __syncthreads();
    // dX columns: wave w, rows kChRpw w ..
    for (int j = 0; j < a.nc; ++j) {
#pragma unroll
        for (int i = 0; i < kChRpw; ++i) {
            const int rr = kChRpw * w + i;
            float z = 0.f;
            for (int k = lane; k < a.H1; k += 64)
                z = __builtin_fmaf(gs1[rr][k], a.W1[(int64_t)k * a.K0 + a.c0 + j], z);
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) z += __shfl_xor(z, m);
            const int r = r0 + rr;
            if (lane == 0 && r < a.B) {
                if (a.t) {  // torch: grad_t = da * gain; grad_z = grad_t * (1 - t*t)
                    const float tt = a.t[(int64_t)r * a.nc + j];
                    z = (z * a.gain[j]) * (1.f - tt * tt);
                }
                a.dx[(int64_t)r * a.nc + j] = z;
            }
        }
    }
}

// launch helpers: the tile counts per wave as template arguments (hidden widths 32 .. 256: one or
// two 16-column tiles per wave)
static_assert(kChMaxNt == 2, "chain launch tables");
using ChainFwdFn = void (*)(ChainArgs, ChainArgs);
inline int chain_nt(int h) { return (h / 16 + kChWaves - 1) / kChWaves; }
constexpr int kChBigRows = 16384;  // rows from which a forward block takes two row tiles
constexpr int kChNarrow = 128;     // widths up to which one 16-column tile per wave covers a layer
template <int RT, int NTM>
constexpr ChainFwdFn chain_fwd_fn(int nt1, int nt2) {
    return nt1 == 1 ? (nt2 == 1 ? chain3_fwd_kernel<1, 1, RT, NTM> : chain3_fwd_kernel<1, 2, RT, NTM>)
                    : (nt2 == 1 ? chain3_fwd_kernel<2, 1, RT, NTM> : chain3_fwd_kernel<2, 2, RT, NTM>);
}
void chain_fwd_launch(const ChainArgs &c0, const ChainArgs &c1, int nchains, hipStream_t s) {
    // two 16-row tiles per block when the rows fill every CU twice over (batched inference, the
    // PPO2 update's chunks: each layer-2 weight fragment then feeds twice the MFMAs, half the
    // weight reads from L2)
    const int rt = c0.B >= kChBigRows ? 2 : 1, n1 = chain_nt(c0.H1), n2 = chain_nt(c0.H2);
    ChainFwdFn f = rt == 1 ? (c0.Hm ? chain_fwd_fn<1, 1>(n1, n2) : chain_fwd_fn<1, 0>(n1, n2))
                           : (c0.Hm ? chain_fwd_fn<2, 1>(n1, n2) : chain_fwd_fn<2, 0>(n1, n2));
    // nets no wider than 128 with at most 8 inputs (the PPO2-SOI demo's) with two row tiles:
    // half-width LDS rows and an 8-column input tile, four blocks per CU instead of two (35
    // instead of 75 KB)
    if (rt == 2 && c0.H1 <= kChNarrow && c0.H2 <= kChNarrow && c0.Hm <= kChNarrow && c0.K0 <= 8)
        f = c0.Hm ? chain3_fwd_kernel<1, 1, 2, 1, kChNarrow + 4, 8> : chain3_fwd_kernel<1, 1, 2, 0, kChNarrow + 4, 8>;
    f<<<dim3((c0.B + kChRows * rt - 1) / (kChRows * rt), nchains), kChThreads, 0, s>>>(c0, c1);
}
using ChainBwdFn = void (*)(ChainBwdArgs, ChainBwdArgs);
void chain_bwd_launch(const ChainBwdArgs &c0, const ChainBwdArgs &c1, int nchains, hipStream_t s) {
    static const ChainBwdFn tab[2][3] = {
        {chain3_bwd_kernel<1, 0>, chain3_bwd_kernel<1, 1>, chain3_bwd_kernel<1, 2>},
        {chain3_bwd_kernel<2, 0>, chain3_bwd_kernel<2, 1>, chain3_bwd_kernel<2, 2>}};
    const ChainBwdFn f = tab[chain_nt(c0.H1) - 1][c0.Hm ? chain_nt(c0.H2) : 0];
    f<<<dim3((c0.B + kChRows - 1) / kChRows, nchains), kChThreads, 0, s>>>(c0, c1);
}

// ---- host side ------------------------------------------------------------------------------

inline Opnd mat(const float *p, int rows, int cols, int ld) {  // row-major rows x cols
    return Opnd{p, p, ld, 1, ld, 1, rows, cols, cols, -1, 0};
}
inline Opnd cat2(const float *p0, int c0, int ld0, const float *p1, int c1, int ld1, int rows) {
    return Opnd{p0, p1, ld0, 1, ld1, 1, rows, c0 + c1, c0, -1, 0};
}
inline Opnd transposed(const float *p, int rows, int cols, int ld) {  // (i, j) = p[j * ld + i]
    return Opnd{p, p, 1, ld, 1, ld, rows, cols, cols, -1, 0};
}

constexpr size_t kDenseLds = 2 * kDT * kDLd * sizeof(float);  // 67 584 B: two blocks per CU

// splits >= ceil(R / 256) slices of the reduction (each <= 256 rows); returns the slice count
// a problem's reduction slicing (splits >= ceil(R / 256) slices, each <= 256 rows) and tiling
inline Prob make_prob(const Opnd &A, const Opnd &B, const Epi &e, int R, int splits) {
    const int need = (R + kDSlice - 1) / kDSlice;
    const int sp = splits > need ? splits : need;
    const int rchunk = ((R + sp - 1) / sp + 15) / 16 * 16;
    const int nz = R > 0 ? (R + rchunk - 1) / rchunk : 1;
    return Prob{A, B, e, R, rchunk, (e.N + kDT - 1) / kDT, (e.M + kDT - 1) / kDT, nz};
}

// The kernel's dynamic LDS (67.6 KB) is above the 64 KiB default: the attribute is set once per
// process (std::call_once: thread-safe), and a failure is reported at every launch.
static_assert(sizeof(ProbSet) <= 4096 - 256, "ProbSet kernarg within the 4 KiB kernarg segment");
static hipError_t dense_gemm_attr() {
    static std::once_flag once;
    static hipError_t rc = hipSuccess;
    std::call_once(once, [] {
        rc = hipFuncSetAttribute((const void *)dense_gemm_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDenseLds);
    });
    return rc;
}

// problems qs[0 .. n) in one launch (0 < n <= kMaxProbs). A refusal (nothing launched) returns
// RLP_EINVAL and is also left pending (fail_pending), so the entry point's RLP_CHECK_LAUNCH returns
// it through the C-ABI even where the caller's call chain drops this return value.
int gemm_multi(const Prob *qs, int n, hipStream_t s) {
    if (n < 1 || n > kMaxProbs)
        return fail_pending(RLP_EINVAL, "dense GEMM: %d problems (1..%d)", n, kMaxProbs);
    if (dense_gemm_attr() != hipSuccess)
        return fail_pending(RLP_EINVAL, "dense GEMM: dynamic LDS attribute (%d B) not set", (int)kDenseLds);
    ProbSet ps{};
    int nb = 0;
    for (int i = 0; i < n; ++i) {
        ps.p[i] = qs[i];
        ps.start[i] = nb;
        nb += qs[i].nx * qs[i].ny * qs[i].nz;
    }
    ps.start[n] = nb;
    ps.n = n;
    dense_gemm_kernel<<<nb, 256, kDenseLds, s>>>(ps);
    return RLP_OK;
}
// one problem, or two (q1 != nullptr) in one launch; returns p0's slice count (a refused launch is
// pending, see gemm_multi)
int gemm_launch(const Prob &q0, const Prob *q1, hipStream_t s) {
    const Prob qs[2] = {q0, q1 ? *q1 : q0};
    gemm_multi(qs, q1 ? 2 : 1, s);
    return q0.nz;
}

// test hook (include/rlp.h rlp_selftest_gemm_guard): a refused gemm_multi inside a call chain that
// drops its return value must still reach the caller as a non-OK status
int selftest_gemm_guard(int nprobs) {
    take_pending();
    if (nprobs >= 1 && nprobs <= kMaxProbs)
        return fail(RLP_EINVAL, "rlp_selftest_gemm_guard: only out-of-range counts (not %d)", nprobs);
    Prob qs[kMaxProbs + 1] = {};
    gemm_multi(qs, nprobs, nullptr);  // return value dropped, as chain_grad & co. do
    RLP_CHECK_LAUNCH("rlp_selftest_gemm_guard");
    return RLP_OK;
}
int gemm_impl(const Opnd &A, const Opnd &B, const Epi &e, const Opnd *A1, const Opnd *B1,
              const Epi *e1, int M, int N, int R, int splits, hipStream_t s) {
    const Prob q0 = make_prob(A, B, e, R, splits);
    if (!A1) return gemm_launch(q0, nullptr, s);
    const Prob q1 = make_prob(*A1, *B1, *e1, R, splits);
    return gemm_launch(q0, &q1, s);
}
int gemm(const Opnd &A, const Opnd &B, int M, int N, int R, int splits, const Epi &e, hipStream_t s) {
    return gemm_impl(A, B, e, nullptr, nullptr, nullptr, M, N, R, splits, s);
}

struct Layer {
    const float *W, *b;
    int in, out;
};
inline Layer layer_of(const rlp_dense_net &n, const float *params, int l) {
    const float *W = params + n.offset[l];
    return Layer{W, W + (int64_t)n.dims[l] * n.dims[l + 1], n.dims[l], n.dims[l + 1]};
}

// y = act(x W^T + b); x is [B][in] (or the concatenation of two row-major sources)
void dense_fwd(const Opnd &x, const Layer &L, int B, int act, float *y, const float *gain,
               const float *off, float *aux, hipStream_t s) {
    Epi e{};
    e.y = y; e.ldy = L.out; e.bias = L.b; e.kind = act; e.M = B; e.N = L.out;
    e.gain = gain; e.off = off; e.aux = aux; e.ldaux = L.out;
    // B(r, n) = W[n][r]: column stride in, row stride 1
    gemm(x, Opnd{L.W, L.W, 1, L.in, 1, L.in, L.in, L.out, L.out, -1, 0}, B, L.out, L.in, 1, e, s);
}

// dX[:, c0:c0+nc] = (dY W[:, c0:c0+nc]) with the epilogue (relu' mask or tanh-affine backward)
Prob bwd_data_prob(const float *dy, const Layer &L, int B, int c0, int nc, int kind, const float *mask,
                   int64_t ldm, const float *gain, float *dx) {
    Epi e{};
    e.y = dx; e.ldy = nc; e.kind = kind; e.M = B; e.N = nc; e.mask = mask; e.ldm = ldm; e.gain = gain;
    return make_prob(mat(dy, B, L.out, L.out), mat(L.W + c0, L.out, nc, L.in), e, L.out, 1);
}

void dense_bwd_data(const float *dy, const Layer &L, int B, int c0, int nc, int kind,
                    const float *mask, int64_t ldm, const float *gain, float *dx, hipStream_t s) {
    const Prob q = bwd_data_prob(dy, L, B, c0, nc, kind, mask, ldm, gain, dx);
    gemm_launch(q, nullptr, s);
}

// gW = dY^T X, gb = column sums of dY: split over the batch, partials reduced in fixed order
Prob wgrad_prob(const float *dy, const Opnd &x, const Layer &L, int B, float *part, int splits,
                int64_t ldy) {
    Epi e{};
    e.y = part; e.kind = kEpiPartial; e.M = L.out; e.N = L.in + 1;
    Opnd xo = x;
    xo.cols = L.in + 1;
    xo.ones = L.in;
    return make_prob(transposed(dy, L.out, B, (int)(ldy < 0 ? L.out : ldy)), xo, e, B, splits);
}
void wgrad_reduce(const Layer &L, const float *part, int z, float *gW, float *gb, hipStream_t s) {
    const int tot = L.out * (L.in + 1);
    wgrad_reduce_kernel<<<(tot + 63) / 64, 64 * kWrSlices, 0, s>>>(part, z, L.out, L.in + 1, gW, gb, part, gW, gb);
}

// record a layer's partials (its own region) in np for adam_reduce_kernel
bool parts_add(NetParts *np, const float *part, int z, int in, int out, int64_t woff) {
    if (np->n >= kMaxParts) return false;
    np->part[np->n] = part;
    np->z[np->n] = z;
    np->in[np->n] = in;
    np->out[np->n] = out;
    np->off[np->n] = woff;
    ++np->n;
    return true;
}

// the layer's partials reduced into gW / gb now, or (np) left for adam_reduce_kernel (part must
// then be the layer's own region)
void wgrad_finish(const Layer &L, const float *part, int z, float *gW, float *gb, NetParts *np,
                  int64_t woff, hipStream_t s) {
    if (!np || !parts_add(np, part, z, L.in, L.out, woff)) wgrad_reduce(L, part, z, gW, gb, s);
}

void dense_wgrad(const float *dy, const Opnd &x, const Layer &L, int B, float *part, int splits,
                 float *gW, float *gb, hipStream_t s, int64_t ldy = -1, NetParts *np = nullptr,
                 int64_t woff = 0) {
    const Prob q = wgrad_prob(dy, x, L, B, part, splits, ldy);
    wgrad_finish(L, part, gemm_launch(q, nullptr, s), gW, gb, np, woff, s);
}

// a layer's weight gradient and its backward data pass (both read only dY) in one launch
void dense_wgrad_bwd(const float *dy, const Opnd &x, const Layer &L, int B, float *part, int splits,
                     float *gW, float *gb, int c0, int nc, int kind, const float *mask, int64_t ldm,
                     const float *gain, float *dx, hipStream_t s, NetParts *np = nullptr,
                     int64_t woff = 0) {
    const Prob qw = wgrad_prob(dy, x, L, B, part, splits, -1);
    const Prob qb = bwd_data_prob(dy, L, B, c0, nc, kind, mask, ldm, gain, dx);
    wgrad_finish(L, part, gemm_launch(qw, &qb, s), gW, gb, np, woff, s);
}

void adam_dev(float *p, const float *g, float *m, float *v, int64_t n, const rlp_adam_cfg &c,
              const int32_t *step, hipStream_t s) {
    const int64_t b = (n + 255) / 256;
    adam_dev_kernel<<<(int)(b < 2048 ? b : 2048), 256, 0, s>>>(p, g, m, v, n, c.lr, c.beta1, c.beta2,
                                                              c.eps, step);
}

void adam_reduce(float *p, float *g, float *m, float *v, int64_t n, const NetParts &np,
                 const rlp_adam_cfg &c, const int32_t *step, float *tp, float tau, hipStream_t s) {
    const int64_t b = (n + 255) / 256;
    adam_reduce_kernel<<<(int)(b < 2048 ? b : 2048), 256, 0, s>>>(
        p, g, m, v, n, np, c.lr, c.beta1, c.beta2, c.eps, step, tp, (float)(1.0 - (double)tau), tau);
}

bool net_ok(const rlp_dense_net &n) {
    if (n.n_layers < 1 || n.n_layers > RLP_DENSE_MAX_LAYERS || !n.params) return false;
    for (int l = 0; l <= n.n_layers; ++l)
        if (n.dims[l] < 1 || n.dims[l] > 4096) return false;
    for (int l = 0; l < n.n_layers; ++l) {
        const int64_t sz = (int64_t)n.dims[l] * n.dims[l + 1] + n.dims[l + 1];
        if (n.offset[l] < 0 || n.offset[l] + sz > n.n_params) return false;
    }
    return true;
}
bool same_shape(const rlp_dense_net &a, const rlp_dense_net &b) {
    if (a.n_layers != b.n_layers || a.n_params != b.n_params) return false;
    for (int l = 0; l <= a.n_layers; ++l)
        if (a.dims[l] != b.dims[l]) return false;
    for (int l = 0; l < a.n_layers; ++l)
        if (a.offset[l] != b.offset[l]) return false;
    return true;
}

int max_width(const rlp_dense_net &n) {
    int w = 0;
    for (int l = 0; l <= n.n_layers; ++l) w = w > n.dims[l] ? w : n.dims[l];
    return w;
}
int64_t hidden_sum(const rlp_dense_net &n) {
    int64_t s = 0;
    for (int l = 1; l <= n.n_layers; ++l) s += n.dims[l];
    return s;
}
constexpr int kWgradRows = 256;  // batch rows per weight-gradient split

struct DdpgWs {  // float offsets into the workspace
    int64_t ta, tc, c, pa, pc, ta_t, pa_t, g0, g1, g2, dq, part, total;
};
DdpgWs ddpg_ws(const rlp_ddpg_nets &n, int B) {
    DdpgWs w{};
    int64_t o = 0;
    auto take = [&](int64_t k) { int64_t r = o; o += (k + 63) / 64 * 64; return r; };
    w.ta = take(B * hidden_sum(n.actor));
    w.ta_t = take((int64_t)B * n.actor.dims[n.actor.n_layers]);
    w.tc = take(B * hidden_sum(n.critic));
    w.c = take(B * hidden_sum(n.critic));
    w.pa = take(B * hidden_sum(n.actor));
    w.pa_t = take((int64_t)B * n.actor.dims[n.actor.n_layers]);
    w.pc = take(B * hidden_sum(n.critic));
    const int mw = max_width(n.actor) > max_width(n.critic) ? max_width(n.actor) : max_width(n.critic);
    w.g0 = take((int64_t)B * mw);
    w.g1 = take((int64_t)B * mw);
    w.g2 = take((int64_t)B * mw);
    w.dq = take((int64_t)B * n.actor.dims[n.actor.n_layers]);
    const int splits = (B + kWgradRows - 1) / kWgradRows;
    // every layer's weight-gradient partials at once (left for adam_reduce_kernel)
    auto parts = [](const rlp_dense_net &d) {
        int64_t t = 0;
        for (int l = 0; l < d.n_layers; ++l) t += (int64_t)d.dims[l + 1] * (d.dims[l] + 1);
        return t;
    };
    const int64_t pa = parts(n.actor), pc = parts(n.critic);
    w.part = take((int64_t)splits * (pa > pc ? pa : pc));
    w.total = o;
    return w;
}

// forward of a whole net: layer l's output at act + off_l (row-major [B][dims[l+1]]); the first
// layer reads x (a strided / concatenated view)
// the fused chain takes the net: three layers, relu hidden widths multiples of 32 up to 256, at
// most 64 inputs (a plain or column-concatenated row-major view) and 4 outputs
bool chain3_ok(const rlp_dense_net &n, const Opnd &x) {
    return n.n_layers == 3 && n.dims[0] <= kChK0 && n.dims[1] <= kChH && n.dims[1] % 32 == 0 &&
           n.dims[2] <= kChH && n.dims[2] % 32 == 0 && n.dims[3] <= 4 && x.cs0 == 1 && x.cs1 == 1 &&
           !x.split_rows && x.ones < 0 && x.cols == n.dims[0];
}
ChainArgs chain3_args(const rlp_dense_net &n, const float *params, const Opnd &x, int B, float *act,
                      bool actor_head, const float *gain, const float *off, float *tanh_out) {
    ChainArgs c{};
    c.x0 = x.p0; c.x1 = x.p1; c.ld0 = x.rs0; c.ld1 = x.rs1; c.split = x.split; c.K0 = n.dims[0];
    const Layer L1 = layer_of(n, params, 0), L2 = layer_of(n, params, 1), L3 = layer_of(n, params, 2);
    c.W1 = L1.W; c.b1 = L1.b; c.W2 = L2.W; c.b2 = L2.b; c.W3 = L3.W; c.b3 = L3.b; c.W3b = L3.W;
    c.H1 = n.dims[1]; c.H2 = n.dims[2]; c.NO = n.dims[3]; c.split3 = c.NO; c.B = B;
    c.h1 = act; c.h2 = act + (int64_t)B * c.H1; c.y = c.h2 + (int64_t)B * c.H2;
    c.head = actor_head ? 1 : 0; c.gain = gain; c.off = off; c.aux = tanh_out;
    return c;
}
// the data-only backward chain: three layers, relu hidden widths multiples of 32 up to 256
bool chain3_bwd_ok(const rlp_dense_net &n) {
    return n.n_layers == 3 && n.dims[1] <= kChH && n.dims[1] % 32 == 0 && n.dims[2] <= kChH &&
           n.dims[2] % 32 == 0 && n.dims[3] <= 4;
}
ChainBwdArgs chain3_bwd_args(const rlp_dense_net &n, const float *params, const float *act, int B,
                             const float *dy, int c0, int nc, const float *t_in, const float *gain,
                             float *dx, float *d2 = nullptr, float *d1 = nullptr) {
    ChainBwdArgs c{};
    c.dy = dy;
    c.W1 = layer_of(n, params, 0).W; c.W2 = layer_of(n, params, 1).W; c.W3 = layer_of(n, params, 2).W;
    c.K0 = n.dims[0]; c.H1 = n.dims[1]; c.H2 = n.dims[2]; c.NO = n.dims[3]; c.B = B;
    c.h1 = act; c.h2 = act + (int64_t)B * c.H1;
    c.c0 = c0; c.nc = nc; c.t = t_in; c.gain = gain; c.dx = dx; c.d2 = d2; c.d1 = d1;
    c.W3b = c.W3; c.split3 = c.NO;
    return c;
}

void net_fwd(const rlp_dense_net &n, const float *params, const Opnd &x, int B, float *act,
             bool actor_head, const float *gain, const float *off, float *tanh_out, hipStream_t s) {
    if (chain3_ok(n, x)) {  // one launch for the three layers
        const ChainArgs c = chain3_args(n, params, x, B, act, actor_head, gain, off, tanh_out);
        chain_fwd_launch(c, c, 1, s);
        return;
    }
    int64_t o = 0;
    Opnd in = x;
    for (int l = 0; l < n.n_layers; ++l) {
        const Layer L = layer_of(n, params, l);
        const bool last = l == n.n_layers - 1;
        const int kind = !last ? kEpiRelu : actor_head ? kEpiTanhAff : kEpiNone;
        dense_fwd(in, L, B, kind, act + o, gain, off, tanh_out, s);
        in = mat(act + o, B, L.out, L.out);
        o += (int64_t)B * L.out;
    }
}
const float *layer_out(const rlp_dense_net &n, const float *act, int B, int l) {
    int64_t o = 0;
    for (int k = 0; k < l; ++k) o += (int64_t)B * n.dims[k + 1];
    return act + o;
}

// backward of a relu net from dY of its last layer (in g[0]); weight gradients into grad (same
// layout as params) when grad != NULL; optionally the input gradient of columns [c0, c0 + nc)
// with the tanh-affine backward of the layer that produced them (the actor's head) into dx
// (dy_top: dY of the last layer; g0 / g1 ping-pong for the layers below, either may be dy_top)
// (np: every layer's partials in a region of its own, splits x out x (in + 1) floats from part
// upwards, left for adam_reduce_kernel)
void net_bwd(const rlp_dense_net &n, const float *params, float *grad, const Opnd &x, int B,
             const float *act, const float *dy_top, float *g0, float *g1, float *part, int splits,
             int c0, int nc, const float *t_in, const float *gain, float *dx, hipStream_t s,
             NetParts *np = nullptr) {
    if (!grad && dx && chain3_bwd_ok(n)) {  // the input gradient alone: one launch
        const ChainBwdArgs c = chain3_bwd_args(n, params, act, B, dy_top, c0, nc, t_in, gain, dx);
        chain_bwd_launch(c, c, 1, s);
        return;
    }
    const float *dy = dy_top;
    float *dn = dy_top == g0 ? g1 : g0;
    int64_t po = 0;
    for (int l = n.n_layers - 1; l >= 0; --l) {
        const Layer L = layer_of(n, params, l);
        const Opnd xin = l == 0 ? x : mat(layer_out(n, act, B, l - 1), B, L.in, L.in);
        float *gW = grad ? grad + n.offset[l] : nullptr, *gb = grad ? gW + (int64_t)L.in * L.out : nullptr;
        float *pl = part + po;
        if (np) po += (int64_t)splits * L.out * (L.in + 1);
        if (l > 0) {
            const float *h = layer_out(n, act, B, l - 1);
            if (grad)
                dense_wgrad_bwd(dy, xin, L, B, pl, splits, gW, gb, 0, L.in, kEpiReluBack, h, L.in,
                                nullptr, dn, s, np, n.offset[l]);
            else
                dense_bwd_data(dy, L, B, 0, L.in, kEpiReluBack, h, L.in, nullptr, dn, s);
            float *nxt = dn == g0 ? g1 : g0;
            dy = dn;
            dn = nxt;
        } else if (dx) {
            const int kind = t_in ? kEpiTanhAffBack : kEpiNone;
            if (grad)
                dense_wgrad_bwd(dy, xin, L, B, pl, splits, gW, gb, c0, nc, kind, t_in, nc, gain, dx, s,
                                np, n.offset[l]);
            else
                dense_bwd_data(dy, L, B, c0, nc, kind, t_in, nc, gain, dx, s);
        } else if (grad) {
            dense_wgrad(dy, xin, L, B, pl, splits, gW, gb, s, -1, np, n.offset[l]);
        }
    }
}

// ---- twin chains (the SAC critic's Q1 / Q2: same shapes, one parameter buffer) in shared launches
bool same_dims(const rlp_dense_net &a, const rlp_dense_net &b) {
    if (a.n_layers != b.n_layers) return false;
    for (int l = 0; l <= a.n_layers; ++l)
        if (a.dims[l] != b.dims[l]) return false;
    return true;
}

// two same-shaped chains, each with its own parameters and input (p2 / x2 default to p1 / x1)
void twin_fwd(const rlp_dense_net &n1, const rlp_dense_net &n2, const float *params, const Opnd &x,
              int B, float *act1, float *act2, hipStream_t s, const float *params2 = nullptr,
              const Opnd *x2 = nullptr) {
    if (same_dims(n1, n2) && chain3_ok(n1, x) && chain3_ok(n2, x2 ? *x2 : x)) {  // both chains, one launch
        const ChainArgs c1 = chain3_args(n1, params, x, B, act1, false, nullptr, nullptr, nullptr);
        const ChainArgs c2 = chain3_args(n2, params2 ? params2 : params, x2 ? *x2 : x, B, act2, false,
                                         nullptr, nullptr, nullptr);
        chain_fwd_launch(c1, c2, 2, s);
        return;
    }
    int64_t o = 0;
    Opnd in1 = x, in2 = x2 ? *x2 : x;
    for (int l = 0; l < n1.n_layers; ++l) {
        const Layer L1 = layer_of(n1, params, l), L2 = layer_of(n2, params2 ? params2 : params, l);
        const int kind = l == n1.n_layers - 1 ? kEpiNone : kEpiRelu;
        Epi e1{}, e2{};
        e1.y = act1 + o; e1.ldy = L1.out; e1.bias = L1.b; e1.kind = kind; e1.M = B; e1.N = L1.out;
        e2 = e1;
        e2.y = act2 + o; e2.bias = L2.b;
        const Opnd W1{L1.W, L1.W, 1, L1.in, 1, L1.in, L1.in, L1.out, L1.out, -1, 0};
        const Opnd W2{L2.W, L2.W, 1, L2.in, 1, L2.in, L2.in, L2.out, L2.out, -1, 0};
        gemm_impl(in1, W1, e1, &in2, &W2, &e2, B, L1.out, L1.in, 1, s);
        in1 = mat(act1 + o, B, L1.out, L1.out);
        in2 = mat(act2 + o, B, L2.out, L2.out);
        o += (int64_t)B * L1.out;
    }
}

// backward of both chains from their last layers' dY (dy1 / dy2): weight gradients into grad
// (when non-null; part1 / part2 the two problems' partials), input gradients of columns
// [c0, c0 + nc) into dx1 / dx2 (when non-null). d[0..3]: ping-pong buffers (two per chain).
// (np: each layer's two partial sets in regions of their own from part1 upwards — part2 unused —
// left for adam_reduce_kernel)
void twin_bwd(const rlp_dense_net &n1, const rlp_dense_net &n2, const float *params, float *grad,
              const Opnd &x, int B, const float *act1, const float *act2, const float *dy1,
              const float *dy2, float *const d[4], float *part1, float *part2, int splits, int c0,
              int nc, float *dx1, float *dx2, hipStream_t s, NetParts *np = nullptr) {
    if (!grad && dx1 && dx2 && same_dims(n1, n2) && chain3_bwd_ok(n1)) {  // both chains, one launch
        const ChainBwdArgs c1 = chain3_bwd_args(n1, params, act1, B, dy1, c0, nc, nullptr, nullptr, dx1);
        const ChainBwdArgs c2 = chain3_bwd_args(n2, params, act2, B, dy2, c0, nc, nullptr, nullptr, dx2);
        chain_bwd_launch(c1, c2, 2, s);
        return;
    }
    const float *y1 = dy1, *y2 = dy2;
    int pp = 0;
    int64_t po = 0;
    for (int l = n1.n_layers - 1; l >= 0; --l) {
        const Layer L1 = layer_of(n1, params, l), L2 = layer_of(n2, params, l);
        const Opnd x1 = l == 0 ? x : mat(layer_out(n1, act1, B, l - 1), B, L1.in, L1.in);
        const Opnd x2 = l == 0 ? x : mat(layer_out(n2, act2, B, l - 1), B, L2.in, L2.in);
        if (grad) {
            const bool keep = np && np->n + 2 <= kMaxParts;
            const int64_t region = (int64_t)splits * L1.out * (L1.in + 1);
            float *p1 = keep ? part1 + po : part1, *p2 = keep ? part1 + po + region : part2;
            if (keep) po += 2 * region;
            Epi e1{}, e2{};
            e1.y = p1; e1.kind = kEpiPartial; e1.M = L1.out; e1.N = L1.in + 1;
            e2 = e1;
            e2.y = p2;
            Opnd xo1 = x1, xo2 = x2;
            xo1.cols = xo2.cols = L1.in + 1;
            xo1.ones = xo2.ones = L1.in;
            const Opnd t1 = transposed(y1, L1.out, B, L1.out), t2 = transposed(y2, L2.out, B, L2.out);
            const int z = gemm_impl(t1, xo1, e1, &t2, &xo2, &e2, L1.out, L1.in + 1, B, splits, s);
            if (keep) {
                parts_add(np, p1, z, L1.in, L1.out, n1.offset[l]);
                parts_add(np, p2, z, L2.in, L2.out, n2.offset[l]);
            } else {
                const int tot = L1.out * (L1.in + 1);
                wgrad_reduce_kernel<<<dim3((tot + 63) / 64, 2), 64 * kWrSlices, 0, s>>>(
                    p1, z, L1.out, L1.in + 1, grad + n1.offset[l], grad + n1.offset[l] + (int64_t)L1.in * L1.out,
                    p2, grad + n2.offset[l], grad + n2.offset[l] + (int64_t)L2.in * L2.out);
            }
        }
        if (l > 0 || dx1) {
            const int cc = l > 0 ? 0 : c0, nn = l > 0 ? L1.in : nc;
            float *o1 = l > 0 ? d[pp] : dx1, *o2 = l > 0 ? d[2 + pp] : dx2;
            Epi e1{}, e2{};
            e1.y = o1; e1.ldy = nn; e1.kind = l > 0 ? kEpiReluBack : kEpiNone; e1.M = B; e1.N = nn;
            e2 = e1;
            e2.y = o2;
            if (l > 0) {
                e1.mask = layer_out(n1, act1, B, l - 1); e1.ldm = L1.in;
                e2.mask = layer_out(n2, act2, B, l - 1); e2.ldm = L2.in;
            }
            const Opnd a1 = mat(y1, B, L1.out, L1.out), a2 = mat(y2, B, L2.out, L2.out);
            const Opnd w1 = mat(L1.W + cc, L1.out, nn, L1.in), w2 = mat(L2.W + cc, L2.out, nn, L2.in);
            gemm_impl(a1, w1, e1, &a2, &w2, &e2, B, nn, L1.out, 1, s);
            if (l > 0) {
                y1 = o1;
                y2 = o2;
                pp ^= 1;
            }
        }
    }
}

// dY -> every layer's weight-gradient partials (left in np for adam_reduce_kernel) of a
// three-layer relu chain: the data chain writes dH2 / dH1 to d2 / d1, then all three dW | db
// products in one launch (instead of three launches that each paired a layer's weight gradient
// with its backward data GEMM). Partial regions in net_bwd's order (the last layer first).
bool chain_grad(const rlp_dense_net &n, const float *params, const Opnd &x, int B, const float *act,
                const float *dy, float *d2, float *d1, float *part, int splits, NetParts *np,
                hipStream_t s) {
    if (!np || !d2 || !d1 || !chain3_bwd_ok(n) || np->n + 3 > kMaxParts) return false;
    const ChainBwdArgs c = chain3_bwd_args(n, params, act, B, dy, 0, 0, nullptr, nullptr, nullptr, d2, d1);
    chain_bwd_launch(c, c, 1, s);
    const float *dys[3] = {dy, d2, d1};  // layers 2, 1, 0
    Prob q[3];
    int64_t po = 0;
    for (int k = 0; k < 3; ++k) {
        const int l = 2 - k;
        const Layer L = layer_of(n, params, l);
        const Opnd xin = l == 0 ? x : mat(layer_out(n, act, B, l - 1), B, L.in, L.in);
        q[k] = wgrad_prob(dys[k], xin, L, B, part + po, splits, -1);
        parts_add(np, part + po, q[k].nz, L.in, L.out, n.offset[l]);
        po += (int64_t)splits * L.out * (L.in + 1);
    }
    gemm_multi(q, 3, s);
    return true;
}

// the same for two same-shaped chains (the SAC critic's Q1 / Q2: one data-chain launch, six
// weight-gradient problems in one launch; regions per layer Q1 then Q2, as twin_bwd's)
bool twin_chain_grad(const rlp_dense_net &n1, const rlp_dense_net &n2, const float *params, const Opnd &x,
                     int B, const float *act1, const float *act2, const float *dy1, const float *dy2,
                     float *const d[4], float *part, int splits, NetParts *np, hipStream_t s) {
    if (!np || !same_dims(n1, n2) || !chain3_bwd_ok(n1) || np->n + 6 > kMaxParts) return false;
    const ChainBwdArgs c1 = chain3_bwd_args(n1, params, act1, B, dy1, 0, 0, nullptr, nullptr, nullptr, d[0], d[1]);
    const ChainBwdArgs c2 = chain3_bwd_args(n2, params, act2, B, dy2, 0, 0, nullptr, nullptr, nullptr, d[2], d[3]);
    chain_bwd_launch(c1, c2, 2, s);
    const float *dys[2][3] = {{dy1, d[0], d[1]}, {dy2, d[2], d[3]}};
    const rlp_dense_net *ns[2] = {&n1, &n2};
    const float *acts[2] = {act1, act2};
    Prob q[6];
    int64_t po = 0;
    for (int k = 0; k < 3; ++k) {
        const int l = 2 - k;
        for (int h = 0; h < 2; ++h) {
            const rlp_dense_net &nn = *ns[h];
            const Layer L = layer_of(nn, params, l);
            const Opnd xin = l == 0 ? x : mat(layer_out(nn, acts[h], B, l - 1), B, L.in, L.in);
            q[2 * k + h] = wgrad_prob(dys[h][k], xin, L, B, part + po, splits, -1);
            parts_add(np, part + po, q[2 * k + h].nz, L.in, L.out, nn.offset[l]);
            po += (int64_t)splits * L.out * (L.in + 1);
        }
    }
    gemm_multi(q, 6, s);
    return true;
}

// three or four layers with one hidden activation (relu: the DDPG / SAC actors' batched
// inference; tanh: the PPO2 demo nets' plain-layout rollout), tanh / none at the output, <= 64
// inputs, the first two hidden widths multiples of 32 up to 256, a third up to 128: one chain launch
bool mlp_chain_ok(const rlp_mlp_desc &d) {
    const int L = d.n_layers;
    bool chain = (L == 3 || L == 4) && d.dims[0] <= kChK0 && d.dims[L] <= 8 &&
                 (d.act[L - 1] == RLP_ACT_NONE || d.act[L - 1] == RLP_ACT_TANH) &&
                 (d.act[0] == RLP_ACT_RELU || d.act[0] == RLP_ACT_TANH) && (L == 3 || d.dims[3] <= 16 * kChWaves);
    for (int l = 1; chain && l <= 2; ++l) chain = d.dims[l] <= kChH && d.dims[l] % 32 == 0;
    for (int l = 1; chain && l < L - 1; ++l) chain = d.act[l] == d.act[0];
    return chain;
}
// floats of dense_mlp_forward's scratch (two hidden activations of the per-layer path; 0 for a chain)
int64_t dense_mlp_scratch_floats(const rlp_mlp_desc &d, int n) {
    if (mlp_chain_ok(d) || d.n_layers < 2) return 0;
    int maxw = 0;
    for (int l = 1; l < d.n_layers; ++l) maxw = d.dims[l] > maxw ? d.dims[l] : maxw;
    return 2 * (int64_t)n * maxw;
}

// rlp_mlp_forward on the tiled GEMM (one launch per layer) for large batches: y = MLP(x) for
// the plain Linear-stack layout (W_l [out][in] then b_l), activations RLP_ACT_*; the hidden
// activations in the caller's scratch (dense_mlp_scratch_floats)
int dense_mlp_forward(const rlp_mlp_desc &d, const float *params, const float *x, float *y, int n,
                      float *scratch, hipStream_t s) {
    take_pending();
    const int L = d.n_layers;
    if (mlp_chain_ok(d)) {
        int64_t off[RLP_MLP_MAX_LAYERS], o = 0;
        for (int l = 0; l < L; ++l) {
            off[l] = o;
            o += (int64_t)d.dims[l] * d.dims[l + 1] + d.dims[l + 1];
        }
        auto lw = [&](int l) { return params + off[l]; };
        auto lb = [&](int l) { return params + off[l] + (int64_t)d.dims[l] * d.dims[l + 1]; };
        ChainArgs c{};
        c.x0 = c.x1 = x; c.ld0 = c.ld1 = d.dims[0]; c.split = d.dims[0]; c.K0 = d.dims[0];
        c.W1 = lw(0); c.b1 = lb(0); c.W2 = lw(1); c.b2 = lb(1);
        if (L == 4) {
            c.Wm = lw(2); c.bm = lb(2); c.Hm = d.dims[3];
        }
        c.W3 = c.W3b = lw(L - 1); c.b3 = lb(L - 1);
        c.H1 = d.dims[1]; c.H2 = d.dims[2]; c.NO = d.dims[L]; c.split3 = c.NO; c.B = n;
        c.y = y; c.head = d.act[L - 1] == RLP_ACT_TANH ? 2 : 0; c.hact = d.act[0] == RLP_ACT_TANH;
        chain_fwd_launch(c, c, 1, s);
        RLP_CHECK_LAUNCH("rlp_mlp_forward (chain)");
        return RLP_OK;
    }
    int maxw = 0;
    for (int l = 1; l < d.n_layers; ++l) maxw = d.dims[l] > maxw ? d.dims[l] : maxw;
    float *buf = scratch;
    const float *in = x;
    int64_t off = 0;
    for (int l = 0; l < d.n_layers; ++l) {
        const int K = d.dims[l], N = d.dims[l + 1];
        const Layer L{params + off, params + off + (int64_t)K * N, K, N};
        off += (int64_t)K * N + N;
        const int kind = d.act[l] == RLP_ACT_RELU ? kEpiRelu : d.act[l] == RLP_ACT_TANH ? kEpiTanh : kEpiNone;
        float *out = l == d.n_layers - 1 ? y : buf + (size_t)(l & 1) * n * maxw;
        dense_fwd(mat(in, n, K, K), L, n, kind, out, nullptr, nullptr, nullptr, s);
        in = out;
    }
    RLP_CHECK_LAUNCH("rlp_mlp_forward (dense)");
    return RLP_OK;
}

}  // namespace rlp

using namespace rlp;

extern "C" {

int rlp_selftest_gemm_guard(int nprobs) { return selftest_gemm_guard(nprobs); }

int64_t rlp_ddpg_workspace(const rlp_ddpg_nets *nets, int batch) {
    if (!nets || batch < 1 || !net_ok(nets->actor) || !net_ok(nets->critic)) return RLP_EINVAL;
    return ddpg_ws(*nets, batch).total;
}

int rlp_ddpg_update(const rlp_ddpg_nets *nets, const rlp_ddpg_cfg *cfg, const float *s, const float *a,
                    const float *r, const float *s_next, const float *end, float *work,
                    float *losses, rlp_stream_t stream) {
    take_pending();
    RLP_REQUIRE(nets && cfg && s && a && r && s_next && end && work && losses,
                "rlp_ddpg_update: null argument");
    const rlp_ddpg_nets &n = *nets;
    RLP_REQUIRE(net_ok(n.actor) && net_ok(n.critic), "rlp_ddpg_update: bad net description");
    RLP_REQUIRE(same_shape(n.actor, n.target_actor) && same_shape(n.critic, n.target_critic),
                "rlp_ddpg_update: target nets must have their nets' layout");
    RLP_REQUIRE(n.target_actor.params && n.target_critic.params && n.actor_grad && n.actor_m &&
                    n.actor_v && n.critic_grad && n.critic_m && n.critic_v && n.steps && n.gain && n.off,
                "rlp_ddpg_update: null buffer in the net state");
    const int S = n.actor.dims[0], A = n.actor.dims[n.actor.n_layers];
    RLP_REQUIRE(n.critic.dims[0] == S + A && n.critic.dims[n.critic.n_layers] == 1,
                "rlp_ddpg_update: critic must map cat(s, a) (%d inputs) to 1 output, has %d -> %d",
                S + A, n.critic.dims[0], n.critic.dims[n.critic.n_layers]);
    const int B = cfg->batch;
    RLP_REQUIRE(B >= 1, "rlp_ddpg_update: batch=%d", B);
    hipStream_t st = as_stream(stream);
    const DdpgWs w = ddpg_ws(n, B);
    float *ta = work + w.ta, *tc = work + w.tc, *c = work + w.c, *pa = work + w.pa, *pc = work + w.pc;
    float *ta_t = work + w.ta_t, *pa_t = work + w.pa_t, *g0 = work + w.g0, *g1 = work + w.g1;
    float *g2 = work + w.g2, *dq = work + w.dq, *part = work + w.part;
    const int splits = (B + kWgradRows - 1) / kWgradRows;
    const int La = n.actor.n_layers, Lc = n.critic.n_layers;

    // target: Q' = target_critic(s', target_actor(s'))
    net_fwd(n.target_actor, n.target_actor.params, mat(s_next, B, S, S), B, ta, true, n.gain, n.off,
            ta_t, st);
    const float *a_next = layer_out(n.target_actor, ta, B, La - 1);
    // Q'(s', a') of the target critic and Q(s, a) of the critic: same shapes, shared launches
    const Opnd tx = cat2(s_next, S, S, a_next, A, A, B), sa = cat2(s, S, S, a, A, A, B);
    twin_fwd(n.target_critic, n.critic, n.target_critic.params, tx, B, tc, c, st, n.critic.params, &sa);
    ddpg_td_kernel<<<1, 1024, 0, st>>>(r, end, layer_out(n.target_critic, tc, B, Lc - 1),
                                       layer_out(n.critic, c, B, Lc - 1), B, cfg->gamma, g0, losses,
                                       n.steps);
    NetParts cp{};
    if (!chain_grad(n.critic, n.critic.params, sa, B, c, g0, g1, g2, part, splits, &cp, st))
        net_bwd(n.critic, n.critic.params, n.critic_grad, sa, B, c, g0, g0, g1, part, splits, 0, 0,
                nullptr, nullptr, nullptr, st, &cp);
    // critic Adam + its soft target update (DDPG.py:113-115; the target critic is not read again)
    adam_reduce(n.critic.params, n.critic_grad, n.critic_m, n.critic_v, n.critic.n_params, cp,
                cfg->critic_adam, n.steps + 1, n.target_critic.params, cfg->critic_tau, st);
    // actor: a = mu(s), Q(s, a) with the updated critic (no critic gradients), -mean(Q) backward
    net_fwd(n.actor, n.actor.params, mat(s, B, S, S), B, pa, true, n.gain, n.off, pa_t, st);
    const float *a_pi = layer_out(n.actor, pa, B, La - 1);
    const Opnd sp = cat2(s, S, S, a_pi, A, A, B);
    net_fwd(n.critic, n.critic.params, sp, B, pc, false, nullptr, nullptr, nullptr, st);
    ddpg_actor_loss_kernel<<<1, 1024, 0, st>>>(layer_out(n.critic, pc, B, Lc - 1), B, g0, losses);
    net_bwd(n.critic, n.critic.params, nullptr, sp, B, pc, g0, g0, g1, part, splits, S, A, pa_t, n.gain,
            dq, st);
    // dq now holds dL/dz of the actor's head ([B][A]); back through the actor
    const Opnd s_in = mat(s, B, S, S);
    NetParts ap{};
    if (!chain_grad(n.actor, n.actor.params, s_in, B, pa, dq, g0, g1, part, splits, &ap, st)) {
        float *dy = dq, *d0 = g0, *d1 = g1;
        int64_t po = 0;
        for (int l = La - 1; l >= 0; --l) {
            const Layer L = layer_of(n.actor, n.actor.params, l);
            const Opnd xin = l == 0 ? s_in : mat(layer_out(n.actor, pa, B, l - 1), B, L.in, L.in);
            float *gW = n.actor_grad + n.actor.offset[l], *gb = gW + (int64_t)L.in * L.out;
            float *pl = part + po;
            po += (int64_t)splits * L.out * (L.in + 1);
            if (l > 0) {
                dense_wgrad_bwd(dy, xin, L, B, pl, splits, gW, gb, 0, L.in, kEpiReluBack,
                                layer_out(n.actor, pa, B, l - 1), L.in, nullptr, d0, st, &ap,
                                n.actor.offset[l]);
                dy = d0;
                float *tmp = d0; d0 = d1; d1 = tmp;
            } else {
                dense_wgrad(dy, xin, L, B, pl, splits, gW, gb, st, -1, &ap, n.actor.offset[l]);
            }
        }
    }
    // actor Adam + its soft target update (DDPG.py:116-118)
    adam_reduce(n.actor.params, n.actor_grad, n.actor_m, n.actor_v, n.actor.n_params, ap,
                cfg->actor_adam, n.steps, n.target_actor.params, cfg->actor_tau, st);
    RLP_CHECK_LAUNCH("rlp_ddpg_update");
    return RLP_OK;
}

}  // extern "C"

// ---- SAC host side ----------------------------------------------------------------------------
namespace rlp {

struct SacWs {
    int64_t tn_act, tn_z, tn_a, tn_lp, tq1, tq2, ta, tz, ta_a, ta_lp, save, p1, p2, c1, c2, y, g1,
        g2, da1, da2, gz, d0, d1, d2, d3, part, part2, apart, total;
};
int64_t layer_parts(const rlp_dense_net &d) {  // sum over layers of out x (in + 1)
    int64_t t = 0;
    for (int l = 0; l < d.n_layers; ++l) t += (int64_t)d.dims[l + 1] * (d.dims[l] + 1);
    return t;
}
SacWs sac_ws(const rlp_sac_nets &n, int B) {
    SacWs w{};
    int64_t o = 0;
    auto take = [&](int64_t k) { int64_t r = o; o += (k + 63) / 64 * 64; return r; };
    const int A = n.action_dim;
    const int64_t ha = B * hidden_sum(n.actor), hq1 = B * hidden_sum(n.q1), hq2 = B * hidden_sum(n.q2);
    w.tn_act = take(ha); w.tn_z = take((int64_t)B * 2 * A); w.tn_a = take((int64_t)B * A); w.tn_lp = take(B);
    w.tq1 = take(hq1); w.tq2 = take(hq2);
    w.ta = take(ha); w.tz = take((int64_t)B * 2 * A); w.ta_a = take((int64_t)B * A); w.ta_lp = take(B);
    w.save = take((int64_t)6 * B * A);
    w.p1 = take(hq1); w.p2 = take(hq2); w.c1 = take(hq1); w.c2 = take(hq2);
    w.y = take(B); w.g1 = take(B); w.g2 = take(B);
    w.da1 = take((int64_t)B * A); w.da2 = take((int64_t)B * A); w.gz = take((int64_t)B * 2 * A);
    int mw = max_width(n.actor);
    mw = max_width(n.q1) > mw ? max_width(n.q1) : mw;
    mw = max_width(n.q2) > mw ? max_width(n.q2) : mw;
    mw = 2 * A > mw ? 2 * A : mw;
    w.d0 = take((int64_t)B * mw); w.d1 = take((int64_t)B * mw);
    w.d2 = take((int64_t)B * mw); w.d3 = take((int64_t)B * mw);
    const int splits = (B + kWgradRows - 1) / kWgradRows;
    // part: the critic chains' per-layer partial regions (left for adam_reduce_kernel); apart: the
    // actor's (both heads, then the trunk)
    const int64_t pq = layer_parts(n.q1) + layer_parts(n.q2), one = (int64_t)mw * (mw + 1);
    const int H = n.actor.dims[n.actor.n_layers];
    w.part = take((int64_t)splits * (pq > one ? pq : one));
    w.part2 = take((int64_t)splits * one);
    w.apart = take((int64_t)splits * (layer_parts(n.actor) + 2 * (int64_t)A * (H + 1)));
    w.total = o;
    return w;
}

// trunk (relu after every layer) then the head GEMM z = h [Wm; Wl]^T (biases added by the head kernel)
void sac_actor_fwd(const rlp_sac_nets &n, const float *x, int B, float *act, float *z, hipStream_t s) {
    const rlp_dense_net &t = n.actor;
    if (t.n_layers == 2 && t.dims[0] <= kChK0 && t.dims[1] <= kChH && t.dims[1] % 32 == 0 &&
        t.dims[2] <= kChH && t.dims[2] % 32 == 0) {  // trunk + both heads in one launch
        const int A = n.action_dim;
        const Layer L1 = layer_of(t, t.params, 0), L2 = layer_of(t, t.params, 1);
        ChainArgs c{};
        c.x0 = c.x1 = x; c.ld0 = c.ld1 = t.dims[0]; c.split = t.dims[0]; c.K0 = t.dims[0];
        c.W1 = L1.W; c.b1 = L1.b; c.W2 = L2.W; c.b2 = L2.b;
        c.W3 = t.params + n.mean_offset; c.W3b = t.params + n.log_std_offset; c.split3 = A; c.b3 = nullptr;
        c.H1 = t.dims[1]; c.H2 = t.dims[2]; c.NO = 2 * A; c.B = B;
        c.h1 = act; c.h2 = act + (int64_t)B * c.H1; c.y = z;
        chain_fwd_launch(c, c, 1, s);
        return;
    }
    Opnd in = mat(x, B, n.actor.dims[0], n.actor.dims[0]);
    int64_t o = 0;
    for (int l = 0; l < n.actor.n_layers; ++l) {
        const Layer L = layer_of(n.actor, n.actor.params, l);
        dense_fwd(in, L, B, kEpiRelu, act + o, nullptr, nullptr, nullptr, s);
        in = mat(act + o, B, L.out, L.out);
        o += (int64_t)B * L.out;
    }
    const int H = n.actor.dims[n.actor.n_layers], A = n.action_dim;
    Epi e{};
    e.y = z; e.ldy = 2 * A; e.kind = kEpiNone; e.M = B; e.N = 2 * A;
    const float *Wm = n.actor.params + n.mean_offset, *Wl = n.actor.params + n.log_std_offset;
    gemm(in, Opnd{Wm, Wl, 1, H, 1, H, H, 2 * A, A, -1, 0}, B, 2 * A, H, 1, e, s);
}

int sac_head(const rlp_sac_nets &n, const rlp_sac_cfg &c, const float *z, int B, const float *noise,
             uint64_t draw, float *act, float *lp, float *save, hipStream_t s) {
    const float *P = n.actor.params;
    const int H = n.actor.dims[n.actor.n_layers], A = n.action_dim;
    const float *bm = P + n.mean_offset + (int64_t)A * H, *bl = P + n.log_std_offset + (int64_t)A * H;
    const int g = (B + 255) / 256;
#define RLP_SAC_HEAD(AA)                                                                                  \
    if (save)                                                                                             \
        sac_head_kernel<AA, true><<<g, 256, 0, s>>>(z, B, bm, bl, n.ls_lo, n.ls_hi, n.gain, n.off, noise, \
                                                    c.seed, n.counter, draw, act, lp, save);              \
    else                                                                                                  \
        sac_head_kernel<AA, false><<<g, 256, 0, s>>>(z, B, bm, bl, n.ls_lo, n.ls_hi, n.gain, n.off,       \
                                                     noise, c.seed, n.counter, draw, act, lp, nullptr);
    switch (A) {
    case 1: RLP_SAC_HEAD(1) break;
    case 2: RLP_SAC_HEAD(2) break;
    case 3: RLP_SAC_HEAD(3) break;
    case 4: RLP_SAC_HEAD(4) break;
    default: return RLP_EINVAL;
    }
#undef RLP_SAC_HEAD
    return RLP_OK;
}

bool chain_ok(const rlp_dense_net &q, int S, int A) {
    return net_ok(q) && q.dims[0] == S + A && q.dims[q.n_layers] == 1;
}

}  // namespace rlp

extern "C" {

int64_t rlp_sac_workspace(const rlp_sac_nets *nets, int batch) {
    if (!nets || batch < 1 || !net_ok(nets->actor) || !net_ok(nets->q1) || !net_ok(nets->q2) ||
        nets->action_dim < 1 || nets->action_dim > 4)
        return RLP_EINVAL;
    return sac_ws(*nets, batch).total;
}

int rlp_sac_update(const rlp_sac_nets *nets, const rlp_sac_cfg *cfg, const float *s, const float *a,
                   const float *r, const float *s_next, const float *dw, const float *noise,
                   float *work, float *losses, rlp_stream_t stream) {
    take_pending();
    RLP_REQUIRE(nets && cfg && s && a && r && s_next && dw && work && losses,
                "rlp_sac_update: null argument");
    const rlp_sac_nets &n = *nets;
    const int A = n.action_dim, S = n.actor.dims[0], H = n.actor.dims[n.actor.n_layers];
    RLP_REQUIRE(A >= 1 && A <= 4, "rlp_sac_update: action_dim=%d (1..4)", A);
    RLP_REQUIRE(net_ok(n.actor) && chain_ok(n.q1, S, A) && chain_ok(n.q2, S, A) &&
                    n.q1.params == n.q2.params && n.q1.n_params == n.q2.n_params,
                "rlp_sac_update: bad net description (two critic chains cat(s, a) -> 1 in one buffer)");
    RLP_REQUIRE(n.mean_offset >= 0 && n.log_std_offset >= 0 &&
                    n.mean_offset + (int64_t)A * (H + 1) <= n.actor.n_params &&
                    n.log_std_offset + (int64_t)A * (H + 1) <= n.actor.n_params,
                "rlp_sac_update: head offsets outside the actor's parameters");
    RLP_REQUIRE(n.target_critic && n.actor_grad && n.actor_m && n.actor_v && n.critic_grad &&
                    n.critic_m && n.critic_v && n.log_alpha && n.alpha_grad && n.alpha_m &&
                    n.alpha_v && n.steps && n.counter && n.gain && n.off && n.ls_lo && n.ls_hi,
                "rlp_sac_update: null buffer in the net state");
    const int B = cfg->batch;
    RLP_REQUIRE(B >= 1, "rlp_sac_update: batch=%d", B);
    hipStream_t st = as_stream(stream);
    const SacWs w = sac_ws(n, B);
    auto W = [&](int64_t off) { return work + off; };
    const int splits = (B + kWgradRows - 1) / kWgradRows;
    const int Lq1 = n.q1.n_layers, Lq2 = n.q2.n_layers;
    const int g = (B + 255) / 256;
    const int ad = cfg->adaptive_alpha;

    // target: a' ~ pi(s'), Q1', Q2' of the target critic, target_Q
    sac_actor_fwd(n, s_next, B, W(w.tn_act), W(w.tn_z), st);
    int rc = sac_head(n, *cfg, W(w.tn_z), B, noise, 0, W(w.tn_a), W(w.tn_lp), nullptr, st);
    if (rc != RLP_OK) return fail(rc, "rlp_sac_update: action_dim %d", A);
    const Opnd tx = cat2(s_next, S, S, W(w.tn_a), A, A, B);
    const bool twin = same_dims(n.q1, n.q2);  // Q1 / Q2 GEMMs share launches
    float *const dd[4] = {W(w.d0), W(w.d1), W(w.d2), W(w.d3)};
    if (twin) {
        twin_fwd(n.q1, n.q2, n.target_critic, tx, B, W(w.tq1), W(w.tq2), st);
    } else {
        net_fwd(n.q1, n.target_critic, tx, B, W(w.tq1), false, nullptr, nullptr, nullptr, st);
        net_fwd(n.q2, n.target_critic, tx, B, W(w.tq2), false, nullptr, nullptr, nullptr, st);
    }
    sac_target_kernel<<<g, 256, 0, st>>>(r, dw, layer_out(n.q1, W(w.tq1), B, Lq1 - 1),
                                         layer_out(n.q2, W(w.tq2), B, Lq2 - 1), W(w.tn_lp), B,
                                         cfg->gamma, n.log_alpha, ad, cfg->alpha, W(w.y));
    // actor: a ~ pi(s), Q1, Q2 of the critic, loss, backward through the critic into a
    sac_actor_fwd(n, s, B, W(w.ta), W(w.tz), st);
    sac_head(n, *cfg, W(w.tz), B, noise ? noise + (size_t)B * A : nullptr, 1, W(w.ta_a), W(w.ta_lp),
             W(w.save), st);
    const Opnd px = cat2(s, S, S, W(w.ta_a), A, A, B);
    if (twin) {
        twin_fwd(n.q1, n.q2, n.q1.params, px, B, W(w.p1), W(w.p2), st);
    } else {
        net_fwd(n.q1, n.q1.params, px, B, W(w.p1), false, nullptr, nullptr, nullptr, st);
        net_fwd(n.q2, n.q2.params, px, B, W(w.p2), false, nullptr, nullptr, nullptr, st);
    }
    sac_actor_loss_kernel<<<1, 1024, 0, st>>>(layer_out(n.q1, W(w.p1), B, Lq1 - 1),
                                              layer_out(n.q2, W(w.p2), B, Lq2 - 1), W(w.ta_lp), B,
                                              n.log_alpha, ad, cfg->alpha, cfg->target_entropy,
                                              W(w.g1), W(w.g2), losses, n.alpha_grad, n.steps,
                                              n.counter);
    if (twin) {
        twin_bwd(n.q1, n.q2, n.q1.params, nullptr, px, B, W(w.p1), W(w.p2), W(w.g1), W(w.g2), dd,
                 W(w.part), W(w.part2), splits, S, A, W(w.da1), W(w.da2), st);
    } else {
        net_bwd(n.q1, n.q1.params, nullptr, px, B, W(w.p1), W(w.g1), W(w.d0), W(w.d1), W(w.part),
                splits, S, A, nullptr, nullptr, W(w.da1), st);
        net_bwd(n.q2, n.q2.params, nullptr, px, B, W(w.p2), W(w.g2), W(w.d0), W(w.d1), W(w.part),
                splits, S, A, nullptr, nullptr, W(w.da2), st);
    }
    switch (A) {
    case 1: sac_head_back_kernel<1><<<g, 256, 0, st>>>(W(w.save), W(w.da1), W(w.da2), B, n.gain, n.log_alpha, ad, cfg->alpha, W(w.gz)); break;
    case 2: sac_head_back_kernel<2><<<g, 256, 0, st>>>(W(w.save), W(w.da1), W(w.da2), B, n.gain, n.log_alpha, ad, cfg->alpha, W(w.gz)); break;
    case 3: sac_head_back_kernel<3><<<g, 256, 0, st>>>(W(w.save), W(w.da1), W(w.da2), B, n.gain, n.log_alpha, ad, cfg->alpha, W(w.gz)); break;
    default: sac_head_back_kernel<4><<<g, 256, 0, st>>>(W(w.save), W(w.da1), W(w.da2), B, n.gain, n.log_alpha, ad, cfg->alpha, W(w.gz)); break;
    }
    // actor backward: heads' weight gradients, then the trunk (partials left for the actor's Adam)
    NetParts ap{};
    {
        const int Lt = n.actor.n_layers;
        float *P = n.actor.params, *G = n.actor_grad;
        const float *h_last = layer_out(n.actor, W(w.ta), B, Lt - 1);
        const Opnd hx = mat(h_last, B, H, H);
        const Layer Lm{P + n.mean_offset, P + n.mean_offset + (int64_t)A * H, H, A};
        const Layer Ll{P + n.log_std_offset, P + n.log_std_offset + (int64_t)A * H, H, A};
        float *apart = W(w.apart);
        const int64_t hreg = (int64_t)splits * A * (H + 1);
        int64_t po = 2 * hreg;
        const rlp_dense_net &t = n.actor;
        if (Lt == 2 && t.dims[1] <= kChH && t.dims[1] % 32 == 0 && t.dims[2] <= kChH &&
            t.dims[2] % 32 == 0 && ap.n + 4 <= kMaxParts) {
            // the heads' and the trunk's backward as one data chain (dh = (gz [Wm; Wl]) relu'(h2),
            // dh1 = (dh W2) relu'(h1)), then the four weight gradients in one launch
            ChainBwdArgs c{};
            c.dy = W(w.gz); c.NO = 2 * A; c.W3 = Lm.W; c.W3b = Ll.W; c.split3 = A;
            c.W1 = layer_of(t, P, 0).W; c.W2 = layer_of(t, P, 1).W;
            c.K0 = t.dims[0]; c.H1 = t.dims[1]; c.H2 = t.dims[2]; c.B = B;
            c.h1 = W(w.ta); c.h2 = h_last; c.d2 = W(w.d0); c.d1 = W(w.d1);
            chain_bwd_launch(c, c, 1, st);
            Prob q[4];
            q[0] = wgrad_prob(W(w.gz), hx, Lm, B, apart, splits, 2 * A);
            q[1] = wgrad_prob(W(w.gz) + A, hx, Ll, B, apart + hreg, splits, 2 * A);
            parts_add(&ap, apart, q[0].nz, H, A, n.mean_offset);
            parts_add(&ap, apart + hreg, q[1].nz, H, A, n.log_std_offset);
            const float *dys[2] = {W(w.d0), W(w.d1)};  // layers 1, 0
            for (int k = 0; k < 2; ++k) {
                const int l = 1 - k;
                const Layer L = layer_of(t, P, l);
                const Opnd xin = l == 0 ? mat(s, B, S, S) : mat(W(w.ta), B, L.in, L.in);
                q[2 + k] = wgrad_prob(dys[k], xin, L, B, apart + po, splits, -1);
                parts_add(&ap, apart + po, q[2 + k].nz, L.in, L.out, t.offset[l]);
                po += (int64_t)splits * L.out * (L.in + 1);
            }
            gemm_multi(q, 4, st);
        } else {
            {  // both heads' weight gradients in one launch, partials left for the actor's Adam
                const Prob qm = wgrad_prob(W(w.gz), hx, Lm, B, apart, splits, 2 * A);
                const Prob ql = wgrad_prob(W(w.gz) + A, hx, Ll, B, apart + hreg, splits, 2 * A);
                const int z = gemm_launch(qm, &ql, st);
                parts_add(&ap, apart, z, H, A, n.mean_offset);
                parts_add(&ap, apart + hreg, z, H, A, n.log_std_offset);
            }
            // dh = (gz [Wm; Wl]) * relu'(h)
            Epi e{};
            e.y = W(w.d0); e.ldy = H; e.kind = kEpiReluBack; e.M = B; e.N = H; e.mask = h_last; e.ldm = H;
            gemm(mat(W(w.gz), B, 2 * A, 2 * A), Opnd{Lm.W, Ll.W, H, 1, H, 1, 2 * A, H, A, -1, 1}, B, H,
                 2 * A, 1, e, st);
            float *dy = W(w.d0), *dn = W(w.d1);
            for (int l = Lt - 1; l >= 0; --l) {
                const Layer L = layer_of(n.actor, P, l);
                const Opnd xin = l == 0 ? mat(s, B, S, S) : mat(layer_out(n.actor, W(w.ta), B, l - 1), B, L.in, L.in);
                float *gW = G + n.actor.offset[l], *gb = gW + (int64_t)L.in * L.out;
                float *pl = apart + po;
                po += (int64_t)splits * L.out * (L.in + 1);
                if (l > 0) {
                    dense_wgrad_bwd(dy, xin, L, B, pl, splits, gW, gb, 0, L.in, kEpiReluBack,
                                    layer_out(n.actor, W(w.ta), B, l - 1), L.in, nullptr, dn, st, &ap,
                                    n.actor.offset[l]);
                    float *tmp = dy; dy = dn; dn = tmp;
                } else {
                    dense_wgrad(dy, xin, L, B, pl, splits, gW, gb, st, -1, &ap, n.actor.offset[l]);
                }
            }
        }
    }
    // critic: Q1, Q2 on the batch's actions, MSE to target_Q, backward into the critic's gradient
    const Opnd bx = cat2(s, S, S, a, A, A, B);
    if (twin) {
        twin_fwd(n.q1, n.q2, n.q1.params, bx, B, W(w.c1), W(w.c2), st);
    } else {
        net_fwd(n.q1, n.q1.params, bx, B, W(w.c1), false, nullptr, nullptr, nullptr, st);
        net_fwd(n.q2, n.q2.params, bx, B, W(w.c2), false, nullptr, nullptr, nullptr, st);
    }
    sac_critic_loss_kernel<<<1, 1024, 0, st>>>(layer_out(n.q1, W(w.c1), B, Lq1 - 1),
                                               layer_out(n.q2, W(w.c2), B, Lq2 - 1), W(w.y), B,
                                               W(w.g1), W(w.g2), losses);
    NetParts cp{};
    if (twin && twin_chain_grad(n.q1, n.q2, n.q1.params, bx, B, W(w.c1), W(w.c2), W(w.g1), W(w.g2), dd,
                                W(w.part), splits, &cp, st)) {
    } else if (twin) {
        twin_bwd(n.q1, n.q2, n.q1.params, n.critic_grad, bx, B, W(w.c1), W(w.c2), W(w.g1), W(w.g2), dd,
                 W(w.part), W(w.part2), splits, 0, 0, nullptr, nullptr, st, &cp);
    } else {
        net_bwd(n.q1, n.q1.params, n.critic_grad, bx, B, W(w.c1), W(w.g1), W(w.d0), W(w.d1),
                W(w.part), splits, 0, 0, nullptr, nullptr, nullptr, st, &cp);
        net_bwd(n.q2, n.q2.params, n.critic_grad, bx, B, W(w.c2), W(w.g2), W(w.d0), W(w.d1),
                W(w.part) + (int64_t)splits * layer_parts(n.q1), splits, 0, 0, nullptr, nullptr,
                nullptr, st, &cp);
    }
    // optimizer steps (actor; critic with the soft target update, :126-127 — tau p + (1 - tau) tp
    // is the same sum as tp (1 - tau) + p tau; temperature), each reducing its weight gradients
    adam_reduce(n.actor.params, n.actor_grad, n.actor_m, n.actor_v, n.actor.n_params, ap,
                cfg->actor_adam, n.steps, nullptr, 0.f, st);
    adam_reduce(n.q1.params, n.critic_grad, n.critic_m, n.critic_v, n.q1.n_params, cp,
                cfg->critic_adam, n.steps + 1, n.target_critic, cfg->tau, st);
    if (ad) adam_dev(n.log_alpha, n.alpha_grad, n.alpha_m, n.alpha_v, 1, cfg->alpha_adam, n.steps + 2, st);
    RLP_CHECK_LAUNCH("rlp_sac_update");
    return RLP_OK;
}

}  // extern "C"

namespace rlp {

// ---- PPO2 update for any tanh Linear stack (Proximal_Policy_Optimization2.learn, algorithm/
// policy_base/Proximal_Policy_Optimization2.py:133-163) on the dense GEMM -------------------------
// The nets rlp_ppo2_grad's f16x3 kernels do not take: the PPO2-SecondOrderIntegration demo's
// actor 4 -> 128 -> 64 -> 32 -> A and critic 4 -> 64 -> 64 -> 1 (demonstration/PPO2/PPO2-4-
// SecondOrderIntegration/train.py:37-125), the obstacle-avoidance demos' 41-input nets
// (demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/train.py:48-50,95-97). Exact f32
// products (v_mfma_f32_16x16x4_f32) throughout, rows in chunks of kPpoChunk:
//   forward   layer by layer, tanh epilogues (the actor's head keeps t = tanh(z) beside
//             mean = gain t + off), activations of the chunk in the workspace
//   head      per row dL/dz_L: the clipped-surrogate actor loss (torch.min / clamp backward
//             semantics, as ppo2_fd_kernel) or the critic's MSE, and the loss sum
//   backward  per layer: dW | db = dY^T [X | 1] over the chunk (long reduction slices, one
//             partial per slice), dX = dY W with the tanh backward (1 - h^2) epilogue
// Every chunk's gradient lands in its own slot; the slots are summed in chunk order (fixed order
// throughout: the same bits on every run and rank).
constexpr int kPpoChunk = 1 << 18;  // (2^20-row chunks: the same SOI / 1.5 % faster UGV-OA iterations, r4n)

inline Prob make_prob_long(const Opnd &A, const Opnd &B, const Epi &e, int R, int nz) {
    if (nz < 1) nz = 1;
    const int rchunk = ((R + nz - 1) / nz + 15) / 16 * 16;
    const int z = R > 0 ? (R + rchunk - 1) / rchunk : 1;
    return Prob{A, B, e, R, rchunk, (e.N + kDT - 1) / kDT, (e.M + kDT - 1) / kDT, z};
}

struct PpoDenseArgs {
    const float *t, *mean, *v;   // actor: tanh(z_L), gain t + off ([B][A]); critic: V ([B])
    const float *a, *lp, *adv, *vt;
    int B, A;
    float inv_rows, eps_clip, ent_row;
    float gain[4], log_std[4], inv_var[4];
    float *dy;                   // [B][A]: dL/dz_L
    double *lpart;               // per-block loss partials (summed in order by loss_sum_kernel)
};

template <bool ACTOR>
__global__ void __launch_bounds__(256) ppo2_dense_head_kernel(PpoDenseArgs h) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    double l = 0.0;
    if (i < h.B) {
        if constexpr (ACTOR) {
            float lp_now = 0.f, lp_old = 0.f, d[4], t[4];
            for (int a = 0; a < h.A; ++a) {
                t[a] = h.t[(size_t)i * h.A + a];
                d[a] = h.a[(size_t)i * h.A + a] - h.mean[(size_t)i * h.A + a];
                lp_now += -(d[a] * d[a]) * (0.5f * h.inv_var[a]) - h.log_std[a] - 0.91893853320467274178f;
                lp_old += h.lp[(size_t)i * h.A + a];
            }
            const float adv = h.adv[i];
            const float ratio = expf(lp_now - lp_old);
            const float lo = 1.f - h.eps_clip, hi = 1.f + h.eps_clip;
            const float s1 = ratio * adv, rc = fminf(fmaxf(ratio, lo), hi), s2 = rc * adv;
            const float w1 = s1 < s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);  // torch.min: a tie splits
            const float w2 = s2 < s1 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
            const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;  // clamp backward
            const float dl_dlp = -adv * (w1 + w2 * inr) * ratio * h.inv_rows;
            for (int a = 0; a < h.A; ++a)
                h.dy[(size_t)i * h.A + a] = dl_dlp * (d[a] * h.inv_var[a]) * h.gain[a] * (1.f - t[a] * t[a]);
            l = (double)(-fminf(s1, s2) - h.ent_row);
        } else {
            const float diff = h.v[i] - h.vt[i];
            h.dy[i] = 2.f * diff * h.inv_rows;
            l = (double)(diff * diff);
        }
    }
    for (int o = 1; o < 64; o <<= 1) l += __shfl_xor(l, o);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l;
    __syncthreads();
    if (threadIdx.x == 0) h.lpart[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// *loss_sum += the head blocks' partials, in block order then a fixed shuffle / LDS tree
__global__ void __launch_bounds__(256) loss_sum_kernel(const double *__restrict__ lpart, int64_t n,
                                                       double *loss_sum) {
    double l = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 256) l += lpart[i];
    for (int o = 1; o < 64; o <<= 1) l += __shfl_xor(l, o);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l;
    __syncthreads();
    if (threadIdx.x == 0) *loss_sum += (red[0] + red[1]) + (red[2] + red[3]);
}

// the workspace's constant vectors: 1024 ones (the hidden layers' tanh backward through the
// kEpiTanhAffBack epilogue with gain 1) and the actor head's gain / off
struct PpoConsts {
    float gain[4], off[4];
};
__global__ void __launch_bounds__(256) ppo2_consts_kernel(float *ones, float *head, PpoConsts c) {
    for (int i = threadIdx.x; i < 1024; i += 256) ones[i] = 1.f;
    if (threadIdx.x < 4) {
        head[threadIdx.x] = c.gain[threadIdx.x];
        head[4 + threadIdx.x] = c.off[threadIdx.x];
    }
}

// grad[i] = sum over the chunk slots, in chunk order
__global__ void __launch_bounds__(256) chunk_sum_kernel(const float *__restrict__ slots, int nchunks,
                                                        int64_t n, float *__restrict__ grad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float s = 0.f;
#pragma unroll 4
    for (int c = 0; c < nchunks; ++c) s += slots[(size_t)c * n + i];
    grad[i] = s;
}

struct PpoDenseWs {  // float offsets into the workspace
    int64_t act, t, g0, g1, g2, g3, part, ones, head, slots, lpart, fg_part, fg_lpart, total;
};
inline bool ppo2_dense_ok(const rlp_mlp_desc &d, bool actor) {
    if (d.n_layers < 1 || d.n_layers > RLP_MLP_MAX_LAYERS) return false;
    for (int l = 0; l <= d.n_layers; ++l)
        if (d.dims[l] < 1 || d.dims[l] > 1024) return false;
    for (int l = 0; l + 1 < d.n_layers; ++l)
        if (d.act[l] != RLP_ACT_TANH) return false;
    const int A = d.dims[d.n_layers];
    return actor ? (A <= 4 && d.act[d.n_layers - 1] == RLP_ACT_TANH)
                 : (A == 1 && d.act[d.n_layers - 1] == RLP_ACT_NONE);
}
// the whole forward as one chain launch: three or four tanh layers, <= 64 inputs, the first two
// hidden widths multiples of 32 up to 256, a third hidden width up to 128, <= 8 outputs (the
// PPO2-SOI demo's 4-128-64-32-2 / 4-64-64-1, the lidar demos' 41-256-256-{2,1})
inline bool ppo2_chain_ok(const rlp_mlp_desc &d) {
    const int L = d.n_layers;
    if ((L != 3 && L != 4) || d.dims[0] > kChK0 || d.dims[L] > 8) return false;
    for (int l = 1; l <= 2; ++l)
        if (d.dims[l] > kChH || d.dims[l] % 32) return false;
    return L == 3 || d.dims[3] <= 16 * kChWaves;
}
// the backward as one data chain (dH of every hidden layer, tanh') + every layer's weight
// gradient in one launch + one reduce: the forward chain's nets whose third hidden width (four
// layers) is a multiple of 32
inline bool ppo2_chain_bwd_ok(const rlp_mlp_desc &d) {
    return ppo2_chain_ok(d) && (d.n_layers == 3 || d.dims[3] % 32 == 0) && d.n_layers <= kMaxRegions;
}
// reduction slices of layer l's weight gradient over a chunk (512 blocks per launch)
inline int64_t ppo2_wgrad_nz(const rlp_mlp_desc &d, int l) {
    const int64_t tiles = ((d.dims[l] + 1 + kDT - 1) / kDT) * ((d.dims[l + 1] + kDT - 1) / kDT);
    return 512 / tiles > 1 ? 512 / tiles : 1;
}
// the shapes fg_grad_kernel takes: <= 8 inputs, hidden (128, 64, 32) or (64, 64), head <= 4
// (actor) / 1 (critic) — the PPO2-SOI demo's nets
inline int ppo2_fused_kind(const rlp_mlp_desc &d) {
    const int L = d.n_layers;
    if (d.dims[0] > 8 || d.dims[L] > 4) return 0;
    if (L == 4 && d.dims[1] == 128 && d.dims[2] == 64 && d.dims[3] == 32) return 1;
    if (L == 3 && d.dims[1] == 64 && d.dims[2] == 64) return 2;
    return 0;
}
inline int dense_cus() { return device_cus(); }  // the fused kernel's workspace and grid
inline PpoDenseWs ppo2_dense_ws(const rlp_mlp_desc &d, int64_t rows) {
    const int64_t B = rows < kPpoChunk ? rows : kPpoChunk;
    int64_t hid = 0, maxw = 0, np = 0, maxpart = 0, sumpart = 0;
    for (int l = 0; l < d.n_layers; ++l) {
        hid += d.dims[l + 1];
        maxw = d.dims[l + 1] > maxw ? d.dims[l + 1] : maxw;
        np += (int64_t)d.dims[l] * d.dims[l + 1] + d.dims[l + 1];
        const int64_t p = ppo2_wgrad_nz(d, l) * d.dims[l + 1] * (d.dims[l] + 1);
        maxpart = p > maxpart ? p : maxpart;
        sumpart += p;
    }
    const bool chain = ppo2_chain_bwd_ok(d);  // every layer's partials at once
    const int64_t chunks = (rows + kPpoChunk - 1) / kPpoChunk;
    PpoDenseWs w{};
    int64_t o = 0;
    auto take = [&](int64_t k) { int64_t r = o; o += (k + 63) / 64 * 64; return r; };
    w.act = take(B * hid);
    w.t = take(B * 4);
    w.g0 = take(B * maxw);
    w.g1 = take(B * maxw);
    w.g2 = chain ? take(B * maxw) : w.g1;
    w.g3 = chain ? take(B * maxw) : w.g1;
    w.part = take(chain ? sumpart : maxpart);
    w.ones = take(1024);
    w.head = take(8);
    w.slots = take(chunks * np);
    w.lpart = take(2 * ((rows + 255) / 256));  // f64 loss partial per head block
    if (ppo2_fused_kind(d)) {  // fg_grad_kernel: one partial gradient and loss per block
        w.fg_part = take((int64_t)dense_cus() * np);
        w.fg_lpart = take(2 * (int64_t)dense_cus());
    }
    w.total = o;
    return w;
}

// tanh for the EXT layer 1 (l1_fwd_kernel: 0.56 -> 0.50 ms per 2^20 rows; in fg_grad_kernel,
// which LDS bounds, it measured 1-2 % slower, so that kernel keeps tanhf; r5q_tanh_ab.txt):
// ocml's tanhf shape (an odd polynomial near 0, 1 - 2 / (exp(2|x|) + 1) above) with the
// polynomial carried to |x| < 0.8 and the exponential on v_exp_f32 directly (ocml rebuilds exp
// from a split argument and ldexp: 27 VALU against 17). The polynomial x + x^3 P(x^2)
// (coefficients fitted for relative error) is within 0.8 ulp of tanh in f32 Horner form; above
// 0.8 the result is >= 0.66, so 1 - 2r has no cancellation: <= 2.3 ulp with 1-ulp v_exp_f32 /
// v_rcp_f32 (ocml tanhf: <= 2 ulp).
__device__ __forceinline__ float tanh_x3(float x) {
    const float ax = fabsf(x), t = x * x;
    float p = -0.0005696456741425663f;
    p = __builtin_fmaf(p, t, 0.002847711636260569f);
    p = __builtin_fmaf(p, t, -0.008504900349316143f);
    p = __builtin_fmaf(p, t, 0.021770580912164706f);
    p = __builtin_fmaf(p, t, -0.05395333174766384f);
    p = __builtin_fmaf(p, t, 0.13333225206779578f);
    p = __builtin_fmaf(p, t, -0.3333333065982628f);
    const float sm = __builtin_fmaf(ax * t, p, ax);
    const float ex = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);  // exp(2 |x|)
    const float bg = __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(ex + 1.f), 1.f);
    return __builtin_copysignf(ax < 0.8f ? sm : bg, x);
}

// ---- fused per-row gradient for the PPO2-SOI demo's small nets ---------------------------------
// actor 4 -> 128 -> 64 -> 32 -> 2 / critic 4 -> 64 -> 64 -> 1 (demonstration/PPO2/
// PPO2-4-SecondOrderIntegration/train.py:37-125): per 32-row step ONE block runs the forward, the
// loss head, the backward data passes and the weight-gradient accumulation, every activation and
// hidden gradient in LDS (the chunked path sends them through HBM five launches per chunk:
// forward chain, head, backward chain, weight-gradient GEMM, reduce; 18 TF/s, r5h). Exact f32
// MFMA (v_mfma_f32_16x16x4_f32) throughout; one 8-wave block per CU over a static row stride; the
// weight gradient of the block's rows stays in the MFMA accumulators (each wave owns a fixed set
// of 16 x 16 dW | db tiles) and is written once as the block's partial, summed over blocks in a
// fixed order (run-to-run identical, as the chunked path).
// LDS rows are x + (17 - x) mod 32 floats long (== 17 mod 32): the three operand-read patterns
// (lane (g, e) reading [16 e + ..][g] and [g][e + ..]) then hit at most two lanes per bank.
constexpr int kFgRows = 32;
constexpr int kFgWaves = 8;
__host__ __device__ constexpr int fg_ld(int x) { return x + ((17 - x % 32) + 32) % 32; }

template <int H1, int H2, int H3>
struct FgShape {
    static constexpr int L = H3 ? 4 : 3;
    // padded widths: inputs <= 8, hidden H1, H2 (, H3), the head 16
    __host__ __device__ static constexpr int width(int l) {
        return l == 0 ? 8 : l == L ? 16 : l == 1 ? H1 : l == 2 ? H2 : H3;
    }
    // LDS (floats): X | H_1 .. H_{L-1} | Z | dA | dB | W_1 .. W_L | b_1 .. b_L
    __host__ __device__ static constexpr int act_ld(int l) { return fg_ld(l == 0 ? 16 : l == L ? 16 : width(l) + 1); }
    __host__ __device__ static constexpr int hmax() { return H1 > H2 ? H1 : H2; }
    __host__ __device__ static constexpr int w_ld(int l) { return fg_ld(width(l - 1)); }   // W_l [width(l)][w_ld(l)]
    __host__ __device__ static constexpr int off_act(int l) {  // X = 0, H_l = l, Z = L
        int o = 0;
        for (int i = 0; i < l; ++i) o += kFgRows * act_ld(i);
        return o;
    }
    __host__ __device__ static constexpr int off_dA() { return off_act(L + 1); }
    __host__ __device__ static constexpr int off_dB() { return off_dA() + kFgRows * fg_ld(hmax()); }
    __host__ __device__ static constexpr int off_w(int l) {
        int o = off_dB() + kFgRows * fg_ld(hmax());
        for (int i = 1; i < l; ++i) o += width(i) * w_ld(i);
        return o;
    }
    __host__ __device__ static constexpr int off_b(int l) {
        int o = off_w(L + 1);
        for (int i = 1; i < l; ++i) o += width(i);
        return o;
    }
    __host__ __device__ static constexpr int floats() { return off_b(L + 1); }
    // dW | db tiles of layer l: width(l) / 16 x ceil((in + 1) / 16) (in = 8 padded inputs for l = 1)
    __host__ __device__ static constexpr int ntn(int l) { return l == 1 ? 1 : (width(l - 1) + 1 + 15) / 16; }
    __host__ __device__ static constexpr int tiles(int l) { return width(l) / 16 * ntn(l); }
    __host__ __device__ static constexpr int tile0(int l) {
        int o = 0;
        for (int i = 1; i < l; ++i) o += tiles(i);
        return o;
    }
    __host__ __device__ static constexpr int tiles_total() { return tile0(L + 1); }
    __host__ __device__ static constexpr int per_wave() { return (tiles_total() + kFgWaves - 1) / kFgWaves; }
};

struct FgArgs {
    const float *params;       // plain layout (torch order)
    const float *s, *a, *lp, *adv, *vt;
    int64_t rows;
    int S, A;                  // inputs (<= 8), actor outputs (<= 4; critic 1)
    int dims[5];               // true widths: S, hidden..., out
    int64_t off[4];            // W_l offsets in params (b_l follows W_l)
    int64_t np;                // parameters
    float inv_rows, eps_clip, ent_row;
    float gain[4], off_[4], log_std[4], inv_var[4];
    float *part;               // [grid][np]: the blocks' dW | db partials (torch order)
    double *lpart;             // [grid]: the blocks' loss partials
};

template <int H1, int H2, int H3, bool ACTOR>
__global__ void __launch_bounds__(64 * kFgWaves, 1) fg_grad_kernel(FgArgs g) {
    using F = FgShape<H1, H2, H3>;
    constexpr int L = F::L;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int t = threadIdx.x, lane = t & 63, gq = lane >> 4, e = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    // zero everything once (padding rows / columns are read as operands), then weights, biases
    for (int i = t; i < F::floats(); i += 64 * kFgWaves) lds[i] = 0.f;
    __syncthreads();
#pragma unroll
    for (int l = 1; l <= L; ++l) {
        const int in = g.dims[l - 1], out = g.dims[l];
        const float *W = g.params + g.off[l - 1], *b = W + (int64_t)in * out;
        for (int i = t; i < in * out; i += 64 * kFgWaves) {
            const int o = i / in, k = i - o * in;
            lds[F::off_w(l) + o * F::w_ld(l) + k] = W[i];
        }
        for (int i = t; i < out; i += 64 * kFgWaves) lds[F::off_b(l) + i] = b[i];
    }
    // the ones columns (bias of the next layer's weight gradient) of H_1 .. H_{L-1}
#pragma unroll
    for (int l = 1; l < L; ++l)
        for (int r = t; r < kFgRows; r += 64 * kFgWaves) lds[F::off_act(l) + r * F::act_ld(l) + g.dims[l]] = 1.f;
    floatx4 acc[F::per_wave()];
#pragma unroll
    for (int j = 0; j < F::per_wave(); ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // layer 2's weight operands stay in registers for the whole launch (they are a fixed tile per
    // wave: the forward's output tile 16 (wv / 2) and the data pass's input tiles 16 (wv / 2 + 4 i)),
    // a third of the LDS operand reads gone: W2 [H2][H1] row-major in params
    constexpr int NW2 = H1 / 64;   // data-pass tiles of layer 2 per wave
    static_assert(H2 / 16 * (kFgRows / 16) == kFgWaves && (kFgRows / 16) * (H1 / 16) == kFgWaves * NW2,
                  "layer 2: one forward tile and NW2 data-pass tiles per wave (tau = wv + 8 i)");
    float w2f[H1 / 4], w2d[NW2][H2 / 4];
    {
        const float *W2 = g.params + g.off[1];
        const int m2 = wv >> 1;
#pragma unroll
        for (int k4 = 0; k4 < H1 / 4; ++k4) w2f[k4] = W2[(16 * m2 + e) * H1 + 4 * k4 + gq];
#pragma unroll
        for (int i = 0; i < NW2; ++i)
#pragma unroll
            for (int k4 = 0; k4 < H2 / 4; ++k4) w2d[i][k4] = W2[(4 * k4 + gq) * H1 + 16 * (m2 + 4 * i) + e];
    }
    double lsum = 0.0;
    const int S = g.S, A = g.A, ks0 = (S + 3) / 4;
    const int64_t nsteps = (g.rows + kFgRows - 1) / kFgRows;
    // one 16 x 16 output tile: acc over K / 4 MFMA steps, a(k) / b(k) the lane's operands
    // (the 4-layer actor: two accumulation chains, even and odd K steps, added at the end — one
    // chain waits out the f32 MFMA's dependent-accumulator latency at every step: -2.5 %; the
    // 3-layer critic measured 1.5 % slower with them, r5r_fg_chains_ab.txt)
    auto mm = [&](floatx4 c, int K, auto &&av, auto &&bv) {
        floatx4 c1 = {0.f, 0.f, 0.f, 0.f};
        int k0 = 0;
#pragma unroll 2
        for (; H3 > 0 && k0 + 8 <= K; k0 += 8) {
            c = __builtin_amdgcn_mfma_f32_16x16x4f32(av(k0 + gq), bv(k0 + gq), c, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av(k0 + 4 + gq), bv(k0 + 4 + gq), c1, 0, 0, 0);
        }
#pragma unroll 2
        for (; k0 < K; k0 += 4) c = __builtin_amdgcn_mfma_f32_16x16x4f32(av(k0 + gq), bv(k0 + gq), c, 0, 0, 0);
        return H3 > 0 ? c + c1 : c;
    };
    for (int64_t step = blockIdx.x; step < nsteps; step += gridDim.x) {
        const int64_t r0 = step * kFgRows;
        const int nr = (int)(g.rows - r0 < kFgRows ? g.rows - r0 : kFgRows);
        __syncthreads();  // the previous step's X / dZ reads are done
        // X: s | 1 | 0 (rows past the end all zero)
        for (int i = t; i < kFgRows * 16; i += 64 * kFgWaves) {
            const int r = i >> 4, c = i & 15;
            float v = 0.f;
            if (r < nr) v = c < S ? g.s[(r0 + r) * S + c] : (c == S ? 1.f : 0.f);
            lds[F::off_act(0) + r * F::act_ld(0) + c] = v;
        }
        // the head's row inputs (wave 0, lane = row)
        float in_a[4] = {0.f, 0.f, 0.f, 0.f}, in_lp[4] = {0.f, 0.f, 0.f, 0.f}, in_x = 0.f;
        if (wv == 0 && lane < nr) {
            if constexpr (ACTOR) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < A) {
                        in_a[k] = g.a[(r0 + lane) * A + k];
                        in_lp[k] = g.lp[(r0 + lane) * A + k];
                    }
                in_x = g.adv[r0 + lane];
            } else {
                in_x = g.vt[r0 + lane];
            }
        }
        __syncthreads();
        // ---- forward: C[out][row] = W_l H_{l-1}^T + b, tanh (hidden) or z (last) -------------
#pragma unroll
        for (int l = 1; l <= L; ++l) {
            const int M = F::width(l), K = l == 1 ? 4 * ks0 : F::width(l - 1);
            const float *Wl = lds + F::off_w(l), *bl = lds + F::off_b(l);
            const float *Hp = lds + F::off_act(l - 1);
            float *Hc = lds + F::off_act(l);
            const int lwp = F::w_ld(l), lhp = F::act_ld(l - 1), lhc = F::act_ld(l);
            for (int tau = wv; tau < M / 16 * (kFgRows / 16); tau += kFgWaves) {
                const int mt = tau >> 1, rt = tau & 1;
                floatx4 c = {bl[16 * mt + 4 * gq], bl[16 * mt + 4 * gq + 1], bl[16 * mt + 4 * gq + 2],
                             bl[16 * mt + 4 * gq + 3]};
                if (l == 2) {  // one tile per wave (tau = wv), A operands from w2f
                    floatx4 c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int k4 = 0; k4 < H1 / 4; k4 += 2) {
                        c = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[k4], Hp[(16 * rt + e) * lhp + 4 * k4 + gq], c, 0, 0, 0);
                        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[k4 + 1], Hp[(16 * rt + e) * lhp + 4 * k4 + 4 + gq], c1, 0, 0, 0);
                    }
                    c = c + c1;
                } else {
                    c = mm(c, K, [&](int k) { return Wl[(16 * mt + e) * lwp + k]; },
                           [&](int k) { return Hp[(16 * rt + e) * lhp + k]; });
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float v = c[q];
                    Hc[(16 * rt + e) * lhc + 16 * mt + 4 * gq + q] = l < L ? tanhf(v) : v;
                }
            }
            __syncthreads();
        }
        // ---- loss head: dZ_L in place of Z (wave 0, lane = row; padding rows / columns zero) --
        if (wv == 0 && lane < kFgRows) {
            float *z = lds + F::off_act(L) + lane * F::act_ld(L);
            const bool valid = lane < nr;
            double l = 0.0;
            if constexpr (ACTOR) {
                float lp_now = 0.f, lp_old = 0.f, d[4] = {0.f, 0.f, 0.f, 0.f}, tt[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k >= A) continue;
                    tt[k] = tanhf(z[k]);
                    d[k] = in_a[k] - (tt[k] * g.gain[k] + g.off_[k]);
                    lp_now += -(d[k] * d[k]) * (0.5f * g.inv_var[k]) - g.log_std[k] - 0.91893853320467274178f;
                    lp_old += in_lp[k];
                }
                const float adv = in_x;
                const float ratio = expf(lp_now - lp_old);
                const float lo = 1.f - g.eps_clip, hi = 1.f + g.eps_clip;
                const float s1 = ratio * adv, rc = fminf(fmaxf(ratio, lo), hi), s2 = rc * adv;
                const float w1 = s1 < s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);  // torch.min: a tie splits
                const float w2 = s2 < s1 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
                const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;  // clamp backward
                const float dl_dlp = -adv * (w1 + w2 * inr) * ratio * g.inv_rows;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < A) z[k] = valid ? dl_dlp * (d[k] * g.inv_var[k]) * g.gain[k] * (1.f - tt[k] * tt[k]) : 0.f;
                l = valid ? (double)(-fminf(s1, s2) - g.ent_row) : 0.0;
            } else {
                const float diff = z[0] - in_x;
                z[0] = valid ? 2.f * diff * g.inv_rows : 0.f;
                l = valid ? (double)(diff * diff) : 0.0;
            }
            for (int k = ACTOR ? A : 1; k < 16; ++k) z[k] = 0.f;
            lsum += l;
        }
        __syncthreads();
        // ---- backward: per layer (top down) the weight-gradient tiles this wave owns
        // (dW | db += dZ_l^T [H_{l-1} | 1], K = the step's rows) and the data pass
        // dZ_{l-1} = (dZ_l W_l) * (1 - H_{l-1}^2) into the other gradient buffer
#pragma unroll
        for (int l = L; l >= 1; --l) {
            const float *dZ = lds + (l == L ? F::off_act(L) : ((L - l) % 2 ? F::off_dA() : F::off_dB()));
            const int ldz = l == L ? F::act_ld(L) : fg_ld(F::hmax());
            const float *Hp = lds + F::off_act(l - 1);
            const int lhp = F::act_ld(l - 1);
#pragma unroll
            for (int j = 0; j < F::per_wave(); ++j) {
                const int T = wv + kFgWaves * j - F::tile0(l);
                if (T < 0 || T >= F::tiles(l)) continue;
                const int mt = T / F::ntn(l), nt = T - mt * F::ntn(l);
                acc[j] = mm(acc[j], kFgRows, [&](int k) { return dZ[k * ldz + 16 * mt + e]; },
                            [&](int k) { return Hp[k * lhp + 16 * nt + e]; });
            }
            if (l > 1) {
                const int M = F::width(l), N = F::width(l - 1);
                const float *Wl = lds + F::off_w(l);
                const int lw = F::w_ld(l);
                float *dP = lds + ((L - l + 1) % 2 ? F::off_dA() : F::off_dB());
                const int ldp = fg_ld(F::hmax());
                for (int tau = wv; tau < (kFgRows / 16) * (N / 16); tau += kFgWaves) {
                    const int rt = tau % (kFgRows / 16), nt = tau / (kFgRows / 16);
                    floatx4 c = {0.f, 0.f, 0.f, 0.f};
                    if (l == 2) {  // tau = wv + 8 i, B operands from w2d[i]
#pragma unroll
                        for (int i = 0; i < NW2; ++i) {
                            if (tau != wv + kFgWaves * i) continue;
                            floatx4 c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                            for (int k4 = 0; k4 < H2 / 4; k4 += 2) {
                                c = __builtin_amdgcn_mfma_f32_16x16x4f32(dZ[(16 * rt + e) * ldz + 4 * k4 + gq], w2d[i][k4], c, 0, 0, 0);
                                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(dZ[(16 * rt + e) * ldz + 4 * k4 + 4 + gq], w2d[i][k4 + 1], c1, 0, 0, 0);
                            }
                            c = c + c1;
                        }
                    } else {
                        c = mm(c, M, [&](int k) { return dZ[(16 * rt + e) * ldz + k]; },
                               [&](int k) { return Wl[k * lw + 16 * nt + e]; });
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int r = 16 * rt + 4 * gq + q, n = 16 * nt + e;
                        const float h = Hp[r * lhp + n];
                        dP[r * ldp + n] = c[q] * __builtin_fmaf(-h, h, 1.f);
                    }
                }
            }
            __syncthreads();
        }
    }
    // ---- the block's partials: dW | db tiles in torch order, the loss
    float *out = g.part + (int64_t)blockIdx.x * g.np;
#pragma unroll
    for (int j = 0; j < F::per_wave(); ++j) {
        const int T = wv + kFgWaves * j;
        if (T >= F::tiles_total()) continue;
        int l = 1;
#pragma unroll
        for (int i = 2; i <= L; ++i)
            if (T >= F::tile0(i)) l = i;
        const int Tl = T - F::tile0(l), mt = Tl / F::ntn(l), nt = Tl - mt * F::ntn(l);
        const int in = g.dims[l - 1], outw = g.dims[l];
        float *W = out + g.off[l - 1], *b = W + (int64_t)in * outw;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int o = 16 * mt + 4 * gq + q, c = 16 * nt + e;
            if (o >= outw) continue;
            if (c < in) W[o * in + c] = acc[j][q];
            else if (c == in) b[o] = acc[j][q];
        }
    }
    if (wv == 0) {
        for (int o = 1; o < 64; o <<= 1) lsum += __shfl_xor(lsum, o);
        if (lane == 0) g.lpart[blockIdx.x] = lsum;
    }
}

// ---- layer 1 of the 41-input nets for rlp_ppo2_grad (rlp_update.hip, "EXT" kernels) -----------
// The f16x3 FD / wgrad kernels take h1 = tanh(s W1^T + b1) from HBM and hand g1 = dL/dz1 back;
// the two layer-1 products run here as exact-f32 MFMA kernels of their own (v_mfma_f32_16x16x4_f32,
// f32 accumulation, as torch's f32 GEMM). Both are HBM-bound (1 KiB of h1 written / of g1 read per
// row against 164 B of s): the s rows of a tile are one contiguous span, loaded coalesced and
// transposed into LDS (the tiled GEMM's generic loader spent 46 VALU per MFMA on the 41-float rows:
// 1.9 ms for the forward of 2^20 rows, profiles/r5/r5f_ext_pmc_shapes.txt).
constexpr int kL1Waves = 8;        // forward: 8-wave blocks share one W1^T copy in LDS
constexpr int kL1Rows = 16 * kL1Waves;  // rows per forward tile (16 per wave)
constexpr int kL1Ld = 256 + 16;    // LDS row of 256 floats: lane groups g, g + 1 16 banks apart
constexpr int kL1SLd = kL1Rows + 16;
constexpr int kL1WRows = 32;       // rows per weight-gradient step
constexpr int kL1WLd = 48;         // s tile row (features | 1 | 0 pad): 16 banks between rows
constexpr int kL1WBlocks = 512;    // weight-gradient blocks (per-block partials, fixed-order reduce)

// row / column of flat index f of a [*][S] row-major span, without an integer division:
// (f + 0.5) / S lies at least 0.5 / S from an integer, far beyond the float rounding for f < 2^20
__device__ __forceinline__ int l1_row(int f, float invS) { return (int)(((float)f + 0.5f) * invS); }

// h1[row][256] = tanh(W1 s_row + b1) for 128-row tiles (grid-stride), W1^T and the tile's s^T in
// LDS. Wave w: rows 16 w .. 16 w + 15, the 16 neuron tiles in two halves of 8 (C = [neuron][row],
// 32 accumulators); lane (g, e) stores neurons 16 t + 4 g .. + 3 of row e as one float4. Eight
// waves share the block's W1^T (48 KiB) and stay within 128 registers: two blocks per CU give 4
// waves per SIMD to overlap one wave's MFMAs with another's tanh and h1 stores (4-wave blocks,
// 64-row tiles, all 16 tiles at once: LDS and registers allowed 2 waves per SIMD).
template <int KS>
__global__ void __launch_bounds__(64 * kL1Waves, 4) l1_fwd_kernel(const float *__restrict__ s, int S,
                                                                  int64_t rows,
                                                                  const float *__restrict__ W1, int ldw,
                                                                  const float *__restrict__ b1,
                                                                  float *__restrict__ h1) {
    constexpr int NT = 64 * kL1Waves;           // threads
    __shared__ float w1t[4 * KS][kL1Ld];        // [k][neuron]
    __shared__ float st[4 * KS][kL1SLd];        // [k][row]
    const int t = threadIdx.x, lane = t & 63, g = lane >> 4, e = lane & 15, w = t >> 6;
    for (int i = t; i < 4 * KS * 256; i += NT) {
        const int n = i / (4 * KS), k = i - n * (4 * KS);
        w1t[k][n] = k < S ? W1[(int64_t)n * ldw + k] : 0.f;
    }
    const float invS = 1.f / (float)S;
    const int64_t ntiles = (rows + kL1Rows - 1) / kL1Rows;
    // the tile's s span (nr * S <= 128 * 4 KS floats, contiguous) in registers, loaded one tile
    // ahead so that its latency hides under the current tile's MFMAs and stores
    constexpr int NSV = (kL1Rows * 4 * KS + NT - 1) / NT;
    float sv[NSV];
    auto load_s = [&](int64_t tile) {
        const int64_t r0 = tile * kL1Rows;
        const int n = tile < ntiles ? (int)(rows - r0 < kL1Rows ? rows - r0 : kL1Rows) * S : 0;
        const float *src = s + r0 * S;
#pragma unroll
        for (int u = 0; u < NSV; ++u) {
            const int f = t + NT * u;
            sv[u] = f < n ? src[f] : 0.f;
        }
    };
    load_s(blockIdx.x);
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tile * kL1Rows;
        const int nr = (int)(rows - r0 < kL1Rows ? rows - r0 : kL1Rows);
        __syncthreads();  // the previous tile's s^T is read
        for (int f = t; f < kL1Rows * 4 * KS; f += NT) {  // zero the padding columns / rows first
            const int k = f / kL1Rows, r = f - k * kL1Rows;
            if (k >= S || r >= nr) st[k][r] = 0.f;
        }
#pragma unroll
        for (int u = 0; u < NSV; ++u) {  // the span transposed into st (row r, feature f - r S)
            const int f = t + NT * u;
            if (f < nr * S) {
                const int r = l1_row(f, invS);
                st[f - r * S][r] = sv[u];
            }
        }
        __syncthreads();
        load_s(tile + gridDim.x);
        const int r = 16 * w + e;
#pragma unroll 1
        for (int hf = 0; hf < 2; ++hf) {  // neurons 128 hf .. 128 hf + 127: 32 accumulators
            floatx4 acc[8];
#pragma unroll
            for (int nt = 0; nt < 8; ++nt)
                acc[nt] = *reinterpret_cast<const floatx4 *>(b1 + 128 * hf + 16 * nt + 4 * g);
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) {
                const float bv = st[4 * kk + g][16 * w + e];
#pragma unroll
                for (int nt = 0; nt < 8; ++nt)
                    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1t[4 * kk + g][128 * hf + 16 * nt + e],
                                                                   bv, acc[nt], 0, 0, 0);
            }
            if (r < nr) {
                float *dst = h1 + (r0 + r) * 256 + 128 * hf + 4 * g;
#pragma unroll
                for (int nt = 0; nt < 8; ++nt) {
                    floatx4 v;
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = tanh_x3(acc[nt][q]);
                    *reinterpret_cast<floatx4 *>(dst + 16 * nt) = v;
                }
            }
        }
    }
}

// part[b][256][S + 1] = sum over block b's rows of g1[row] (x) [s_row | 1]: dW1 | db1 partials,
// g1 = dL/dh1 * (1 - h1^2) formed here from the FD kernel's dL/dh1 rows and h1 (the same product
// the FD tail formed before: (dL/dh1 * unscale) * fma(-h1, h1, 1), bit-identical).
// Wave w owns neurons 64 w .. 64 w + 63 (4 tiles) x FT feature tiles (C = [neuron][feature]);
// 32-row steps, the next step's g1 rows loaded into registers under the current step's MFMAs.
template <int FT>
__global__ void __launch_bounds__(256) l1_wgrad_kernel(const float *__restrict__ g1,
                                                       const float *__restrict__ h1,
                                                       const float *__restrict__ s, int S, int64_t rows,
                                                       int64_t rpb, float *__restrict__ part) {
    __shared__ __attribute__((aligned(16))) float gt[kL1WRows][kL1Ld];  // [row][neuron]
    __shared__ float sx[kL1WRows][kL1WLd];                              // [row][feature | 1]
    const int t = threadIdx.x, lane = t & 63, g = lane >> 4, e = lane & 15, w = t >> 6;
    const int64_t lo = blockIdx.x * rpb, hi = lo + rpb < rows ? lo + rpb : rows;
    const float invS = 1.f / (float)S;
    floatx4 acc[4][FT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    constexpr int NV = kL1WRows * 256 / 4 / 256;  // float4 of g1 per thread and step (8)
    floatx4 v[NV], hv[NV];
    auto load = [&](int64_t r0) {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int i = t + 256 * u, r = i >> 6;
            const bool in = r0 + r < hi;
            v[u] = in ? *reinterpret_cast<const floatx4 *>(g1 + (r0 + r) * 256 + 4 * (i & 63))
                      : floatx4{0.f, 0.f, 0.f, 0.f};
            hv[u] = in ? *reinterpret_cast<const floatx4 *>(h1 + (r0 + r) * 256 + 4 * (i & 63))
                       : floatx4{0.f, 0.f, 0.f, 0.f};
        }
    };
    // the step's s span (nr * S <= 32 x 44 floats, contiguous) likewise one step ahead
    constexpr int NSV = (kL1WRows * (kL1WLd - 4) + 255) / 256;
    float sv[NSV];
    auto load_s = [&](int64_t r0) {
        const int n = r0 < hi ? (int)(hi - r0 < kL1WRows ? hi - r0 : kL1WRows) * S : 0;
#pragma unroll
        for (int u = 0; u < NSV; ++u) {
            const int f = t + 256 * u;
            sv[u] = f < n ? s[r0 * S + f] : 0.f;
        }
    };
    if (lo < hi) {
        load(lo);
        load_s(lo);
    }
    for (int64_t r0 = lo; r0 < hi; r0 += kL1WRows) {
        const int nr = (int)(hi - r0 < kL1WRows ? hi - r0 : kL1WRows);
        __syncthreads();  // the previous step's tiles are read
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int i = t + 256 * u;
            floatx4 gz;  // dL/dz1 = dL/dh1 * (1 - h1^2)
#pragma unroll
            for (int c = 0; c < 4; ++c) gz[c] = v[u][c] * __builtin_fmaf(-hv[u][c], hv[u][c], 1.f);
            *reinterpret_cast<floatx4 *>(&gt[i >> 6][4 * (i & 63)]) = gz;
        }
        for (int f = t; f < kL1WRows * kL1WLd; f += 256) {  // ones column, zero padding
            const int r = f / kL1WLd, c = f - r * kL1WLd;
            if (c >= S) sx[r][c] = (c == S && r < nr) ? 1.f : 0.f;
            else if (r >= nr) sx[r][c] = 0.f;
        }
#pragma unroll
        for (int u = 0; u < NSV; ++u) {
            const int f = t + 256 * u;
            if (f < nr * S) {
                const int r = l1_row(f, invS);
                sx[r][f - r * S] = sv[u];
            }
        }
        __syncthreads();
        if (r0 + kL1WRows < hi) {  // next step, under this step's MFMAs
            load(r0 + kL1WRows);
            load_s(r0 + kL1WRows);
        }
#pragma unroll
        for (int k0 = 0; k0 < kL1WRows; k0 += 4) {
            float bv[FT];
#pragma unroll
            for (int j = 0; j < FT; ++j) bv[j] = sx[k0 + g][16 * j + e];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float av = gt[k0 + g][64 * w + 16 * i + e];
#pragma unroll
                for (int j = 0; j < FT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[j], acc[i][j], 0, 0, 0);
            }
        }
    }
    // C layout: lane (g, e) holds neurons 64 w + 16 i + 4 g + q, feature 16 j + e
    float *out = part + (int64_t)blockIdx.x * 256 * (S + 1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FT; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = 64 * w + 16 * i + 4 * g + q, c = 16 * j + e;
                if (c <= S) out[n * (S + 1) + c] = acc[i][j][q];
            }
}

int64_t ppo2_ext_floats(int S, int H, int64_t rows) {
    (void)rows;
    return (int64_t)kL1WBlocks * H * (S + 1);
}
void ppo2_ext_h1(const float *W1, int ldw, const float *b1, int S, int H, const float *s,
                 int64_t rows, float *h1, hipStream_t st) {
    (void)H;
    const int64_t ntiles = (rows + kL1Rows - 1) / kL1Rows;
    const int grid = (int)(ntiles < 512 ? ntiles : 512);  // 2 blocks per CU (r6w: -3.5 % vs 2048)
    l1_fwd_kernel<11><<<grid, 64 * kL1Waves, 0, st>>>(s, S, rows, W1, ldw, b1, h1);
}
void ppo2_ext_dw1(const float *g1, const float *h1, const float *s, int S, int H, int64_t rows,
                  float *part, float *gW, float *gb, hipStream_t st) {
    int64_t rpb = (rows + kL1WBlocks - 1) / kL1WBlocks;
    rpb = (rpb + kL1WRows - 1) / kL1WRows * kL1WRows;
    const int nb = (int)((rows + rpb - 1) / rpb);
    l1_wgrad_kernel<3><<<nb, 256, 0, st>>>(g1, h1, s, S, rows, rpb, part);
    wgrad_reduce(Layer{nullptr, nullptr, S, H}, part, nb, gW, gb, st);
}

}  // namespace rlp

extern "C" {

int64_t rlp_ppo2_dense_workspace_floats(const rlp_mlp_desc *desc, int64_t rows) {
    if (!desc || rows < 0 || desc->n_layers < 1 || desc->n_layers > RLP_MLP_MAX_LAYERS) return RLP_EINVAL;
    return ppo2_dense_ws(*desc, rows > 0 ? rows : 1).total;
}

int rlp_ppo2_dense_grad(const rlp_mlp_desc *desc, const float *params, const rlp_ppo2_loss_cfg *cfg,
                        const float *s, const float *a, const float *a_logprob, const float *adv,
                        const float *v_target, int64_t rows, float *grad, double *loss_sum,
                        float *workspace, rlp_stream_t stream) {
    take_pending();
    RLP_REQUIRE(desc && params && cfg && s && grad && workspace, "rlp_ppo2_dense_grad: null argument");
    const bool actor = cfg->kind == RLP_LOSS_ACTOR;
    RLP_REQUIRE(actor || cfg->kind == RLP_LOSS_CRITIC, "rlp_ppo2_dense_grad: loss kind %d", cfg->kind);
    if (!ppo2_dense_ok(*desc, actor))
        return fail(RLP_EUNSUPPORTED, "rlp_ppo2_dense_grad: need a tanh Linear stack (widths <= 1024, "
                                      "%s)", actor ? "tanh output, A <= 4" : "linear 1-output head");
    if (actor) RLP_REQUIRE(a && a_logprob && adv, "rlp_ppo2_dense_grad: actor loss needs a, a_logprob, adv");
    else RLP_REQUIRE(v_target, "rlp_ppo2_dense_grad: critic loss needs v_target");
    RLP_REQUIRE(rows > 0, "rlp_ppo2_dense_grad: rows=%lld", (long long)rows);
    const rlp_mlp_desc &d = *desc;
    const int L = d.n_layers, S = d.dims[0], A = d.dims[L];
    hipStream_t st = as_stream(stream);
    const PpoDenseWs w = ppo2_dense_ws(d, rows);
    float *ws = workspace;
    int64_t np = 0, off[RLP_MLP_MAX_LAYERS];
    for (int l = 0; l < L; ++l) {
        off[l] = np;
        np += (int64_t)d.dims[l] * d.dims[l + 1] + d.dims[l + 1];
    }
    PpoDenseArgs h{};
    h.A = A; h.inv_rows = 1.f / (float)rows; h.eps_clip = cfg->eps_clip;
    PpoConsts pc{};
    float ent = 0.f;
    for (int k = 0; k < A && actor; ++k) {
        pc.off[k] = (cfg->a_min[k] + cfg->a_max[k]) / 2.0f;
        h.gain[k] = pc.gain[k] = cfg->a_max[k] - pc.off[k];
        h.log_std[k] = logf(cfg->std[k]);
        h.inv_var[k] = 1.0f / (cfg->std[k] * cfg->std[k]);
        ent += 0.5f + 0.91893853320467274178f + logf(cfg->std[k]);  // Normal.entropy()
    }
    h.ent_row = cfg->entropy_coef * ent;
    if (const int fk = ppo2_fused_kind(d)) {  // the SOI demo's nets: one fused launch + reduces
        FgArgs f{};
        f.params = params; f.s = s; f.a = a; f.lp = a_logprob; f.adv = adv; f.vt = v_target;
        f.rows = rows; f.S = S; f.A = A;
        for (int l = 0; l <= L; ++l) f.dims[l] = d.dims[l];
        for (int l = 0; l < L; ++l) f.off[l] = off[l];
        f.np = np; f.inv_rows = h.inv_rows; f.eps_clip = h.eps_clip; f.ent_row = h.ent_row;
        for (int k = 0; k < 4; ++k) {
            f.gain[k] = h.gain[k]; f.off_[k] = pc.off[k]; f.log_std[k] = h.log_std[k]; f.inv_var[k] = h.inv_var[k];
        }
        f.part = ws + w.fg_part;
        f.lpart = reinterpret_cast<double *>(ws + w.fg_lpart);
        const int64_t nsteps = (rows + kFgRows - 1) / kFgRows;
        const int grid = (int)(nsteps < dense_cus() ? nsteps : dense_cus());
        using K1 = FgShape<128, 64, 32>;
        using K2 = FgShape<64, 64, 0>;
        const size_t lds = sizeof(float) * (fk == 1 ? K1::floats() : K2::floats());
        const void *fn = fk == 1 ? (actor ? (const void *)fg_grad_kernel<128, 64, 32, true>
                                          : (const void *)fg_grad_kernel<128, 64, 32, false>)
                                 : (actor ? (const void *)fg_grad_kernel<64, 64, 0, true>
                                          : (const void *)fg_grad_kernel<64, 64, 0, false>);
        if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return fail(RLP_EINVAL, "rlp_ppo2_dense_grad: fused kernel LDS attribute (%zu B)", lds);
        if (fk == 1) {
            if (actor) fg_grad_kernel<128, 64, 32, true><<<grid, 64 * kFgWaves, lds, st>>>(f);
            else fg_grad_kernel<128, 64, 32, false><<<grid, 64 * kFgWaves, lds, st>>>(f);
        } else {
            if (actor) fg_grad_kernel<64, 64, 0, true><<<grid, 64 * kFgWaves, lds, st>>>(f);
            else fg_grad_kernel<64, 64, 0, false><<<grid, 64 * kFgWaves, lds, st>>>(f);
        }
        chunk_sum_kernel<<<(int)((np + 255) / 256), 256, 0, st>>>(f.part, grid, np, grad);
        if (loss_sum) loss_sum_kernel<<<1, 256, 0, st>>>(f.lpart, grid, loss_sum);
        RLP_CHECK_LAUNCH("rlp_ppo2_dense_grad (fused)");
        return RLP_OK;
    }
    ppo2_consts_kernel<<<1, 256, 0, st>>>(ws + w.ones, ws + w.head, pc);
    const float *gain_d = ws + w.head, *off_d = ws + w.head + 4;
    const int64_t nchunks = (rows + kPpoChunk - 1) / kPpoChunk;
    for (int64_t c = 0; c < nchunks; ++c) {
        const int64_t r0 = c * kPpoChunk;
        const int B = (int)((rows - r0) < kPpoChunk ? rows - r0 : kPpoChunk);
        // forward
        float *act = ws + w.act;
        int64_t ao[RLP_MLP_MAX_LAYERS];
        int64_t o = 0;
        for (int l = 0; l < L; ++l) {
            ao[l] = o;
            o += (int64_t)B * d.dims[l + 1];
        }
        auto lw = [&](int l) { return params + off[l]; };
        auto lb = [&](int l) { return params + off[l] + (int64_t)d.dims[l] * d.dims[l + 1]; };
        if (ppo2_chain_ok(d)) {  // all layers in one launch (the hidden activations still to HBM)
            ChainArgs ch{};
            ch.x0 = ch.x1 = s + r0 * S; ch.ld0 = ch.ld1 = S; ch.split = S; ch.K0 = S;
            ch.W1 = lw(0); ch.b1 = lb(0); ch.W2 = lw(1); ch.b2 = lb(1);
            ch.H1 = d.dims[1]; ch.H2 = d.dims[2];
            ch.h1 = act + ao[0]; ch.h2 = act + ao[1];
            if (L == 4) {
                ch.Wm = lw(2); ch.bm = lb(2); ch.Hm = d.dims[3]; ch.hm = act + ao[2];
            }
            ch.W3 = ch.W3b = lw(L - 1); ch.b3 = lb(L - 1); ch.NO = A; ch.split3 = A;
            ch.y = act + ao[L - 1]; ch.B = B; ch.hact = 1;
            ch.head = actor ? 1 : 0; ch.gain = gain_d; ch.off = off_d; ch.aux = ws + w.t;
            chain_fwd_launch(ch, ch, 1, st);
        } else {
            Opnd in = mat(s + r0 * S, B, S, S);
            for (int l = 0; l < L; ++l) {
                const Layer Ly{lw(l), lb(l), d.dims[l], d.dims[l + 1]};
                const bool last = l == L - 1;
                const int kind = !last ? kEpiTanh : actor ? kEpiTanhAff : kEpiNone;
                dense_fwd(in, Ly, B, kind, act + ao[l], gain_d, off_d, ws + w.t, st);
                in = mat(act + ao[l], B, Ly.out, Ly.out);
            }
        }
        // head: dL/dz_L into g0
        h.B = B;
        h.dy = ws + w.g0;
        h.lpart = reinterpret_cast<double *>(ws + w.lpart) + r0 / 256;
        if (actor) {
            h.t = ws + w.t; h.mean = act + ao[L - 1];
            h.a = a + r0 * A; h.lp = a_logprob + r0 * A; h.adv = adv + r0;
            ppo2_dense_head_kernel<true><<<(B + 255) / 256, 256, 0, st>>>(h);
        } else {
            h.v = act + ao[L - 1]; h.vt = v_target + r0;
            ppo2_dense_head_kernel<false><<<(B + 255) / 256, 256, 0, st>>>(h);
        }
        // backward: layer by layer from the top; chunk c's gradient into its slot
        float *slot = ws + w.slots + c * np;
        if (ppo2_chain_bwd_ok(d)) {
            // dH of every hidden layer in one data chain (into g1 / g2 / g3), then every layer's
            // dW | db partials in one launch and one reduce into the slot
            float *dh[3] = {ws + w.g1, ws + w.g2, ws + w.g3};  // dH1, dH2, dH3 (four layers)
            ChainBwdArgs cb{};
            cb.dy = ws + w.g0; cb.NO = A; cb.split3 = A; cb.W3 = cb.W3b = lw(L - 1);
            cb.W2 = lw(1); cb.W1 = lw(0); cb.K0 = S; cb.H1 = d.dims[1]; cb.H2 = d.dims[2]; cb.B = B;
            cb.h1 = act + ao[0]; cb.h2 = act + ao[1]; cb.d1 = dh[0]; cb.d2 = dh[1]; cb.hact = 1;
            if (L == 4) {
                cb.Wm = lw(2); cb.hm = act + ao[2]; cb.Hm = d.dims[3]; cb.dm = dh[2];
            }
            chain_bwd_launch(cb, cb, 1, st);
            Prob q[kMaxRegions];
            PartRegions pr{};
            int64_t po = 0;
            for (int l = 0; l < L; ++l) {
                const Layer Ly{lw(l), lb(l), d.dims[l], d.dims[l + 1]};
                const float *dyl = l == L - 1 ? ws + w.g0 : dh[l];
                const Opnd xin = l == 0 ? mat(s + r0 * S, B, S, S) : mat(act + ao[l - 1], B, Ly.in, Ly.in);
                Epi ew{};
                ew.y = ws + w.part + po; ew.kind = kEpiPartial; ew.M = Ly.out; ew.N = Ly.in + 1;
                Opnd xo = xin;
                xo.cols = Ly.in + 1;
                xo.ones = Ly.in;
                q[l] = make_prob_long(transposed(dyl, Ly.out, B, Ly.out), xo, ew, B, (int)ppo2_wgrad_nz(d, l));
                pr.part[l] = ws + w.part + po; pr.off[l] = off[l]; pr.z[l] = q[l].nz;
                pr.in[l] = Ly.in; pr.out[l] = Ly.out;
                po += ppo2_wgrad_nz(d, l) * Ly.out * (Ly.in + 1);
            }
            pr.n = L;
            gemm_multi(q, L, st);
            parts_reduce_kernel<<<(int)((np + 63) / 64), 64 * kWrSlices, 0, st>>>(slot, np, pr);
            continue;
        }
        const float *dy = ws + w.g0;
        float *dn = ws + w.g1;
        for (int l = L - 1; l >= 0; --l) {
            const Layer Ly{params + off[l], params + off[l] + (int64_t)d.dims[l] * d.dims[l + 1],
                           d.dims[l], d.dims[l + 1]};
            const Opnd xin = l == 0 ? mat(s + r0 * S, B, S, S) : mat(act + ao[l - 1], B, Ly.in, Ly.in);
            Epi ew{};
            ew.y = ws + w.part; ew.kind = kEpiPartial; ew.M = Ly.out; ew.N = Ly.in + 1;
            Opnd xo = xin;
            xo.cols = Ly.in + 1;
            xo.ones = Ly.in;
            const int tiles = ((Ly.in + 1 + kDT - 1) / kDT) * ((Ly.out + kDT - 1) / kDT);
            const Prob qw = make_prob_long(transposed(dy, Ly.out, B, Ly.out), xo, ew, B,
                                           512 / tiles > 1 ? 512 / tiles : 1);
            int z;
            if (l > 0) {  // dX = dY W, then (1 - h^2) with h = tanh output of layer l - 1
                const Prob qb = bwd_data_prob(dy, Ly, B, 0, Ly.in, kEpiTanhAffBack, act + ao[l - 1],
                                              Ly.in, ws + w.ones, dn);
                z = gemm_launch(qw, &qb, st);
            } else {
                z = gemm_launch(qw, nullptr, st);
            }
            wgrad_reduce(Ly, ws + w.part, z, slot + off[l], slot + off[l] + (int64_t)Ly.in * Ly.out, st);
            if (l > 0) {
                float *nx = dn == ws + w.g0 ? ws + w.g1 : ws + w.g0;
                dy = dn;
                dn = nx;
            }
        }
    }
    chunk_sum_kernel<<<(int)((np + 255) / 256), 256, 0, st>>>(ws + w.slots, (int)nchunks, np, grad);
    if (loss_sum)
        loss_sum_kernel<<<1, 256, 0, st>>>(reinterpret_cast<const double *>(ws + w.lpart),
                                           (rows + 255) / 256, loss_sum);
    RLP_CHECK_LAUNCH("rlp_ppo2_dense_grad");
    return RLP_OK;
}

}  // extern "C"
