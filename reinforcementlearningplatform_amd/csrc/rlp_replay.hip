// rlp_replay.hip — the off-policy replay buffer resident in HBM (utils/classes.py:189-247
// ReplayBuffer, used by DDPG.learn algorithm/actor_critic/DDPG.py:72-109 and the DDPG-SOI driver
// demonstration/DDPG/DDPG-4-SecondOrderIntegration/train.py:167-251).
//
// Columns are separate device arrays of `capacity` rows (coalesced stores of one env batch per
// step, coalesced gathers of a sampled batch): s [cap][S], a [cap][A], r [cap], s_ [cap][S],
// end [cap] = 1 - done, all fp32 (the reference keeps float64 columns and converts to fp32 in
// learn(); the stored values are the converted ones).
#include <hipcub/hipcub.hpp>

#include "rlp_common.hpp"

namespace rlp {

// store_transition :201-210 for n transitions in order: row (counter + i) % capacity. Only the
// last min(n, capacity) can survive a sequential store, so only they are written (no races).
__global__ void replay_store_kernel(rlp_replay rb, int64_t counter, const float *__restrict__ s,
                                    const float *__restrict__ a, const double *__restrict__ r,
                                    const float *__restrict__ s_next,
                                    const uint8_t *__restrict__ done, int64_t i0, int64_t n) {
    const int S = rb.S, A = rb.A, W = 2 * S + A + 2;
    const int64_t total = (n - i0) * W;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + t / W;
        const int c = (int)(t % W);
        const int64_t row = (counter + i) % rb.capacity;
        if (c < S) rb.s[row * S + c] = s[i * S + c];
        else if (c < 2 * S) rb.s_next[row * S + (c - S)] = s_next[i * S + (c - S)];
        else if (c < 2 * S + A) rb.a[row * A + (c - 2 * S)] = a[i * A + (c - 2 * S)];
        else if (c == 2 * S + A) rb.r[row] = (float)r[i];
        else rb.end[row] = done[i] ? 0.f : 1.f;  // end_mem = 1 - done
    }
}

// np.random.choice(max_mem, batch) :237 — uniform with replacement, Philox-keyed
__global__ void replay_sample_uniform_kernel(int64_t max_mem, int64_t batch, uint64_t seed,
                                             uint64_t counter, int64_t *idx) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    double u[2];
    philox_u01_f64x2(seed, counter, (uint64_t)b, 0x300u, u);
    int64_t k = (int64_t)(u[0] * (double)max_mem);
    idx[b] = k < max_mem ? k : max_mem - 1;
}

__global__ void iota_kernel(int64_t *v, int64_t n, int64_t base) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = base + i;
}

__global__ void random_keys_kernel(const int64_t *__restrict__ pool, int64_t q, uint64_t seed,
                                   uint64_t counter, uint32_t *keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= q) return;
    uint32_t r4[4];
    philox_block(seed, counter, (uint64_t)pool[i], 0x301u, r4);
    keys[i] = r4[0];
}

__global__ void replay_gather_kernel(rlp_replay rb, const int64_t *__restrict__ idx, int64_t batch,
                                     float *s, float *a, float *r, float *s_next, float *end) {
    const int S = rb.S, A = rb.A, W = 2 * S + A + 2;
    const int64_t total = batch * W;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = t / W;
        const int c = (int)(t % W);
        const int64_t row = idx[b];
        if (c < S) s[b * S + c] = rb.s[row * S + c];
        else if (c < 2 * S) s_next[b * S + (c - S)] = rb.s_next[row * S + (c - S)];
        else if (c < 2 * S + A) a[b * A + (c - 2 * S)] = rb.a[row * A + (c - 2 * S)];
        else if (c == 2 * S + A) r[b] = rb.r[row];
        else end[b] = rb.end[row];
    }
}

static int grid_for(int64_t work) {
    int64_t b = (work + 255) / 256;
    return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

// bytes of hipCUB radix-sort scratch for q items (float keys / u32 keys, int64 values)
static size_t sort_temp_bytes(int64_t q) {
    size_t t1 = 0, t2 = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t1, (const float *)nullptr, (float *)nullptr,
                                             (const int64_t *)nullptr, (int64_t *)nullptr, (int)q);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t2, (const uint32_t *)nullptr,
                                             (uint32_t *)nullptr, (const int64_t *)nullptr,
                                             (int64_t *)nullptr, (int)q);
    return (t1 > t2 ? t1 : t2) + 256;
}

static int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }

}  // namespace rlp

using namespace rlp;

extern "C" {

int rlp_replay_store(const rlp_replay *rb, int64_t counter, const float *s, const float *a,
                     const double *reward, const float *s_next, const uint8_t *done, int64_t n,
                     rlp_stream_t stream) {
    RLP_REQUIRE(rb && rb->s && rb->a && rb->r && rb->s_next && rb->end && rb->capacity > 0 &&
                    rb->S >= 1 && rb->A >= 1,
                "rlp_replay_store: bad buffer");
    RLP_REQUIRE(counter >= 0 && n >= 0, "rlp_replay_store: counter=%lld n=%lld", (long long)counter,
                (long long)n);
    if (n == 0) return RLP_OK;
    RLP_REQUIRE(s && a && reward && s_next && done, "rlp_replay_store: null argument");
    const int64_t i0 = n > rb->capacity ? n - rb->capacity : 0;
    const int W = 2 * rb->S + rb->A + 2;
    replay_store_kernel<<<grid_for((n - i0) * W), 256, 0, as_stream(stream)>>>(
        *rb, counter, s, a, reward, s_next, done, i0, n);
    RLP_CHECK_LAUNCH("rlp_replay_store");
    return RLP_OK;
}

int rlp_replay_sample_uniform(int64_t max_mem, int64_t batch, uint64_t seed, uint64_t counter,
                              int64_t *index, rlp_stream_t stream) {
    RLP_REQUIRE(index && max_mem > 0 && batch >= 0, "rlp_replay_sample_uniform: bad argument");
    if (batch == 0) return RLP_OK;
    replay_sample_uniform_kernel<<<(int)((batch + 255) / 256), 256, 0, as_stream(stream)>>>(
        max_mem, batch, seed, counter, index);
    RLP_CHECK_LAUNCH("rlp_replay_sample_uniform");
    return RLP_OK;
}

int64_t rlp_replay_workspace_bytes(int64_t capacity) {
    if (capacity <= 0) return RLP_EINVAL;
    // sorted rewards (f32) + indices (2 x i64) + keys (2 x u32) + radix-sort scratch
    return align256(capacity * 4) * 2 + align256(capacity * 8) * 2 + align256(capacity * 4) * 2 +
           align256((int64_t)sort_temp_bytes(capacity));
}

int rlp_replay_sample_reward_top(const rlp_replay *rb, int64_t max_mem, int64_t batch,
                                 uint64_t seed, uint64_t counter, int64_t *index, int64_t *n_out,
                                 void *workspace, int64_t workspace_bytes, rlp_stream_t stream) {
    RLP_REQUIRE(rb && rb->r && index && n_out && workspace, "rlp_replay_sample_reward_top: null");
    RLP_REQUIRE(max_mem > 0 && max_mem <= rb->capacity && batch >= 0,
                "rlp_replay_sample_reward_top: max_mem=%lld", (long long)max_mem);
    RLP_REQUIRE(workspace_bytes >= rlp_replay_workspace_bytes(max_mem),
                "rlp_replay_sample_reward_top: workspace too small");
    const int64_t q = (int64_t)(0.25 * (double)max_mem);  // int(0.25 * max_mem)
    const int64_t nb = q < batch ? q : batch;              // batchNum
    *n_out = nb;
    if (nb == 0) return RLP_OK;
    hipStream_t st = as_stream(stream);
    char *w = static_cast<char *>(workspace);
    float *rk_out = reinterpret_cast<float *>(w);
    w += align256(max_mem * 4);
    w += align256(max_mem * 4);  // (kept for layout symmetry)
    int64_t *iv_in = reinterpret_cast<int64_t *>(w);
    w += align256(max_mem * 8);
    int64_t *iv_out = reinterpret_cast<int64_t *>(w);
    w += align256(max_mem * 8);
    uint32_t *k_in = reinterpret_cast<uint32_t *>(w);
    w += align256(max_mem * 4);
    uint32_t *k_out = reinterpret_cast<uint32_t *>(w);
    w += align256(max_mem * 4);
    void *temp = w;
    size_t temp_bytes = sort_temp_bytes(max_mem);
    // get_reward_sort :212-217: ascending, stable (radix sort is stable; ties keep index order)
    iota_kernel<<<(int)((max_mem + 255) / 256), 256, 0, st>>>(iv_in, max_mem, 0);
    if (hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, rb->r, rk_out, iv_in, iv_out,
                                           (int)max_mem, 0, 32, st) != hipSuccess)
        return fail(RLP_EINVAL, "rlp_replay_sample_reward_top: sort");
    // random.sample(sorted_index[-q:], batchNum): a uniformly random order of the top-q pool
    // (Philox key per pool entry, sorted) and its first batchNum entries
    const int64_t *pool = iv_out + (max_mem - q);
    random_keys_kernel<<<(int)((q + 255) / 256), 256, 0, st>>>(pool, q, seed, counter, k_in);
    int64_t *perm = iv_in;  // reuse
    if (hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k_in, k_out, pool, perm, (int)q, 0, 32,
                                           st) != hipSuccess)
        return fail(RLP_EINVAL, "rlp_replay_sample_reward_top: shuffle");
    if (hipMemcpyAsync(index, perm, nb * sizeof(int64_t), hipMemcpyDeviceToDevice, st) !=
        hipSuccess)
        return fail(RLP_EINVAL, "rlp_replay_sample_reward_top: copy");
    RLP_CHECK_LAUNCH("rlp_replay_sample_reward_top");
    return RLP_OK;
}

int rlp_replay_gather(const rlp_replay *rb, const int64_t *index, int64_t batch, float *s,
                      float *a, float *r, float *s_next, float *end, rlp_stream_t stream) {
    RLP_REQUIRE(rb && index && s && a && r && s_next && end && batch >= 0,
                "rlp_replay_gather: null argument");
    if (batch == 0) return RLP_OK;
    const int W = 2 * rb->S + rb->A + 2;
    replay_gather_kernel<<<grid_for(batch * W), 256, 0, as_stream(stream)>>>(*rb, index, batch, s,
                                                                             a, r, s_next, end);
    RLP_CHECK_LAUNCH("rlp_replay_gather");
    return RLP_OK;
}

}  // extern "C"
