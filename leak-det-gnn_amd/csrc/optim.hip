// The training step's tail (reference train_detector.py:313-317): clip_grad_norm_(max_norm)
// then AdamW.step(), as ONE launch.  The detector has ~60k parameters in ~20 tensors; torch
// runs the pair as ~11 launches (foreach norms, norm of norms, clamp, foreach mul, the fused
// AdamW), each a few microseconds of dispatch for almost no work.  Here the parameters are
// one flattened index space cut into kOptChunk-element slices, one 1024-thread workgroup each.
// Every workgroup first forms the WHOLE norm itself (thread i sums the squares of float4 i,
// i + 1024, ... of every tensor in fp64, then a fixed LDS tree: the same order in every
// workgroup, so every workgroup clips with the same bits; 242 KB of L2-resident gradients per
// workgroup, float4 loads 8 in flight — element-wise loads made the launch 30 us, r05d),
// then updates its slice:
//     g     = grad * min(1, max_norm / (||grad||_2 + 1e-6))     (written back, as torch does)
//     p    *= 1 - lr * weight_decay                              (decoupled decay)
//     m     = beta1 m + (1 - beta1) g,   v = beta2 v + (1 - beta2) g^2
//     p    -= lr / (1 - beta1^t) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
// The step counter t lives on the device (step[0]), so the step can live in a captured HIP
// graph.  Every workgroup reads step[0] BEFORE it takes a ticket (an agent-scope atomic on
// step[1], used as a uint32 counter); the workgroup that draws the launch's last ticket has
// therefore seen every other workgroup's read done, commits step[0] = t and resets the
// counter.  (Round 4 ran the norm as its own launch of per-slice partials: 6.7 + 9.8 us in the
// step for the pair.)
#include <algorithm>
#include "common.h"

namespace {

constexpr int kOptThreads = 1024;
constexpr int kOptChunk = kOptThreads;  // elements per workgroup (one per thread)
constexpr int kOptMaxTensors = 48;      // by-value kernel argument: a captured launch needs no host copy

struct AdamTensors {
    int64_t ptr[kOptMaxTensors][4];  // param, grad, exp_avg, exp_avg_sq
    int64_t off[kOptMaxTensors + 1];  // prefix offsets in the flattened index space
    int T;
    int vec;  // every gradient 16-byte aligned: the norm reads float4
};

// the next step's dropout seed slots (lg_clip_adamw_seeds): lg_seed_slots_advance's draw, by
// the launch's last workgroup
__device__ __forceinline__ uint64_t opt_splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
struct AdamSeeds {
    uint64_t* slots;
    uint64_t* state;
    int n;
};

__global__ void __launch_bounds__(kOptThreads)
k_adam(AdamTensors a, float* __restrict__ step, float lr, float beta1, float beta2, float eps, float wd,
       float max_norm, float* __restrict__ norm_out, AdamSeeds seeds) {
    __shared__ uint32_t last;
    __shared__ double red[kOptThreads];
    __shared__ float tsh;
    const int tid = threadIdx.x;
    // the committed step count, read before this workgroup's ticket (below)
    if (tid == 0) tsh = __hip_atomic_load(step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1.0f;
    // the whole norm: element i of the flattened space by thread i % kOptThreads, fixed order
    // float4 i of tensor t (its first n & ~3 elements) by thread i % 1024, then the tail elements
    // by threads 0..2; 8 loads in flight per round (242 KB of L2-resident gradients per workgroup)
    double ss = 0.0;
    if (max_norm > 0.f || norm_out) {
        for (int t = 0; t < a.T; ++t) {
            const float* g = reinterpret_cast<const float*>(a.ptr[t][1]);
            const int64_t n = a.off[t + 1] - a.off[t], n4 = n >> 2;
            const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
            if (!a.vec) {  // some gradient is not 16-byte aligned: element by element
                for (int64_t e = tid; e < n; e += kOptThreads) ss += static_cast<double>(g[e]) * g[e];
                continue;
            }
            int64_t j = tid;
            for (; j + 7 * kOptThreads < n4; j += 8 * kOptThreads) {
                f32x4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = g4[j + u * kOptThreads];
#pragma unroll
                for (int u = 0; u < 8; ++u)
#pragma unroll
                    for (int c = 0; c < 4; ++c) ss += static_cast<double>(v[u][c]) * v[u][c];
            }
            for (; j < n4; j += kOptThreads) {
                const f32x4 v = g4[j];
#pragma unroll
                for (int c = 0; c < 4; ++c) ss += static_cast<double>(v[c]) * v[c];
            }
            if (tid < (n & 3)) {
                const double x = g[4 * n4 + tid];
                ss += x * x;
            }
        }
    }
    red[tid] = ss;
    __syncthreads();
    for (int h = kOptThreads / 2; h > 0; h >>= 1) {
        if (tid < h) red[tid] += red[tid + h];
        __syncthreads();
    }
    const double norm = sqrt(red[0]);
    const float t1 = tsh;
    if (tid == 0) {
        // tsh was read above; the ticket is taken only after that read has returned
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        uint32_t* ctr = reinterpret_cast<uint32_t*>(step + 1);
        const uint32_t tk = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = tk + 1 == gridDim.x ? 1u : 0u;
        if (last) {  // every other workgroup has read step[0]: commit t
            __hip_atomic_store(step, t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (blockIdx.x == 0 && norm_out) norm_out[0] = static_cast<float>(norm);
    }
    if (seeds.slots) {  // the next step's dropout seeds: nothing in this launch reads them
        __syncthreads();
        if (last && tid < 64) {
            const uint64_t c = seeds.state[0] + 1;  // every lane reads before lane 0 writes (one wave)
            for (int i = tid; i < seeds.n; i += 64)
                seeds.slots[i] = opt_splitmix64(c * static_cast<uint64_t>(seeds.n) + static_cast<uint64_t>(i) + 1) &
                                 ((1ull << 62) - 1);
            if (tid == 0) seeds.state[0] = c;
        }
    }
    const float coef = max_norm > 0.f ? static_cast<float>(fmin(1.0, static_cast<double>(max_norm) / (norm + 1e-6)))
                                      : 1.0f;
    const float bc1 = 1.0f - powf(beta1, t1), bc2 = 1.0f - powf(beta2, t1);
    const float step_size = lr / bc1, bc2s = sqrtf(bc2), decay = 1.0f - lr * wd;
    const int64_t e = static_cast<int64_t>(blockIdx.x) * kOptChunk + tid;
    int t = 0;
    while (t < a.T && a.off[t + 1] <= e) ++t;
    if (t >= a.T) return;
    const int64_t i = e - a.off[t];
    float* p = reinterpret_cast<float*>(a.ptr[t][0]);
    float* g = reinterpret_cast<float*>(a.ptr[t][1]);
    float* m = reinterpret_cast<float*>(a.ptr[t][2]);
    float* v = reinterpret_cast<float*>(a.ptr[t][3]);
    float gi = g[i];
    if (max_norm > 0.f) {
        gi *= coef;
        g[i] = gi;
    }
    const float pi = p[i] * decay;
    const float mi = beta1 * m[i] + (1.0f - beta1) * gi;
    const float vi = beta2 * v[i] + (1.0f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi - step_size * mi / (sqrtf(vi) / bc2s + eps);
}

}  // namespace

extern "C" int64_t lg_clip_adamw_workspace_bytes(const int64_t* sizes, int T) {
    if (T < 0 || T > kOptMaxTensors || (T > 0 && !sizes)) return LG_EUNSUPPORTED;
    int64_t n = 0;
    for (int t = 0; t < T; ++t) n += std::max<int64_t>(sizes[t], 0);
    (void)n;
    return 8;  // unused since the single-launch form (kept: callers size and pass it)
}

namespace {
int clip_adamw_impl(const int64_t* table, const int64_t* sizes, int T, float* step, float lr, float beta1, float beta2,
                    float eps, float weight_decay, float max_norm, float* norm_out, void* workspace, int64_t ws_bytes,
                    const AdamSeeds& seeds, lg_stream_t stream) {
    if (T > kOptMaxTensors) return LG_EUNSUPPORTED;
    if (T < 0 || (T > 0 && (!table || !sizes)) || !step || !workspace) return LG_EINVAL;
    if (!(beta1 >= 0.f && beta1 < 1.f) || !(beta2 >= 0.f && beta2 < 1.f) || !(eps >= 0.f)) return LG_EINVAL;
    AdamTensors a{};
    a.off[0] = 0;
    for (int t = 0; t < T; ++t) {
        for (int j = 0; j < 4; ++j) {
            if (!table[4 * t + j]) return LG_EINVAL;
            a.ptr[t][j] = table[4 * t + j];
        }
        if (sizes[t] < 0) return LG_EINVAL;
        a.off[t + 1] = a.off[t] + sizes[t];
    }
    a.T = T;
    a.vec = 1;
    for (int t = 0; t < T; ++t) a.vec &= (a.ptr[t][1] % 16) == 0;
    const int G = static_cast<int>(std::max<int64_t>(1, (a.off[T] + kOptChunk - 1) / kOptChunk));
    if (ws_bytes < 8) return LG_EINVAL;  // the (unused) workspace keeps the sized-workspace contract
    lg_launch(k_adam, G, kOptThreads, 0, lg_stream(stream), a, step, lr, beta1, beta2, eps, weight_decay, max_norm,
              norm_out, seeds);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}
}  // namespace

extern "C" int lg_clip_adamw(const int64_t* table, const int64_t* sizes, int T, float* step, float lr, float beta1,
                             float beta2, float eps, float weight_decay, float max_norm, float* norm_out,
                             void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    return clip_adamw_impl(table, sizes, T, step, lr, beta1, beta2, eps, weight_decay, max_norm, norm_out, workspace,
                           ws_bytes, AdamSeeds{nullptr, nullptr, 0}, stream);
}

extern "C" int lg_clip_adamw_seeds(const int64_t* table, const int64_t* sizes, int T, float* step, float lr,
                                   float beta1, float beta2, float eps, float weight_decay, float max_norm,
                                   float* norm_out, void* workspace, int64_t ws_bytes, uint64_t* seed_slots,
                                   int64_t n_slots, uint64_t* seed_state, lg_stream_t stream) {
    if (n_slots < 0 || n_slots > 4096 || (n_slots > 0 && (!seed_slots || !seed_state))) return LG_EINVAL;
    return clip_adamw_impl(table, sizes, T, step, lr, beta1, beta2, eps, weight_decay, max_norm, norm_out, workspace,
                           ws_bytes, AdamSeeds{n_slots > 0 ? seed_slots : nullptr, seed_state, static_cast<int>(n_slots)},
                           stream);
}
