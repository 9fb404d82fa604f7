// The training step's tail (reference train_detector.py:313-317): clip_grad_norm_(max_norm)
// then AdamW.step(), as TWO launches.  The detector has ~60k parameters in ~20 tensors; torch
// runs the pair as ~11 launches (foreach norms, norm of norms, clamp, foreach mul, the fused
// AdamW), each a few microseconds of dispatch for almost no work.  Here the parameters are
// one flattened index space cut into kOptChunk-element slices, one workgroup each:
//   launch 1: per-slice sums of squared gradients (fp64, fixed order) -> partial[G]
//   launch 2: every workgroup sums partial[0..G) in the same fixed order, forms
//     g     = grad * min(1, max_norm / (||grad||_2 + 1e-6))     (written back, as torch does)
//     p    *= 1 - lr * weight_decay                              (decoupled decay)
//     m     = beta1 m + (1 - beta1) g,   v = beta2 v + (1 - beta2) g^2
//     p    -= lr / (1 - beta1^t) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
//   for its slice.  t lives on the device (step[0]; launch 1 stages t + 1 in step[1], launch 2
//   reads it and commits it), so the step can live in a captured HIP graph.
#include <algorithm>
#include "common.h"

namespace {

constexpr int kOptThreads = 256;
constexpr int kOptChunk = 512;       // elements per workgroup (two per thread: one round trip)
constexpr int kOptMaxTensors = 48;   // by-value kernel argument: a captured launch needs no host copy

struct AdamTensors {
    int64_t ptr[kOptMaxTensors][4];  // param, grad, exp_avg, exp_avg_sq
    int64_t off[kOptMaxTensors + 1];  // prefix offsets in the flattened index space
    int T;
};

// visit f(tensor, index) for the flattened indices [lo, hi) of this workgroup, thread-strided
template <typename F>
__device__ __forceinline__ void for_slice(const AdamTensors& a, int64_t lo, int64_t hi, F&& f) {
    for (int t = 0; t < a.T; ++t) {
        const int64_t b0 = max(lo, a.off[t]), b1 = min(hi, a.off[t + 1]);
        for (int64_t i = b0 + threadIdx.x; i < b1; i += kOptThreads) f(t, i - a.off[t]);
    }
}

__device__ __forceinline__ double block_sum(double x) {
    __shared__ double red[kOptThreads];
    red[threadIdx.x] = x;
    __syncthreads();
    for (int h = kOptThreads / 2; h > 0; h >>= 1) {
        if (static_cast<int>(threadIdx.x) < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}

__global__ void __launch_bounds__(kOptThreads) k_adam_norm(AdamTensors a, double* __restrict__ partial,
                                                           float* __restrict__ step) {
    const int64_t lo = static_cast<int64_t>(blockIdx.x) * kOptChunk, hi = lo + kOptChunk;
    double ss = 0.0;
    for_slice(a, lo, hi, [&](int t, int64_t i) {
        const double x = reinterpret_cast<const float*>(a.ptr[t][1])[i];
        ss += x * x;
    });
    ss = block_sum(ss);
    if (threadIdx.x == 0) {
        partial[blockIdx.x] = ss;
        if (blockIdx.x == 0) step[1] = step[0] + 1.0f;
    }
}

__global__ void __launch_bounds__(kOptThreads)
k_adam_update(AdamTensors a, const double* __restrict__ partial, int G, float* __restrict__ step, float lr,
              float beta1, float beta2, float eps, float wd, float max_norm, float* __restrict__ norm_out) {
    double ss = 0.0;
    for (int g = threadIdx.x; g < G; g += kOptThreads) ss += partial[g];
    const double norm = sqrt(block_sum(ss));
    const float coef = max_norm > 0.f ? static_cast<float>(fmin(1.0, static_cast<double>(max_norm) / (norm + 1e-6)))
                                      : 1.0f;
    const float t1 = step[1];
    const float bc1 = 1.0f - powf(beta1, t1), bc2 = 1.0f - powf(beta2, t1);
    const float step_size = lr / bc1, bc2s = sqrtf(bc2), decay = 1.0f - lr * wd;
    const int64_t lo = static_cast<int64_t>(blockIdx.x) * kOptChunk, hi = lo + kOptChunk;
    for_slice(a, lo, hi, [&](int t, int64_t i) {
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
    });
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        step[0] = t1;  // step[1] stays t1: no workgroup of this launch writes what another reads
        if (norm_out) norm_out[0] = static_cast<float>(norm);
    }
}

}  // namespace

extern "C" int64_t lg_clip_adamw_workspace_bytes(const int64_t* sizes, int T) {
    if (T < 0 || T > kOptMaxTensors || (T > 0 && !sizes)) return LG_EUNSUPPORTED;
    int64_t n = 0;
    for (int t = 0; t < T; ++t) n += std::max<int64_t>(sizes[t], 0);
    return std::max<int64_t>(1, (n + kOptChunk - 1) / kOptChunk) * static_cast<int64_t>(sizeof(double));
}

extern "C" int lg_clip_adamw(const int64_t* table, const int64_t* sizes, int T, float* step, float lr, float beta1,
                             float beta2, float eps, float weight_decay, float max_norm, float* norm_out,
                             void* workspace, int64_t ws_bytes, lg_stream_t stream) {
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
    const int G = static_cast<int>(std::max<int64_t>(1, (a.off[T] + kOptChunk - 1) / kOptChunk));
    if (ws_bytes < G * static_cast<int64_t>(sizeof(double))) return LG_EINVAL;  // one fp64 partial per slice
    double* partial = static_cast<double*>(workspace);
    hipStream_t s = lg_stream(stream);
    lg_launch(k_adam_norm, G, kOptThreads, 0, s, a, partial, step);
    LG_RET_IF_LAUNCH_FAILED();
    lg_launch(k_adam_update, G, kOptThreads, 0, s, a, partial, G, step, lr, beta1, beta2, eps, weight_decay, max_norm,
              norm_out);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}
