// The training loss (reference train_detector.py:235, 311: nn.CrossEntropyLoss(), mean
// reduction, ignore_index -100) over the (B, P+1) logits, forward and backward.  torch runs
// it as six launches (log_softmax, nll forward, two fills, nll backward, log_softmax
// backward); here:
//   forward : one wave per row: lse = max + log(sum exp(x - max)) (fp32, fixed lane order
//             then a fixed shuffle tree), row loss = lse - x[target] -> lse[b], rowloss[b];
//             the workgroup that finishes last sums the counted rows in row order
//             (deterministic), in the same launch.  The hand-off is fence-free
//             (MI355X_MICROARCH.md, the sc1 hand-off table's first row): the row losses are
//             stored sc1 (agent-scope relaxed atomic stores, 4 B), every wave waits for its
//             stores (vmcnt 0), then behind a workgroup barrier one lane adds to the counter
//             (agent scope); the workgroup whose add returns gridDim - 1 reads the row losses
//             with sc1 loads and resets the counter.  (Round 3 took the mean behind a release /
//             acquire fence pair: on gfx950 that is an L2 writeback + invalidate in every
//             workgroup — buffer_wbl2 / buffer_inv — which, right after the EdgeHead forward's
//             100 MB of stores, made the launch 12 us for 0.8 MB of logits; round 4 ran the
//             mean as a second, single-wave launch, ~5 us in the step.)
//   backward: dx[b][c] = g / n * (exp(x - lse[b]) - [c == target[b]])   (0 for ignored rows)
#include <algorithm>
#include "common.h"

namespace {

constexpr int kCeWaves = 4;
constexpr int kCeThreads = 64 * kCeWaves;
constexpr int kCePer = 16;  // row elements per lane held in registers (C <= 1024)

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// the mean over the counted rows, in row order (one wave; sc1 loads: the rows were stored sc1
// by other workgroups of the same launch)
__device__ __forceinline__ void ce_mean_wave(float* rowloss, const int64_t* __restrict__ target, int64_t B,
                                             int64_t ignore, float* __restrict__ loss) {
    const int lane = threadIdx.x & 63;
    float acc = 0.f, cnt = 0.f;
    for (int64_t b0 = 0; b0 < B; b0 += 64) {
        const int64_t b = b0 + lane;
        float v = 0.f, c = 0.f;
        if (b < B) {
            v = __hip_atomic_load(rowloss + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            c = target[b] == ignore ? 0.f : 1.f;
        }
        acc += wave_sum(v);
        cnt += wave_sum(c);
    }
    if (lane == 0) loss[0] = acc / cnt;  // NaN when every row is ignored, as torch
}

__global__ void __launch_bounds__(kCeThreads)
k_ce_fwd(const float* __restrict__ x, const int64_t* __restrict__ target, int64_t B, int64_t C, int64_t ldx,
         int64_t ignore, float* __restrict__ lse, float* rowloss, unsigned* counter, float* __restrict__ loss) {
    __shared__ unsigned is_last;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int64_t b = static_cast<int64_t>(blockIdx.x) * kCeWaves + w; b < B; b += static_cast<int64_t>(gridDim.x) * kCeWaves) {
        const float* row = x + b * ldx;
        float m = -__builtin_huge_valf(), s = 0.f;
        if (C <= 64 * kCePer) {  // the whole row in registers: every load in flight at once
            float v[kCePer];
#pragma unroll
            for (int k = 0; k < kCePer; ++k) {
                const int64_t c = lane + 64 * k;
                v[k] = c < C ? row[c] : -__builtin_huge_valf();
            }
#pragma unroll
            for (int k = 0; k < kCePer; ++k) m = fmaxf(m, v[k]);
            m = wave_max(m);
#pragma unroll
            for (int k = 0; k < kCePer; ++k) s += lane + 64 * k < C ? expf(v[k] - m) : 0.f;
        } else {
            for (int64_t c = lane; c < C; c += 64) m = fmaxf(m, row[c]);
            m = wave_max(m);
            for (int64_t c = lane; c < C; c += 64) s += expf(row[c] - m);
        }
        s = wave_sum(s);
        const float l = m + logf(s);
        if (lane == 0) {
            const int64_t t = target[b];
            lse[b] = l;
            // a target outside [0, C) (torch raises) poisons the loss with NaN, never reads out of bounds
            const float rl = t == ignore ? 0.f : (t >= 0 && t < C ? l - row[t] : __builtin_nanf(""));
            __hip_atomic_store(rowloss + b, rl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's row losses have left
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = old + 1 == gridDim.x ? 1u : 0u;
    }
    __syncthreads();
    if (!is_last) return;
    if (w == 0) ce_mean_wave(rowloss, target, B, ignore, loss);
    if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(kCeThreads)
k_ce_bwd(const float* __restrict__ x, const int64_t* __restrict__ target, const float* __restrict__ lse,
         const float* __restrict__ gout, int64_t B, int64_t C, int64_t ldx, int64_t ignore, float* __restrict__ dx,
         int64_t ldd) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // n = counted rows (every workgroup counts them the same way)
    float cnt = 0.f;
    for (int64_t b0 = 0; b0 < B; b0 += 64) {
        const int64_t b = b0 + lane;
        cnt += wave_sum((b < B && target[b] != ignore) ? 1.f : 0.f);
    }
    const float g = gout[0] / cnt;
    for (int64_t b = static_cast<int64_t>(blockIdx.x) * kCeWaves + w; b < B; b += static_cast<int64_t>(gridDim.x) * kCeWaves) {
        const float* row = x + b * ldx;
        float* drow = dx + b * ldd;
        const int64_t t = target[b];
        const float l = lse[b];
        const float gi = t == ignore ? 0.f : g;
        if (C <= 64 * kCePer) {
            float v[kCePer];
#pragma unroll
            for (int k = 0; k < kCePer; ++k) {
                const int64_t c = lane + 64 * k;
                v[k] = c < C ? row[c] : 0.f;
            }
#pragma unroll
            for (int k = 0; k < kCePer; ++k) {
                const int64_t c = lane + 64 * k;
                if (c < C) drow[c] = gi * (expf(v[k] - l) - (c == t ? 1.f : 0.f));
            }
        } else {
            for (int64_t c = lane; c < C; c += 64) drow[c] = gi * (expf(row[c] - l) - (c == t ? 1.f : 0.f));
        }
    }
}

}  // namespace

extern "C" int lg_cross_entropy_fwd(const float* logits, const int64_t* target, int64_t B, int64_t C, int64_t ldx,
                                    int64_t ignore_index, float* loss, float* lse, float* rowloss, unsigned* counter,
                                    lg_stream_t stream) {
    if (B < 0 || C <= 0 || ldx < C || !loss || !counter) return LG_EINVAL;
    hipStream_t s = lg_stream(stream);
    if (B == 0) {  // the mean over no rows is NaN (torch); a memset node, so the call stays capturable
        return hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(loss), 0x7FC00000, 1, s) == hipSuccess ? LG_OK
                                                                                                          : LG_EHIP;
    }
    if (!logits || !target || !lse || !rowloss) return LG_EINVAL;
    // at most one workgroup per CU: the sc1 hand-off above was measured in that configuration
    // at most one workgroup per CU: every workgroup of the launch is co-resident, so the last
    // ticket is taken only after every workgroup's row losses have left (the fence-free
    // hand-off above was validated at this grid; larger B loops inside the workgroups,
    // tests/test_gpu_library.py::test_cross_entropy_matches_torch at B = 65,536)
    const int grid = static_cast<int>(std::min<int64_t>((B + kCeWaves - 1) / kCeWaves, lg_num_cus()));
    lg_launch(k_ce_fwd, grid, kCeThreads, 0, s, logits, target, B, C, ldx, ignore_index, lse, rowloss, counter, loss);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_cross_entropy_bwd(const float* logits, const int64_t* target, const float* lse,
                                    const float* grad_loss, int64_t B, int64_t C, int64_t ldx, int64_t ignore_index,
                                    float* dlogits, int64_t ldd, lg_stream_t stream) {
    if (B < 0 || C <= 0 || ldx < C || ldd < C || !grad_loss) return LG_EINVAL;
    if (B == 0) return LG_OK;
    if (!logits || !target || !lse || !dlogits) return LG_EINVAL;
    hipStream_t s = lg_stream(stream);
    const int grid = static_cast<int>(std::min<int64_t>((B + kCeWaves - 1) / kCeWaves, 4 * lg_num_cus()));
    lg_launch(k_ce_bwd, grid, kCeThreads, 0, s, logits, target, lse, grad_loss, B, C, ldx, ignore_index, dlogits, ldd);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}
