// K10 global_mean_pool + NoLeakHead (reference detector.py:91-102, 214-216), fused.
//
// Forward, one 1024-thread workgroup per window b:
//   pooled[b] = (1/N) sum_n x[b][n]        16 lanes per row (D = 64), 64 row groups
//                                          striding the window, fixed-order LDS fold
//   hid[b]    = dropout(relu(pooled[b] W1^T + b1))      one thread per hidden unit
//   logits[b * ldo + col] = hid[b] . w2 + b2            fixed-order LDS tree
// so the (B, P+1) logits of detector.py:216 are written in place (no torch.cat) and
// the NoLeakHead's four tiny GEMMs never reach hipBLASLt.
// Backward, windows dealt to a persistent grid: dhid = dlogit * w2 * scale * [hid > 0]
// (ReLU and the dropout mask read back from the saved hid), dpooled = dhid W1 (fed to
// lg_pipe_scatter_bwd, which adds dpooled / N to every node row), and per-block
// dW1 / db1 / dw2 partials plus an fp64 db2 partial, reduced in fixed order.
#include <algorithm>
#include "common.h"
#include "reduce.h"

namespace {

constexpr int kPoolThreads = 1024;
constexpr int kHid = 128;

// pooled_lds[d] = mean over the N rows of window b (all threads participate).  Row of
// (window b, node n) = b * sb + n * sn: (N, 1) window-major, (1, B) node-major.
template <int D>
__device__ __forceinline__ void pool_window(const float* __restrict__ x, int64_t b, int64_t N, int64_t sb, int64_t sn,
                                            f32x4* __restrict__ part, float* __restrict__ pooled_lds) {
    constexpr int LPR = D / 4, G = kPoolThreads / LPR;
    const int g = threadIdx.x / LPR, fg = threadIdx.x % LPR;
    const float* xb = x + b * sb * D + 4 * fg;
    const int64_t step = sn * D;
    f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
    int64_t n = g;
    for (; n + G < N; n += 2 * G) {  // two independent loads in flight per lane
        a0 += ld4(xb + n * step);
        a1 += ld4(xb + (n + G) * step);
    }
    if (n < N) a0 += ld4(xb + n * step);
    part[threadIdx.x] = a0 + a1;
    __syncthreads();
    if (threadIdx.x < D) {
        const int d = threadIdx.x, f = d / 4, i = d % 4;
        float s = 0.f;
        for (int gg = 0; gg < G; ++gg) s += part[gg * LPR + f][i];
        pooled_lds[d] = s / static_cast<float>(N);
    }
    __syncthreads();
}

template <int D>
__global__ void __launch_bounds__(kPoolThreads) k_mean_pool(const float* __restrict__ x, float* __restrict__ out,
                                                            int64_t N) {
    __shared__ f32x4 part[kPoolThreads];
    __shared__ float pooled[D];
    const int64_t b = blockIdx.x;
    pool_window<D>(x, b, N, N, 1, part, pooled);
    if (threadIdx.x < D) out[b * D + threadIdx.x] = pooled[threadIdx.x];
}

template <int D, bool DROP>
__global__ void __launch_bounds__(kPoolThreads)
k_pool_head_fwd(const float* __restrict__ x, const float* __restrict__ W1, const float* __restrict__ b1,
                const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ pooled_out,
                float* __restrict__ hid_out, float* __restrict__ logits, int64_t ldo, int64_t col, int64_t N,
                int64_t sb, int64_t sn, float p_drop, float dscale, uint64_t seed, uint32_t salt) {
    __shared__ f32x4 part[kPoolThreads];
    __shared__ float pooled[D];
    __shared__ float red[kHid];
    const int64_t b = blockIdx.x;
    pool_window<D>(x, b, N, sb, sn, part, pooled);
    const int t = threadIdx.x;
    if (t < D) pooled_out[b * D + t] = pooled[t];
    if (t < kHid) {
        float pre = b1[t];
#pragma unroll 8
        for (int d = 0; d < D; ++d) pre = fmaf(W1[t * D + d], pooled[d], pre);
        float v = fmaxf(pre, 0.f);
        if constexpr (DROP) v = lg_dropout(v, p_drop, dscale, lg_dropout_key_dev(seed, salt), b * kHid + t);
        hid_out[b * kHid + t] = v;
        red[t] = v * w2[t];
    }
    __syncthreads();
    for (int h = kHid / 2; h > 0; h >>= 1) {
        if (t < h) red[t] += red[t + h];
        __syncthreads();
    }
    if (t == 0) logits[b * ldo + col] = red[0] + b2[0];
}

// slab per workgroup: [dW1 kHid*D][db1 kHid][dw2 kHid]; dslab: db2 partial (fp64)
template <int D>
__global__ void __launch_bounds__(kHid)
k_pool_head_bwd(const float* __restrict__ pooled, const float* __restrict__ hid, const float* __restrict__ W1,
                const float* __restrict__ w2, const float* __restrict__ dlogits, int64_t ldo, int64_t col,
                float* __restrict__ dpooled, float* __restrict__ slab, double* __restrict__ dslab, int64_t B,
                float scale) {
    constexpr int SL = kHid * D + 2 * kHid;
    constexpr int WS = D + 1;  // W1 / dW1 rows in LDS (odd stride: conflict-free row-per-thread access)
    __shared__ float w1l[kHid * WS];
    __shared__ float pl[D];
    __shared__ float dh[kHid];
    const int k = threadIdx.x;
    for (int i = k; i < kHid * D; i += kHid) w1l[(i / D) * WS + (i % D)] = W1[i];
    const float w2k = w2[k];
    float dw1[D];
#pragma unroll
    for (int d = 0; d < D; ++d) dw1[d] = 0.f;
    float db1 = 0.f, dw2 = 0.f;
    double db2 = 0.0;
    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        const float dout = dlogits[b * ldo + col];
        const float hk = hid[b * kHid + k];
        if (k < D) pl[k] = pooled[b * D + k];
        const float dhk = hk > 0.f ? dout * w2k * scale : 0.f;
        dh[k] = dhk;
        db1 += dhk;
        dw2 = fmaf(dout, hk, dw2);
        if (k == 0) db2 += static_cast<double>(dout);
        __syncthreads();  // pl, dh (and on the first pass w1l) visible
#pragma unroll
        for (int d = 0; d < D; ++d) dw1[d] = fmaf(dhk, pl[d], dw1[d]);
        if (k < D) {
            float s = 0.f;
#pragma unroll 16
            for (int kk = 0; kk < kHid; ++kk) s = fmaf(dh[kk], w1l[kk * WS + k], s);
            dpooled[b * D + k] = s;
        }
        __syncthreads();
    }
    // dW1 rows through LDS (reusing the W1 copy) so the slab store is coalesced
#pragma unroll
    for (int d = 0; d < D; ++d) w1l[k * WS + d] = dw1[d];
    __syncthreads();
    float* out = slab + static_cast<int64_t>(blockIdx.x) * SL;
    for (int i = k; i < kHid * D; i += kHid) out[i] = w1l[(i / D) * WS + (i % D)];
    out[kHid * D + k] = db1;
    out[kHid * D + kHid + k] = dw2;
    if (k == 0) dslab[blockIdx.x] = db2;
}

int pool_bwd_grid(int64_t B) {
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(B, 2LL * lg_num_cus())));
}

}  // namespace

extern "C" int lg_mean_pool_fwd(const float* x, float* out, int64_t B, int64_t N, int64_t D, lg_stream_t stream) {
    if (B < 0 || N <= 0) return LG_EINVAL;
    if (B == 0) return LG_OK;
    if (!x || !out || B > INT32_MAX) return LG_EINVAL;
    hipStream_t s = lg_stream(stream);
    switch (D) {
        case 64: lg_launch(k_mean_pool<64>, static_cast<unsigned>(B), kPoolThreads, 0, s, x, out, N); break;
        case 32: lg_launch(k_mean_pool<32>, static_cast<unsigned>(B), kPoolThreads, 0, s, x, out, N); break;
        default: return LG_EUNSUPPORTED;
    }
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_pool_head_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                                float* pooled, float* hid, float* logits, int64_t ldo, int64_t col, int64_t B,
                                int64_t N, int64_t D, int64_t hidden, int flags, float dropout_p, uint64_t seed,
                                uint32_t salt, lg_stream_t stream) {
    if (B < 0 || N <= 0 || col < 0 || ldo <= col) return LG_EINVAL;
    if (hidden != kHid || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const bool drop = (flags & LG_F_DROPOUT) != 0;
    if (drop && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (B == 0) return LG_OK;
    if (!x || !w1 || !b1 || !w2 || !b2 || !pooled || !hid || !logits || B > INT32_MAX) return LG_EINVAL;
    const float scale = drop ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
    const unsigned grid = static_cast<unsigned>(B);
    const bool nm = (flags & LG_F_NODE_MAJOR) != 0;  // x is [N][B][D] instead of [B][N][D]
    const int64_t sb = nm ? 1 : N, sn = nm ? B : 1;
#define LG_PH(DD, DR)                                                                                             \
    lg_launch(k_pool_head_fwd<DD, DR>, grid, kPoolThreads, 0, s, x, w1, b1, w2, b2, pooled, hid, logits, ldo, col, N,    \
                                                           sb, sn, dropout_p, scale, seed, salt)
    if (D == 64) {
        if (drop) LG_PH(64, true); else LG_PH(64, false);
    } else {
        if (drop) LG_PH(32, true); else LG_PH(32, false);
    }
#undef LG_PH
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int64_t lg_pool_head_bwd_workspace_bytes(int64_t B, int64_t D, int64_t hidden) {
    if (B < 0 || hidden != kHid || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const int64_t G = pool_bwd_grid(B);
    return ((G * (kHid * D + 2 * kHid) * 4 + 255) & ~int64_t(255)) + G * 8;
}

extern "C" int lg_pool_head_bwd(const float* pooled, const float* hid, const float* w1, const float* w2,
                                const float* dlogits, int64_t ldo, int64_t col, float* dpooled, float* dw1,
                                float* db1, float* dw2, float* db2, int64_t B, int64_t D, int64_t hidden, int flags,
                                float dropout_p, void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    if (B < 0 || col < 0 || ldo <= col) return LG_EINVAL;
    if (hidden != kHid || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const bool drop = (flags & LG_F_DROPOUT) != 0;
    if (drop && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (!w1 || !w2 || !dw1 || !db1 || !dw2 || !db2 || !workspace) return LG_EINVAL;
    if (B > 0 && (!pooled || !hid || !dlogits || !dpooled)) return LG_EINVAL;
    const float scale = drop ? 1.0f / (1.0f - dropout_p) : 1.0f;
    const int G = pool_bwd_grid(B);
    const int64_t SL = kHid * D + 2 * kHid;
    if (ws_bytes < ((G * SL * 4 + 255) & ~int64_t(255)) + G * 8) return LG_EINVAL;
    float* slab = static_cast<float*>(workspace);
    double* dslab = reinterpret_cast<double*>(static_cast<char*>(workspace) + ((G * SL * 4 + 255) & ~int64_t(255)));
    hipStream_t s = lg_stream(stream);
    if (B == 0) {
        if (hipMemsetAsync(slab, 0, SL * G * sizeof(float), s) != hipSuccess) return LG_EHIP;
        if (hipMemsetAsync(dslab, 0, G * sizeof(double), s) != hipSuccess) return LG_EHIP;
    } else if (D == 64) {
        lg_launch(k_pool_head_bwd<64>, G, kHid, 0, s, pooled, hid, w1, w2, dlogits, ldo, col, dpooled, slab, dslab, B, scale);
    } else {
        lg_launch(k_pool_head_bwd<32>, G, kHid, 0, s, pooled, hid, w1, w2, dlogits, ldo, col, dpooled, slab, dslab, B, scale);
    }
    LG_RET_IF_LAUNCH_FAILED();
    const LgSlabSeg segs[3] = {{0, kHid * D, dw1}, {kHid * D, kHid, db1}, {kHid * D + kHid, kHid, dw2}};
    return lg_launch_slab_reduce_multi(slab, G, SL, segs, 3, dslab, db2, s);
}
