// Deterministic slab reduction shared by the backward kernels:
//   seg k:  out_k[i] = sum_g slab[g * stride + off_k + i],  i < len_k
// in a fixed order, all segments of one backward op in ONE launch, accumulated in fp64
// (the bias gradients are sums with heavy cancellation over hundreds of block partials;
// fp32 accumulation left them ~2e-5 of scale off at B = 256).  One 1024-thread
// block per 64 columns of a segment: wave w sums slabs g = w, w + 16, ... for its
// column (one column per lane, coalesced rows), then the 16 wave partials are added
// in wave order through LDS.  An optional fp64 column (sum of G doubles, used for
// the cancellation-heavy output-bias gradients) is reduced by one extra block as a
// fixed-shape tree.  Per-column work and the combine order depend only on (G, len),
// never on scheduling.
#include "common.h"
#include "reduce.h"

namespace {

struct Segs {
    int64_t off[kLgMaxSlabSegs];
    int64_t len[kLgMaxSlabSegs];
    float* out[kLgMaxSlabSegs];
    int first[kLgMaxSlabSegs + 1];  // first block of each segment; first[n] = total column blocks
    int n;
};

__global__ void __launch_bounds__(1024) k_slab_reduce(const float* __restrict__ slab, int G, int64_t stride, Segs sg,
                                                      const double* __restrict__ dslab, float* __restrict__ dout) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int b = blockIdx.x;
    if (b >= sg.first[sg.n]) {  // fp64 column: 1024 strided partials, then a fixed tree
        __shared__ double dp[1024];
        double acc = 0.0;
        for (int g = threadIdx.x; g < G; g += 1024) acc += dslab[g];
        dp[threadIdx.x] = acc;
        __syncthreads();
        for (int h = 512; h > 0; h >>= 1) {
            if (threadIdx.x < h) dp[threadIdx.x] += dp[threadIdx.x + h];
            __syncthreads();
        }
        if (threadIdx.x == 0) dout[0] = static_cast<float>(dp[0]);
        return;
    }
    int k = 0;
    while (k + 1 < sg.n && b >= sg.first[k + 1]) ++k;
    const int64_t col = static_cast<int64_t>(b - sg.first[k]) * 64 + lane;
    const int64_t len = sg.len[k];
    const float* src = slab + sg.off[k];
    __shared__ double part[16][64];
    double acc = 0.0;
    if (col < len) {
        // slabs g = w, w + 16, ... added in that order; kRedInflight independent loads per
        // round trip (a 512-slab reduce is 2 round trips per wave instead of 8)
        constexpr int kRedInflight = 16;
        int g = w;
        for (; g + 16 * (kRedInflight - 1) < G; g += 16 * kRedInflight) {
            float v[kRedInflight];
#pragma unroll
            for (int u = 0; u < kRedInflight; ++u) v[u] = src[static_cast<int64_t>(g + 16 * u) * stride + col];
#pragma unroll
            for (int u = 0; u < kRedInflight; ++u) acc += v[u];
        }
        for (; g < G; g += 16) acc += src[static_cast<int64_t>(g) * stride + col];
    }
    part[w][lane] = acc;
    __syncthreads();
    if (w == 0 && col < len) {
        double s = part[0][lane];
        for (int i = 1; i < 16; ++i) s += part[i][lane];
        sg.out[k][col] = static_cast<float>(s);
    }
}

}  // namespace

int lg_launch_slab_reduce_multi(const float* slab, int G, int64_t stride, const LgSlabSeg* segs, int nseg,
                                const double* dslab, float* dout, hipStream_t s) {
    if (nseg < 0 || nseg > kLgMaxSlabSegs || G < 0 || (dslab && !dout)) return LG_EINVAL;
    Segs sg{};
    int blocks = 0, n = 0;
    for (int i = 0; i < nseg; ++i) {
        if (segs[i].out == nullptr || segs[i].len <= 0) continue;
        sg.off[n] = segs[i].off;
        sg.len[n] = segs[i].len;
        sg.out[n] = segs[i].out;
        sg.first[n] = blocks;
        blocks += static_cast<int>((segs[i].len + 63) / 64);
        ++n;
    }
    sg.first[n] = blocks;
    sg.n = n;
    const int total = blocks + (dslab ? 1 : 0);
    if (total == 0) return LG_OK;
    k_slab_reduce<<<total, 1024, 0, s>>>(slab, G, stride, sg, dslab, dout);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

int lg_launch_slab_reduce(const float* slab, int G, int64_t stride, int64_t len, float* out, hipStream_t s) {
    const LgSlabSeg seg{0, len, out};
    return lg_launch_slab_reduce_multi(slab, G, stride, &seg, 1, nullptr, nullptr, s);
}
