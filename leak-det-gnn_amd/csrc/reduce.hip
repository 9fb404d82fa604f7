// Deterministic slab reduction shared by the backward kernels:
// out[i] = sum_g slab[g * stride + i], i < len
// in a fixed order.  One 1024-thread block per 64 columns: wave w sums slabs
// g = w, w + 16, ... for its column (one column per lane, coalesced rows), then the
// 16 wave partials are added in wave order through LDS.  Per-column work and the
// combine order depend only on (G, len), never on scheduling.
#include "common.h"
#include "reduce.h"

namespace {

__global__ void __launch_bounds__(1024) k_slab_reduce(const float* __restrict__ slab, int G, int64_t stride,
                                                      int64_t len, float* __restrict__ out) {
    __shared__ float part[16][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t col = static_cast<int64_t>(blockIdx.x) * 64 + lane;
    float acc = 0.f;
    if (col < len) {
        int g = w;
        for (; g + 48 < G; g += 64) {  // four independent loads in flight
            const float a = slab[static_cast<int64_t>(g) * stride + col];
            const float b = slab[static_cast<int64_t>(g + 16) * stride + col];
            const float c = slab[static_cast<int64_t>(g + 32) * stride + col];
            const float d = slab[static_cast<int64_t>(g + 48) * stride + col];
            acc += a;
            acc += b;
            acc += c;
            acc += d;
        }
        for (; g < G; g += 16) acc += slab[static_cast<int64_t>(g) * stride + col];
    }
    part[w][lane] = acc;
    __syncthreads();
    if (w == 0 && col < len) {
        float s = part[0][lane];
        for (int i = 1; i < 16; ++i) s += part[i][lane];
        out[col] = s;
    }
}

}  // namespace

int lg_launch_slab_reduce(const float* slab, int G, int64_t stride, int64_t len, float* out, hipStream_t s) {
    if (len <= 0) return LG_OK;
    const unsigned grid = static_cast<unsigned>((len + 63) / 64);
    k_slab_reduce<<<grid, 1024, 0, s>>>(slab, G, stride, len, out);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}
