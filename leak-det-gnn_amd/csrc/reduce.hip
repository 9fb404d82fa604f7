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
// never on scheduling.  A reduce batch (lg_reduce_batch_begin / _flush, include/leakgnn.h)
// takes the reductions of several backward calls into ONE launch (up to 24 segments and
// 4 fp64 columns per launch); each column keeps its own order, so results do not change.
#include "common.h"
#include "reduce.h"

#include <algorithm>
#include <vector>

namespace {

constexpr int kJobSegs = 24;  // segments per launch (a whole detector backward: trunk 8, heads 6, GRU 4)
constexpr int kJobD = 4;      // fp64 columns per launch
#ifndef LG_SLAB_VEC_G
#define LG_SLAB_VEC_G 256  // most slab rows a vector segment takes (lab: 512, 32 rows in flight: 11.2 -> 14.7 us, r06zh)
#endif
#ifndef LG_SLAB_VEC
#define LG_SLAB_VEC 1  // 16-byte column loads for aligned segments (lab: 0 = one column per lane)
#endif

struct Segs {
    const float* slab[kJobSegs];
    const float* slab2[kJobSegs];
    int64_t stride[kJobSegs], off[kJobSegs], stride2[kJobSegs], off2[kJobSegs], len[kJobSegs];
    float* out[kJobSegs];
    int G[kJobSegs], G2[kJobSegs];
    int vec[kJobSegs];        // 1: 16-byte aligned rows (stride, off, len multiples of 4): a lane sums 4 columns
    int first[kJobSegs + 1];  // first block of each segment; first[n] = total column blocks
    int n;
    const double* dslab[kJobD];
    float* dout[kJobD];
    int dG[kJobD];
    int nd;
};

// fp64 sum over slabs g = w, w + 16, ... < G of src[g * stride + col], in that order,
// kRedInflight independent loads per round trip
__device__ __forceinline__ void slab_col_sum(const float* __restrict__ src, int G, int64_t stride, int64_t col, int w,
                                             double& acc) {
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

// the same as slab_col_sum for 4 adjacent columns (one 16-byte load per slab row): each column
// keeps slab_col_sum's order, so the sums are bit-identical to the scalar form
template <int kRedInflight>
__device__ __forceinline__ void slab_col_sum4(const float* __restrict__ src, int G, int64_t stride, int64_t col, int w,
                                              double (&acc)[4]) {
    int g = w;
    for (; g + 16 * (kRedInflight - 1) < G; g += 16 * kRedInflight) {
        f32x4 v[kRedInflight];
#pragma unroll
        for (int u = 0; u < kRedInflight; ++u)
            v[u] = *reinterpret_cast<const f32x4*>(src + static_cast<int64_t>(g + 16 * u) * stride + col);
#pragma unroll
        for (int u = 0; u < kRedInflight; ++u)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] += v[u][c];
    }
    for (; g < G; g += 16) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(src + static_cast<int64_t>(g) * stride + col);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] += v[c];
    }
}

__global__ void __launch_bounds__(1024) k_slab_reduce(Segs sg) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int b = blockIdx.x;
    if (b >= sg.first[sg.n]) {  // fp64 column: 1024 strided partials, then a fixed tree
        const int d = b - sg.first[sg.n];
        __shared__ double dp[1024];
        double acc = 0.0;
        for (int g = threadIdx.x; g < sg.dG[d]; g += 1024) acc += sg.dslab[d][g];
        dp[threadIdx.x] = acc;
        __syncthreads();
        for (int h = 512; h > 0; h >>= 1) {
            if (threadIdx.x < h) dp[threadIdx.x] += dp[threadIdx.x + h];
            __syncthreads();
        }
        if (threadIdx.x == 0) sg.dout[d][0] = static_cast<float>(dp[0]);
        return;
    }
    int k = 0;
    while (k + 1 < sg.n && b >= sg.first[k + 1]) ++k;
    if (sg.vec[k]) {  // 256 columns per block, 4 per lane
        __shared__ double part4[16][256];
        const int64_t col = static_cast<int64_t>(b - sg.first[k]) * 256 + 4 * lane;
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
        if (col < sg.len[k]) {  // one round of loads per wave: 16 rows (G <= 256) or 32 (G <= 512)
            if (sg.G[k] > 256)
                slab_col_sum4<32>(sg.slab[k] + sg.off[k], sg.G[k], sg.stride[k], col, w, acc);
            else
                slab_col_sum4<16>(sg.slab[k] + sg.off[k], sg.G[k], sg.stride[k], col, w, acc);
            if (sg.slab2[k]) {
                if (sg.G2[k] > 256)
                    slab_col_sum4<32>(sg.slab2[k] + sg.off2[k], sg.G2[k], sg.stride2[k], col, w, acc);
                else
                    slab_col_sum4<16>(sg.slab2[k] + sg.off2[k], sg.G2[k], sg.stride2[k], col, w, acc);
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) part4[w][4 * lane + c] = acc[c];
        __syncthreads();
        if (threadIdx.x < 256) {
            const int64_t cc = static_cast<int64_t>(b - sg.first[k]) * 256 + threadIdx.x;
            if (cc < sg.len[k]) {
                double t = part4[0][threadIdx.x];
                for (int i = 1; i < 16; ++i) t += part4[i][threadIdx.x];
                sg.out[k][cc] = static_cast<float>(t);
            }
        }
        return;
    }
    const int64_t col = static_cast<int64_t>(b - sg.first[k]) * 64 + lane;
    __shared__ double part[16][64];
    double acc = 0.0;
    if (col < sg.len[k]) {
        slab_col_sum(sg.slab[k] + sg.off[k], sg.G[k], sg.stride[k], col, w, acc);
        if (sg.slab2[k]) slab_col_sum(sg.slab2[k] + sg.off2[k], sg.G2[k], sg.stride2[k], col, w, acc);
    }
    part[w][lane] = acc;
    __syncthreads();
    if (w == 0 && col < sg.len[k]) {
        double s = part[0][lane];
        for (int i = 1; i < 16; ++i) s += part[i][lane];
        sg.out[k][col] = static_cast<float>(s);
    }
}

struct SegJob {
    const float* slab;
    int G;
    int64_t stride;
    LgSlabSeg seg;
};
struct DJob {
    const double* dslab;
    int G;
    float* out;
};

// The reduce batch of this host thread (lg_reduce_batch_begin / _flush)
struct Batch {
    bool active = false;
    std::vector<SegJob> segs;
    std::vector<DJob> djobs;
};
thread_local Batch t_batch;

int launch_jobs(const SegJob* segs, int nseg, const DJob* dj, int nd, hipStream_t s) {
    Segs sg{};
    int blocks = 0;
    for (int i = 0; i < nseg; ++i) {
        const SegJob& j = segs[i];
        sg.slab[i] = j.slab;
        sg.G[i] = j.G;
        sg.stride[i] = j.stride;
        sg.off[i] = j.seg.off;
        sg.len[i] = j.seg.len;
        sg.out[i] = j.seg.out;
        sg.slab2[i] = j.seg.slab2;
        sg.G2[i] = j.seg.G2;
        sg.stride2[i] = j.seg.stride2;
        sg.off2[i] = j.seg.off2;
        auto al4 = [](uint64_t v) { return (v & 3u) == 0; };
        // 4 columns a lane cut the blocks 4x: only where each wave's rows fit one round of loads
        // (G <= 256: the heads' and the GRU's slabs; the trunk's 512 rows measured slower, r06zd)
        const bool vec = LG_SLAB_VEC && j.G <= LG_SLAB_VEC_G && (!j.seg.slab2 || j.seg.G2 <= LG_SLAB_VEC_G) && al4(reinterpret_cast<uintptr_t>(j.slab) / 4) && al4(j.stride) &&
                         al4(j.seg.off) && al4(j.seg.len) &&
                         (!j.seg.slab2 || (al4(reinterpret_cast<uintptr_t>(j.seg.slab2) / 4) && al4(j.seg.stride2) &&
                                           al4(j.seg.off2)));
        sg.vec[i] = vec ? 1 : 0;
        sg.first[i] = blocks;
        blocks += static_cast<int>(vec ? (j.seg.len + 255) / 256 : (j.seg.len + 63) / 64);
    }
    sg.first[nseg] = blocks;
    sg.n = nseg;
    for (int d = 0; d < nd; ++d) {
        sg.dslab[d] = dj[d].dslab;
        sg.dG[d] = dj[d].G;
        sg.dout[d] = dj[d].out;
    }
    sg.nd = nd;
    const int total = blocks + nd;
    if (total == 0) return LG_OK;
    k_slab_reduce<<<total, 1024, 0, s>>>(sg);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

int launch_all(const std::vector<SegJob>& segs, const std::vector<DJob>& dj, hipStream_t s) {
    size_t i = 0, d = 0;
    while (i < segs.size() || d < dj.size()) {
        const int ns = static_cast<int>(std::min<size_t>(kJobSegs, segs.size() - i));
        const int nd = static_cast<int>(std::min<size_t>(kJobD, dj.size() - d));
        const int rc = launch_jobs(segs.data() + i, ns, dj.data() + d, nd, s);
        if (rc != LG_OK) return rc;
        i += ns;
        d += nd;
    }
    return LG_OK;
}

}  // namespace

int lg_launch_slab_reduce_multi(const float* slab, int G, int64_t stride, const LgSlabSeg* segs, int nseg,
                                const double* dslab, float* dout, hipStream_t s) {
    if (nseg < 0 || nseg > kLgMaxSlabSegs || G < 0 || (dslab && !dout)) return LG_EINVAL;
    std::vector<SegJob> js;
    std::vector<DJob> dj;
    for (int i = 0; i < nseg; ++i) {
        if (segs[i].out == nullptr || segs[i].len <= 0) continue;
        js.push_back(SegJob{slab, G, stride, segs[i]});
    }
    if (dslab) dj.push_back(DJob{dslab, G, dout});
    if (t_batch.active) {
        t_batch.segs.insert(t_batch.segs.end(), js.begin(), js.end());
        t_batch.djobs.insert(t_batch.djobs.end(), dj.begin(), dj.end());
        return LG_OK;
    }
    return launch_all(js, dj, s);
}

int lg_launch_slab_reduce(const float* slab, int G, int64_t stride, int64_t len, float* out, hipStream_t s) {
    const LgSlabSeg seg{0, len, out};
    return lg_launch_slab_reduce_multi(slab, G, stride, &seg, 1, nullptr, nullptr, s);
}

bool lg_reduce_batch_pending(const float* out, const float** slab, int* G, int64_t* stride, int64_t* off) {
    if (!t_batch.active || out == nullptr) return false;
    for (const SegJob& j : t_batch.segs) {
        if (j.seg.out == out && j.seg.slab2 == nullptr) {
            *slab = j.slab;
            *G = j.G;
            *stride = j.stride;
            *off = j.seg.off;
            return true;
        }
    }
    return false;
}

extern "C" int lg_reduce_batch_begin(void) {
    if (t_batch.active) return LG_EINVAL;
    t_batch.segs.clear();
    t_batch.djobs.clear();
    t_batch.active = true;
    return LG_OK;
}

extern "C" int lg_reduce_batch_flush(lg_stream_t stream) {
    if (!t_batch.active) return LG_EINVAL;
    t_batch.active = false;
    const int rc = launch_all(t_batch.segs, t_batch.djobs, lg_stream(stream));
    t_batch.segs.clear();
    t_batch.djobs.clear();
    return rc;
}

// ---------------------------------------------------------------- measured copy peak
// The box's achievable HBM rate for a read + write stream (bench.py stream_copy): one 16-byte
// non-temporal load and store per lane, one workgroup per 4 KiB, no grid stride.  Measured
// (profiles/r03/r03n/copy_lab.txt, 2 GiB): this flat shape 6.52 TB/s; grid-stride loops with
// 4-64 workgroups per CU and 1-8 vectors in flight per lane 4.3-5.5 TB/s (the round-2 kernel,
// U=4 at 16/CU, 4.7); hipMemcpyAsync D2D 4.8.  Short-lived workgroups keep every channel fed
// as the dispatcher refills CUs; long-lived strided ones drift into channel-hot phases.
namespace {
__global__ void __launch_bounds__(256) k_stream_copy(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                     int64_t n4) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n4) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}
}  // namespace

extern "C" int lg_stream_copy(const void* src, void* dst, int64_t bytes, lg_stream_t stream) {
    if (bytes < 0 || (bytes % 16) != 0 || (bytes > 0 && (!src || !dst))) return LG_EINVAL;
    if (bytes == 0) return LG_OK;
    const int64_t n4 = bytes / 16;
    if ((n4 + 255) / 256 > 0x7FFFFFFFLL) return LG_EINVAL;
    const unsigned grid = static_cast<unsigned>((n4 + 255) / 256);
    k_stream_copy<<<grid, 256, 0, lg_stream(stream)>>>(static_cast<const f32x4*>(src), static_cast<f32x4*>(dst), n4);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

// ---------------------------------------------------------------- dropout seed slots
// Re-draw of a captured step's device seed slots (models/ops.py SeedSlots.refresh): the
// state word advances by one and slot i becomes splitmix64(state * n + i + 1) & (2^62 - 1).
// One wave, no host involvement, so a replayed graph draws fresh seeds with ONE launch
// (torch's generator inside a graph costs a random_ kernel plus two fills per replay).
namespace {
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void __launch_bounds__(64) k_seed_advance(uint64_t* __restrict__ slots, int n, uint64_t* __restrict__ state) {
    const uint64_t c = state[0] + 1;  // every lane reads before lane 0 writes (one wave, same address)
    for (int i = threadIdx.x; i < n; i += 64)
        slots[i] = splitmix64(c * static_cast<uint64_t>(n) + static_cast<uint64_t>(i) + 1) & ((1ull << 62) - 1);
    if (threadIdx.x == 0) state[0] = c;
}
}  // namespace

extern "C" int lg_seed_slots_advance(uint64_t* slots, int64_t n, uint64_t* state, lg_stream_t stream) {
    if (n < 0 || n > 4096 || (n > 0 && (!slots || !state))) return LG_EINVAL;
    if (n == 0) return LG_OK;
    k_seed_advance<<<1, 64, 0, lg_stream(stream)>>>(slots, static_cast<int>(n), state);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

// ---------------------------------------------------------------- graph replay
// A captured training step (models/graph_step.py) replayed by hipGraphLaunch of its
// instantiated executable: torch's CUDAGraph.replay() adds its own per-replay host work
// (generator-state prologue) in front of the same launch.
extern "C" int lg_graph_replay(void* graph_exec, int64_t n, lg_stream_t stream) {
    if (!graph_exec || n < 0) return LG_EINVAL;
    for (int64_t i = 0; i < n; ++i)
        if (hipGraphLaunch(static_cast<hipGraphExec_t>(graph_exec), lg_stream(stream)) != hipSuccess) return LG_EHIP;
    return LG_OK;
}
