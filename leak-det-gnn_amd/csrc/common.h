// Shared device helpers for libleakgnn (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "leakgnn.h"

#define LG_RET_IF_LAUNCH_FAILED()                 \
    do {                                          \
        if (hipGetLastError() != hipSuccess)      \
            return LG_EHIP;                       \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

static inline hipStream_t lg_stream(lg_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Kernel timing (lg_timing_arm, include/leakgnn.h): the armed event pair of this host
// thread, or nullptr; taking it disarms.  lg_launch sends a launch through
// hipExtLaunchKernelGGL with that pair, so the events carry the kernel's own start and end
// (its dispatch packet), not the enqueue gap around it; unarmed it is a plain launch.
struct LgTimingPair {
    hipEvent_t start, stop;
};
LgTimingPair* lg_timing_take();

template <typename... P, typename... A>
inline void lg_launch(void (*kernel)(P...), dim3 grid, dim3 block, uint32_t lds, hipStream_t s, A... args) {
    static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
    if (LgTimingPair* t = lg_timing_take())
        hipExtLaunchKernelGGL(kernel, grid, block, lds, s, t->start, t->stop, 0, static_cast<P>(args)...);
    else
        hipLaunchKernelGGL(kernel, grid, block, lds, s, static_cast<P>(args)...);
}

static inline int lg_num_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return 256;
    return cus;
}

// Counter-based dropout RNG: a pure function of (seed, salt, element index), so the
// forward mask never has to be stored (the backward reads it back as [y > 0] or
// recomputes it).  32-bit "lowbias32" finaliser (~10 VALU ops per element); the
// per-call key folds the 64-bit seed and the call-site salt once per thread.
// keep <=> (h >> 8) * 2^-24 >= p, kept values scaled by 1 / (1 - p).
// Restated for the tests in oracle/dropout_ref.py.
__host__ __device__ __forceinline__ uint32_t lg_mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__host__ __device__ __forceinline__ uint32_t lg_dropout_key(uint64_t seed, uint32_t salt) {
    return lg_mix32(static_cast<uint32_t>(seed) ^ lg_mix32(static_cast<uint32_t>(seed >> 32) ^ (salt * 0x9E3779B9U)));
}

// Salt bit 31 (LG_SALT_SEED_PTR, include/leakgnn.h): `seed` is then the device address of
// the uint64 seed, read at launch — a captured HIP graph re-draws its dropout streams on
// every replay by refreshing that word on the device.
constexpr uint32_t kLgSaltSeedPtr = 0x80000000u;
__device__ __forceinline__ uint32_t lg_dropout_key_dev(uint64_t seed, uint32_t salt) {
    if (salt & kLgSaltSeedPtr) seed = *reinterpret_cast<const uint64_t*>(seed);
    return lg_dropout_key(seed, salt & ~kLgSaltSeedPtr);
}

__device__ __forceinline__ bool lg_keep(uint32_t key, uint64_t idx, float p) {
    const uint32_t h = lg_mix32((static_cast<uint32_t>(idx) * 0x9E3779B9U) ^ key ^
                                (static_cast<uint32_t>(idx >> 32) * 0x85EBCA6BU));
    return static_cast<float>(h >> 8) * (1.0f / 16777216.0f) >= p;
}

__device__ __forceinline__ float lg_dropout(float v, float p, float scale, uint32_t key, uint64_t idx) {
    return lg_keep(key, idx, p) ? v * scale : 0.0f;
}

// Row-stream variant (fused GCN forward, whose backward reads the mask back as [y > 0]):
// one seed per (global row, lane group q) from two lowbias32 rounds, then one xorshift32
// step per PAIR of the lane's channels 16 mt + 4 q + reg, in (mt, reg) order: the low
// 16 bits decide the even reg, the high 16 bits the odd one (lg_keep_threshold16) —
// ~3 full-rate VALU per channel instead of a 4-multiply hash.
// Restated in oracle/dropout_ref.py (row_stream_mask).
__host__ __device__ __forceinline__ uint32_t lg_row_stream_seed(uint32_t key, uint64_t row, uint32_t q) {
    const uint32_t a = lg_mix32((static_cast<uint32_t>(row) * 0x9E3779B9U) ^ key);
    const uint32_t s = lg_mix32(a ^ (static_cast<uint32_t>(row >> 32) * 0x85EBCA6BU) ^ (q * 0x632BE5ABU));
    return s ? s : 0x6D2B79F5U;
}
__host__ __device__ __forceinline__ uint32_t lg_xorshift32(uint32_t s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}
// Row-stream keep bits of channels c4 .. c4 + 3 (c4 % 4 == 0) of one global row: the lane
// group is q = (c4 / 4) % 4, block mt = c4 / 16, and pair k of the group's stream is the
// state after k + 1 xorshift32 steps (bit i = channel c4 + i).  For a lane that owns only
// these four channels (the node init's sensor rows).
__device__ __forceinline__ uint32_t lg_row_stream_keep4(uint32_t key, uint64_t row, int c4, uint32_t thr) {
    uint32_t s = lg_row_stream_seed(key, row, static_cast<uint32_t>((c4 >> 2) & 3));
    for (int k = 0; k <= 2 * (c4 >> 4); ++k) s = lg_xorshift32(s);
    const uint32_t s2 = lg_xorshift32(s);
    return static_cast<uint32_t>((s & 0xFFFFu) >= thr) | (static_cast<uint32_t>((s >> 16) >= thr) << 1) |
           (static_cast<uint32_t>((s2 & 0xFFFFu) >= thr) << 2) | (static_cast<uint32_t>((s2 >> 16) >= thr) << 3);
}
__device__ __forceinline__ bool lg_keep_u(uint32_t s, float p) {
    return static_cast<float>(s >> 8) * (1.0f / 16777216.0f) >= p;
}
// 16-bit keep threshold of the fused GCN forward: keep <=> u16 >= rint(p * 2^16)
// (p quantised to 1/65536), two decisions per xorshift step.
__host__ __device__ __forceinline__ uint32_t lg_keep_threshold16(float p) {
    return static_cast<uint32_t>(rintf(p * 65536.0f));
}

// Division by a runtime divisor that is fixed per launch (N nodes, P pipes, S sensors):
// magic multiplier computed on the host (Granlund & Montgomery 1994, round-up
// variant), so a row index splits into (window, node) with one v_mul_hi_u32 and
// three cheap ops instead of a ~130-instruction 64-bit division.  Exact for every
// dividend n < 2^32; kernels using it require B*N < 2^31 (checked at the API).
struct lg_fastdiv {
    uint32_t d, m, s1, s2;
};

static inline lg_fastdiv lg_make_fastdiv(uint32_t d) {
    uint32_t l = 0;
    while (l < 32 && (uint64_t{1} << l) < d) ++l;  // l = ceil(log2 d)
    const uint64_t m = ((uint64_t{1} << 32) * ((uint64_t{1} << l) - d)) / d + 1;
    return lg_fastdiv{d, static_cast<uint32_t>(m), l < 1 ? l : 1u, l > 0 ? l - 1 : 0u};
}

__device__ __forceinline__ uint32_t lg_div(uint32_t n, const lg_fastdiv& f) {
    const uint32_t t = __umulhi(n, f.m);
    return (t + ((n - t) >> f.s1)) >> f.s2;
}

constexpr int kLgNmInline = 6;  // CSR entries held inline in a node-table record (graph.hip k_nm_table)
constexpr int32_t kLgSensorCol = 0x40000000;  // sensor-marked node-table col: kLgSensorCol | sensor slot

constexpr int64_t kLgMaxRows = int64_t{1} << 31;  // row-index space of the fast-division kernels

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// Cache policy (the raw buffer stores' aux operand) of the activation stores: the large
// per-launch outputs that later kernels read (trunk y and its mask words, dx, the EdgeHead
// hidden layer, the GRU's h and gates).  16 = sc1: agent-scope stores, written through the
// XCD's L2 while the kernel runs.  With the default write-back policy the last few MiB of
// each XCD's L2 were still dirty when the kernel ended and were written back then, after
// its work (r06h-j, same box: the trunk forward without its y stores ran 16-17 us against
// 21; sc1 on them, in the step, layer 1 21.1 -> 19.8-20.0 us and layer 0 24.9 -> 23.0, with
// the kernels that read y unchanged; nt (2) instead sent y past the Infinity Cache and the
// next layer's gather took 26.6 us).  0 restores write-back (lab A/B).  Stores that write
// partial cache lines per instruction keep write-back: the GRU forward's h / gate stores
// (64 B of a row per lane group) took 88-91 us under sc1 against 82-83 (r06k).
#ifndef LG_ACT_AUX
#define LG_ACT_AUX 16
#endif
constexpr int kLgActAux = LG_ACT_AUX;
// A buffer descriptor over n floats at p for activation stores (n * 4 < 2^31; callers with a
// larger buffer use st4), and one 16-byte store at float offset e with the activation policy.
// The data registers stay unwritten for a few wait states after the store (lg_store_guard:
// the compiler was seen reusing them at once, gcn_nm.hip).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t lg_act_rsrc(float* p, int64_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(p, static_cast<short>(0), static_cast<int>(n * 4), 0x00020000);
}
template <int AUX = kLgActAux>
__device__ __forceinline__ void st4_act(__amdgpu_buffer_rsrc_t rs, uint32_t e, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v), rs,
                                           4u * e, 0, AUX);
}
