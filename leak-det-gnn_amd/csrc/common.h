// Shared device helpers for libleakgnn (gfx950 / CDNA4 only).
#pragma once
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

static inline int lg_num_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return 256;
    return cus;
}

// Counter-based dropout RNG: a pure function of (seed, salt, element index), so
// the forward mask never has to be stored (backward reads the mask back as
// [y > 0]).  splitmix64 finaliser; top 24 bits -> uniform in [0, 1).
__device__ __forceinline__ uint32_t lg_hash(uint64_t seed, uint32_t salt, uint64_t idx) {
    uint64_t z = seed ^ (static_cast<uint64_t>(salt) << 32) ^ (idx * 0x9E3779B97F4A7C15ull);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return static_cast<uint32_t>(z >> 40);  // 24 bits
}

__device__ __forceinline__ float lg_dropout(float v, float p, float scale, uint64_t seed, uint32_t salt,
                                            uint64_t idx) {
    const float u = static_cast<float>(lg_hash(seed, salt, idx)) * (1.0f / 16777216.0f);
    return u >= p ? v * scale : 0.0f;
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
