// Internal (not part of the C ABI): deterministic fixed-order slab reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kLgMaxSlabSegs = 6;

// One output segment: out[i] = sum_{g < G} slab[g * stride + off + i], i < len.
struct LgSlabSeg {
    int64_t off;
    int64_t len;
    float* out;  // NULL: segment skipped
};

// All segments (and optionally dout[0] = (float) sum_{g < G} dslab[g] in fp64) in one
// launch on stream s.
int lg_launch_slab_reduce_multi(const float* slab, int G, int64_t stride, const LgSlabSeg* segs, int nseg,
                                const double* dslab, float* dout, hipStream_t s);

int lg_launch_slab_reduce(const float* slab, int G, int64_t stride, int64_t len, float* out, hipStream_t s);
