// Internal (not part of the C ABI): deterministic fixed-order slab reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kLgMaxSlabSegs = 6;

// One output segment: out[i] = sum_{g < G} slab[g * stride + off + i], i < len, then (when
// slab2 is set) + sum_{g < G2} slab2[g * stride2 + off2 + i]: a second partial set summed
// into the same fp64 column (a gradient whose producer's reduction is still pending in a
// reduce batch, see lg_reduce_batch_begin).
struct LgSlabSeg {
    int64_t off;
    int64_t len;
    float* out;  // NULL: segment skipped
    const float* slab2 = nullptr;
    int G2 = 0;
    int64_t stride2 = 0;
    int64_t off2 = 0;
};

// All segments (and optionally dout[0] = (float) sum_{g < G} dslab[g] in fp64) in one
// launch on stream s — or, inside a reduce batch on this host thread, recorded for the
// batch's single launch.
int lg_launch_slab_reduce_multi(const float* slab, int G, int64_t stride, const LgSlabSeg* segs, int nseg,
                                const double* dslab, float* dout, hipStream_t s);

int lg_launch_slab_reduce(const float* slab, int G, int64_t stride, int64_t len, float* out, hipStream_t s);

// Inside a reduce batch: the partial set of a recorded segment whose output is `out`
// (true), so a consumer of that output can take the partials instead (LgSlabSeg::slab2).
bool lg_reduce_batch_pending(const float* out, const float** slab, int* G, int64_t* stride, int64_t* off);
