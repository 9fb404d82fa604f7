// Internal (not part of the C ABI): deterministic fixed-order slab reduction,
// out[i] = sum_{g < G} slab[g * stride + i] for i < len, enqueued on stream s.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

int lg_launch_slab_reduce(const float* slab, int G, int64_t stride, int64_t len, float* out, hipStream_t s);
