// Copy-rate lab: which read+write stream shape reaches the box's HBM ceiling (bench.py
// stream_copy).  Build: hipcc --offload-arch=gfx950 -O3 tools/lab/copy_lab.hip -o build/copy_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) k_stride(const f32x4* __restrict__ s, f32x4* __restrict__ d, int64_t n4) {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
    int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], d + i + u * stride);
            else d[i + u * stride] = v[u];
        }
    }
    for (; i < n4; i += stride) d[i] = s[i];
}

// one block of U * 256 vectors per workgroup, no grid stride (a grid of n4 / (256 U) workgroups)
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_flat(const f32x4* __restrict__ s, f32x4* __restrict__ d, int64_t n4) {
    const int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * U + threadIdx.x;
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + u * 256;
        v[u] = i < n4 ? (NT ? __builtin_nontemporal_load(s + i) : s[i]) : f32x4{};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + u * 256;
        if (i < n4) {
            if (NT) __builtin_nontemporal_store(v[u], d + i);
            else d[i] = v[u];
        }
    }
}

template <typename F>
static float timeit(F f, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) f();
    hipEventRecord(a);
    for (int i = 0; i < iters; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / iters;
}

int main() {
    const int64_t bytes = 2ll << 30, n4 = bytes / 16;
    f32x4 *s, *d;
    if (hipMalloc(&s, bytes) || hipMalloc(&d, bytes)) return 1;
    hipMemset(s, 1, bytes);
    hipMemset(d, 0, bytes);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto rep = [&](const char* name, float ms) { printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms, 2.0 * bytes / (ms * 1e6)); };
    for (int wpc : {4, 8, 16, 32, 64}) {
        const unsigned g = wpc * cus;
        char nm[64];
        snprintf(nm, sizeof nm, "stride U4 nt  grid %d/CU", wpc);
        rep(nm, timeit([&] { k_stride<4, true><<<g, 256>>>(s, d, n4); }, 10));
        snprintf(nm, sizeof nm, "stride U4 plain grid %d/CU", wpc);
        rep(nm, timeit([&] { k_stride<4, false><<<g, 256>>>(s, d, n4); }, 10));
        snprintf(nm, sizeof nm, "stride U8 plain grid %d/CU", wpc);
        rep(nm, timeit([&] { k_stride<8, false><<<g, 256>>>(s, d, n4); }, 10));
        snprintf(nm, sizeof nm, "stride U1 plain grid %d/CU", wpc);
        rep(nm, timeit([&] { k_stride<1, false><<<g, 256>>>(s, d, n4); }, 10));
    }
    rep("flat U1 plain", timeit([&] { k_flat<1, false><<<(n4 + 255) / 256, 256>>>(s, d, n4); }, 10));
    rep("flat U1 nt", timeit([&] { k_flat<1, true><<<(n4 + 255) / 256, 256>>>(s, d, n4); }, 10));
    rep("flat U4 plain", timeit([&] { k_flat<4, false><<<(n4 + 1023) / 1024, 256>>>(s, d, n4); }, 10));
    rep("flat U4 nt", timeit([&] { k_flat<4, true><<<(n4 + 1023) / 1024, 256>>>(s, d, n4); }, 10));
    rep("hipMemcpyAsync D2D", timeit([&] { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); }, 10));
    hipFree(s);
    hipFree(d);
    return 0;
}
