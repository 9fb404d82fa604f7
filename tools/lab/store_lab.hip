// Store-pattern lab: does a write-only stream reach the same rate when each store instruction
// covers 64-byte pieces of 16 rows (the MFMA-layout epilogues: node init before ABI 20, the
// EdgeHead forward's hidden rows, the GRU forward's h / gates) as when it covers whole rows?
// Build: hipcc --offload-arch=gfx950 -O3 tools/lab/store_lab.hip -o tools/lab/store_lab.bin
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// rows of RW floats; a 256-thread workgroup writes 64 rows.
// LINES: lane -> (row, 16-byte group), consecutive lanes along the row (whole-line stores).
// PIECES: lane -> (row = lane & 15, group q = lane >> 4): one instruction covers 64 bytes of
// 16 rows; RW / 16 instructions finish the rows.
template <int RW, bool LINES>
__global__ void __launch_bounds__(256) k_store(float* __restrict__ d, int64_t rows, float v) {
    constexpr int G4 = RW / 4;  // float4 per row
    const int64_t r0 = static_cast<int64_t>(blockIdx.x) * 64;
    const f32x4 val = f32x4{v, v + 1.f, v + 2.f, v + 3.f};
    if (LINES) {
        constexpr int RPI = 256 / G4;  // rows per workgroup instruction
#pragma unroll
        for (int it = 0; it < 64 / RPI; ++it) {
            const int64_t r = r0 + it * RPI + threadIdx.x / G4;
            if (r < rows) *reinterpret_cast<f32x4*>(d + r * RW + 4 * (threadIdx.x % G4)) = val;
        }
    } else {
        const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
        const int64_t r = r0 + 16 * w + j;
        if (r < rows)
#pragma unroll
            for (int mt = 0; mt < G4 / 4; ++mt) *reinterpret_cast<f32x4*>(d + r * RW + 16 * mt + 4 * q) = val;
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
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / iters;
}

template <int RW>
static void run(float* d, int64_t bytes) {
    const int64_t rows = bytes / (4 * RW);
    const unsigned grid = static_cast<unsigned>((rows + 63) / 64);
    const float tl = timeit([&] { k_store<RW, true><<<grid, 256>>>(d, rows, 1.f); }, 20);
    const float tp = timeit([&] { k_store<RW, false><<<grid, 256>>>(d, rows, 1.f); }, 20);
    const double b = static_cast<double>(rows) * RW * 4;
    printf("{\"row_floats\": %d, \"MB\": %.1f, \"lines_us\": %.2f, \"lines_GBps\": %.0f, \"pieces_us\": %.2f, "
           "\"pieces_GBps\": %.0f}\n",
           RW, b / 1e6, tl, b / tl / 1e3, tp, b / tp / 1e3);
}

int main() {
    float* d = nullptr;
    const int64_t big = int64_t{342} << 20;
    if (hipMalloc(&d, big) != hipSuccess) return 1;
    run<64>(d, int64_t{43} << 20);    // node init: 43 MB of 256-byte rows
    run<128>(d, int64_t{100} << 20);  // EdgeHead hidden rows: 100 MB of 512-byte rows
    run<64>(d, big);                  // GRU forward h / gates scale
    hipFree(d);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
