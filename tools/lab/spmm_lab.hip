// Tuning lab (not product code): sweeps gather structures for y = Ahat x on an
// L-TOWN-A-shaped problem (N = 661, ~3.3 entries/row incl. self loop, D = 64,
// B = 256 windows) and prints time and algorithmic GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/spmm_lab.hip -o tools/_spmm_lab && tools/_spmm_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

constexpr int D = 64;

struct TileRange { long first, end, stride; };
__device__ __forceinline__ TileRange tiles(long ntiles, int wave, int waves) {
    const long G = gridDim.x, b = blockIdx.x;
    if (G < 8) return TileRange{b * waves + wave, ntiles, G * waves};
    const long x = b % 8, k = b / 8, nbx = (G - x + 7) / 8, chunk = (ntiles + 7) / 8;
    const long begin = x * chunk, end = min(ntiles, begin + chunk);
    return TileRange{begin + k * waves + wave, end, nbx * waves};
}

// ---- variant A: lane = (row j, quarter q), 16 rows per wave, U neighbours in flight
template <int WAVES, bool LDS_CSR, int U>
__global__ void __launch_bounds__(64 * WAVES) kA(const int* rp, const int* col, const float* w, const float* x,
                                                 float* y, int N, long R) {
    extern __shared__ char smem[];
    const int* Rp = rp; const int* C = col; const float* Wt = w;
    if (LDS_CSR) {
        int* s_rp = (int*)smem; const int nnz = rp[N];
        int* s_c = s_rp + ((N + 4) & ~3); float* s_w = (float*)(s_c + ((nnz + 3) & ~3));
        for (int i = threadIdx.x; i <= N; i += blockDim.x) s_rp[i] = rp[i];
        for (int i = threadIdx.x; i < nnz; i += blockDim.x) { s_c[i] = col[i]; s_w[i] = w[i]; }
        __syncthreads();
        Rp = s_rp; C = s_c; Wt = s_w;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const long ntiles = (R + 15) / 16;
    const TileRange tr = tiles(ntiles, wave, WAVES);
    for (long t = tr.first; t < tr.end; t += tr.stride) {
        const long r = t * 16 + j;
        if (r >= R) continue;
        const long b = r / N, n = r - b * N;
        const float* base = x + b * (long)N * D + 4 * q;
        f32x4 acc[4] = {};
        const int e0 = Rp[n], e1 = Rp[n + 1];
        for (int e = e0; e < e1; e += U) {
            int s[U]; float ww[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool ok = e + u < e1;
                s[u] = ok ? C[e + u] : (int)n;
                ww[u] = ok ? Wt[e + u] : 0.f;
            }
            f32x4 v[U][4];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int a = 0; a < 4; ++a) v[u][a] = ld4(base + (long)s[u] * D + 16 * a);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int a = 0; a < 4; ++a) acc[a] += ww[u] * v[u][a];
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) st4(y + r * D + 16 * a + 4 * q, acc[a]);
    }
}

// ---- variant D: 16 lanes per row (one float4 each), 4 rows per wave-instruction,
// ROWS rows per lane in flight (row groups interleaved), U neighbours unrolled.
template <int WAVES, bool LDS_CSR, int ROWS, int U>
__global__ void __launch_bounds__(64 * WAVES) kD(const int* rp, const int* col, const float* w, const float* x,
                                                 float* y, int N, long R) {
    extern __shared__ char smem[];
    const int* Rp = rp; const int* C = col; const float* Wt = w;
    if (LDS_CSR) {
        int* s_rp = (int*)smem; const int nnz = rp[N];
        int* s_c = s_rp + ((N + 4) & ~3); float* s_w = (float*)(s_c + ((nnz + 3) & ~3));
        for (int i = threadIdx.x; i <= N; i += blockDim.x) s_rp[i] = rp[i];
        for (int i = threadIdx.x; i < nnz; i += blockDim.x) { s_c[i] = col[i]; s_w[i] = w[i]; }
        __syncthreads();
        Rp = s_rp; C = s_c; Wt = s_w;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, rl = lane >> 4, fg = lane & 15;
    constexpr int RPW = 4 * ROWS;  // rows per wave per iteration
    const long ntiles = (R + RPW - 1) / RPW;
    const TileRange tr = tiles(ntiles, wave, WAVES);
    for (long t = tr.first; t < tr.end; t += tr.stride) {
        long r[ROWS]; int e0[ROWS], e1[ROWS]; const float* base[ROWS]; f32x4 acc[ROWS];
        int maxd = 0;
#pragma unroll
        for (int k = 0; k < ROWS; ++k) {
            r[k] = t * RPW + 4 * k + rl;
            acc[k] = f32x4{0, 0, 0, 0};
            if (r[k] < R) {
                const long b = r[k] / N, n = r[k] - b * N;
                e0[k] = Rp[n]; e1[k] = Rp[n + 1];
                base[k] = x + b * (long)N * D + 4 * fg;
            } else { e0[k] = e1[k] = 0; base[k] = x; }
            maxd = max(maxd, e1[k] - e0[k]);
        }
        for (int d = 0; d < maxd; d += U) {
            f32x4 v[ROWS][U]; float ww[ROWS][U];
#pragma unroll
            for (int k = 0; k < ROWS; ++k)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int e = e0[k] + d + u;
                    const bool ok = e < e1[k];
                    const int s = ok ? C[e] : 0;
                    ww[k][u] = ok ? Wt[e] : 0.f;
                    v[k][u] = ld4(base[k] + (long)s * D);
                }
#pragma unroll
            for (int k = 0; k < ROWS; ++k)
#pragma unroll
                for (int u = 0; u < U; ++u) acc[k] += ww[k][u] * v[k][u];
        }
#pragma unroll
        for (int k = 0; k < ROWS; ++k)
            if (r[k] < R) st4(y + r[k] * D + 4 * fg, acc[k]);
    }
}

// ---- variant S: plain streaming copy (upper bound for read x + write y)
__global__ void __launch_bounds__(256) kcopy(const float* x, float* y, long n4) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
        st4(y + 4 * i, ld4(x + 4 * i));
}

template <typename F>
float timeit(F f, int iters) {
    for (int i = 0; i < 3; ++i) f();
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / iters;
}

int main(int argc, char** argv) {
    const int N = 661, B = argc > 1 ? atoi(argv[1]) : 256;
    const long R = (long)B * N;
    std::mt19937 rng(1);
    // symmetric random graph with degrees 1..5 (+ self loop), nnz ~ 2193
    std::vector<std::vector<int>> adj(N);
    for (int i = 1; i < N; ++i) { int p = rng() % i; adj[i].push_back(p); adj[p].push_back(i); }
    for (int k = 0; k < 105; ++k) { int a = rng() % N, b = rng() % N; if (a != b && adj[a].size() < 5 && adj[b].size() < 5) { adj[a].push_back(b); adj[b].push_back(a); } }
    std::vector<int> rp(N + 1, 0), col; std::vector<float> w;
    for (int i = 0; i < N; ++i) {
        for (int s : adj[i]) { col.push_back(s); w.push_back(0.3f); }
        col.push_back(i); w.push_back(0.3f);
        rp[i + 1] = (int)col.size();
    }
    const int nnz = (int)col.size();
    printf("N=%d nnz=%d B=%d\n", N, nnz, B);
    int *d_rp, *d_col; float *d_w, *d_x, *d_y;
    CK(hipMalloc(&d_rp, 4 * (N + 1))); CK(hipMalloc(&d_col, 4 * nnz)); CK(hipMalloc(&d_w, 4 * nnz));
    CK(hipMalloc(&d_x, 4 * R * D)); CK(hipMalloc(&d_y, 4 * R * D));
    CK(hipMemcpy(d_rp, rp.data(), 4 * (N + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), 4 * nnz, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_w, w.data(), 4 * nnz, hipMemcpyHostToDevice));
    std::vector<float> hx(R * D);
    for (auto& v : hx) v = (rng() % 1000) / 1000.f;
    CK(hipMemcpy(d_x, hx.data(), 4 * R * D, hipMemcpyHostToDevice));
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const double bytes = 8.0 * R * D;
    const size_t lds = 4 * ((N + 4) & ~3) + 8 * ((nnz + 3) & ~3);
    std::vector<float> ref;
    auto check = [&](const char* name, float us) {
        std::vector<float> hy(R * D);
        CK(hipMemcpy(hy.data(), d_y, 4 * R * D, hipMemcpyDeviceToHost));
        if (ref.empty()) ref = hy;
        double err = 0; for (long i = 0; i < R * D; i += 97) err = fmax(err, fabs(hy[i] - ref[i]));
        printf("%-34s %8.2f us  %7.0f GB/s  maxdiff %.1e\n", name, us, bytes / us / 1e3, err);
    };
    const int it = 50;
    float us;
    us = timeit([&] { kcopy<<<cus * 8, 256>>>(d_x, d_y, R * D / 4); }, it);
    printf("%-34s %8.2f us  %7.0f GB/s\n", "stream copy (read x + write y)", us, bytes / us / 1e3);
#define RUN_A(WV, L, U, PERCU)                                                                          \
    us = timeit([&] { kA<WV, L, U><<<cus * PERCU, 64 * WV, L ? lds : 0>>>(d_rp, d_col, d_w, d_x, d_y, N, R); }, it); \
    check("A waves=" #WV " lds=" #L " U=" #U " perCU=" #PERCU, us);
    RUN_A(4, true, 2, 8) RUN_A(4, true, 1, 8) RUN_A(4, true, 4, 8) RUN_A(16, true, 2, 2) RUN_A(16, true, 1, 2)
    RUN_A(4, false, 2, 8) RUN_A(16, false, 2, 2) RUN_A(8, true, 2, 4)
#define RUN_D(WV, L, ROWS, U, PERCU)                                                                            \
    us = timeit([&] { kD<WV, L, ROWS, U><<<cus * PERCU, 64 * WV, L ? lds : 0>>>(d_rp, d_col, d_w, d_x, d_y, N, R); }, it); \
    check("D waves=" #WV " lds=" #L " rows=" #ROWS " U=" #U " perCU=" #PERCU, us);
    RUN_D(4, true, 1, 1, 8) RUN_D(4, true, 2, 1, 8) RUN_D(4, true, 4, 1, 8) RUN_D(4, true, 2, 2, 8)
    RUN_D(4, true, 4, 2, 8) RUN_D(16, true, 4, 1, 2) RUN_D(16, true, 2, 2, 2) RUN_D(4, false, 4, 1, 8)
    RUN_D(16, false, 4, 1, 2) RUN_D(8, true, 4, 1, 4) RUN_D(4, true, 8, 1, 8)
    return 0;
}
