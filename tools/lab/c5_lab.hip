// C5 gather lab (not product code): which gather structure reaches HBM speed for
// y = Ahat x on ONE large graph (BASELINE configs[4]: 100k nodes, ~3 neighbours + self
// loop per row on a grid, D = 64, B = 1).  Prints time and SURVEY §8(d) GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lab/c5_lab.hip -o build/c5_lab && build/c5_lab
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);       \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr int D = 64;
static int h_f2i(float f) { int i; memcpy(&i, &f, 4); return i; }
static float h_i2f(int i) { float f; memcpy(&f, &i, 4); return f; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), static_cast<short>(0), static_cast<int>(bytes),
                                             0x00020000);
}

// ---- V1: 16 lanes per row (one float4 each), 4 rows per instruction, 16-row tiles per wave,
// CSR from global memory per row, NS neighbour slots in flight (the product row kernels' shape)
template <int NS, bool XCD = false>
__global__ void __launch_bounds__(256) k_v1(const int* __restrict__ rp, const int2* __restrict__ pr,
                                            const float* __restrict__ x, float* __restrict__ y, int N) {
    const int lane = threadIdx.x & 63, rl = lane >> 4, fg = lane & 15;
    int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    const int ntiles = (N + 15) / 16;
    int tend = ntiles;
    if (XCD) {  // XCD-aware: the blocks of XCD b % 8 walk chunk b % 8 of the tiles
        const int xb = blockIdx.x % 8, k = blockIdx.x / 8, nbx = (gridDim.x - xb + 7) / 8, chunk = (ntiles + 7) / 8;
        wave = xb * chunk + k * 4 + (threadIdx.x >> 6);
        nw = nbx * 4;
        tend = min(ntiles, xb * chunk + chunk);
    }
    const __amdgpu_buffer_rsrc_t xs = rsrc(x, N * 256u), ys = rsrc(y, N * 256u);
    for (int t = wave; t < tend; t += nw) {
        int e0[4], e1[4];
        for (int k = 0; k < 4; ++k) {
            const int r = min(16 * t + 4 * k + rl, N - 1);
            e0[k] = rp[r];
            e1[k] = 16 * t + 4 * k + rl < N ? rp[r + 1] : e0[k];
        }
        f32x4 acc[4] = {};
        for (int s0 = 0; s0 < 6; s0 += NS) {
            int2 c[4][NS];
            f32x4 v[4][NS];
            for (int k = 0; k < 4; ++k)
                for (int s = 0; s < NS; ++s) c[k][s] = e0[k] + s0 + s < e1[k] ? pr[e0[k] + s0 + s] : int2{0, 0};
            for (int k = 0; k < 4; ++k)
                for (int s = 0; s < NS; ++s)
                    v[k][s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                            xs, e0[k] + s0 + s < e1[k] ? c[k][s].x * 256u + 16u * fg : 0xFFFFFFF0u, 0, 0));
            for (int k = 0; k < 4; ++k)
                for (int s = 0; s < NS; ++s) acc[k] += __int_as_float(c[k][s].y) * v[k][s];
        }
        for (int k = 0; k < 4; ++k) {
            const int r = 16 * t + 4 * k + rl;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, acc[k]),
                                                   ys, r < N ? r * 256u + 16u * fg : 0xFFFFFFF0u, 0, 0);
        }
    }
}

// ---- V2: lane = feature, a wave owns RW consecutive rows; the rows' CSR range is contiguous
// and read with scalar loads (wave-uniform), every neighbour row is one 256-byte dword load
// with a scalar base; all RW rows' loads in flight before the first add
template <int RW, int MAXE>
__global__ void __launch_bounds__(256) k_v2(const int* __restrict__ rp, const int2* __restrict__ pr,
                                            const float* __restrict__ x, float* __restrict__ y, int N) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)), nw = gridDim.x * 4;
    const __amdgpu_buffer_rsrc_t xs = rsrc(x, N * 256u), ys = rsrc(y, N * 256u);
    for (int r0 = wave * RW; r0 < N; r0 += nw * RW) {
        const int E0 = __builtin_amdgcn_readfirstlane(rp[r0]);
        const int ne = __builtin_amdgcn_readfirstlane(rp[min(r0 + RW, N)]) - E0;
        float v[MAXE];
        int2 c[MAXE];
#pragma unroll
        for (int e = 0; e < MAXE; ++e) c[e] = e < ne ? pr[E0 + e] : int2{0, 0};
#pragma unroll
        for (int e = 0; e < MAXE; ++e)
            v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                 xs, e < ne ? 4u * lane : 0xFFFFFFF0u, __builtin_amdgcn_readfirstlane(c[e].x) * 256u, 0));
        // entries are in row order (every row has its self loop): flush at each row end
        int row = r0;
        int rend = __builtin_amdgcn_readfirstlane(rp[row + 1]) - E0;
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < MAXE; ++k) {
            if (k < ne) {
                a = fmaf(__int_as_float(c[k].y), v[k], a);
                if (k + 1 == rend) {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a), ys, 4u * lane, row * 256u, 0);
                    a = 0.f;
                    ++row;
                    rend = row < N ? __builtin_amdgcn_readfirstlane(rp[row + 1]) - E0 : 0;
                }
            }
        }
        // rows past MAXE entries (not in this graph) would need a tail loop
    }
}


// ---- V3: cluster-staged gather.  The host cuts the graph into clusters of <= C nodes (BFS
// balls); a workgroup stages its cluster's rows AND their halo (neighbours outside the
// cluster) in LDS once — each x row is read ~(C + halo) / C times instead of once per edge —
// then aggregates every member row from LDS with a cluster-local CSR.
template <int MAXR>
__global__ void __launch_bounds__(256) k_v3(const int* __restrict__ cl_off, const int* __restrict__ cl_rows,
                                            const int* __restrict__ cl_nm, const int* __restrict__ mp0,
                                            const int* __restrict__ lrp, const int2* __restrict__ le,
                                            const float* __restrict__ x, float* __restrict__ y, int N) {
    __shared__ f32x4 rows[MAXR][16];
    const int c = blockIdx.x, tid = threadIdx.x, rl = tid >> 4, fg = tid & 15;
    const int r0 = cl_off[c], nr = cl_off[c + 1] - r0, nm = cl_nm[c], p0 = mp0[c];
    const __amdgpu_buffer_rsrc_t xs = rsrc(x, N * 256u), ys = rsrc(y, N * 256u);
    constexpr int PER = MAXR / 16;
    f32x4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int s = 16 * i + rl;
        const int g = s < nr ? cl_rows[r0 + s] : 0;
        v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xs, s < nr ? g * 256u + 16u * fg : 0xFFFFFFF0u, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) rows[16 * i + rl][fg] = v[i];
    __syncthreads();
    for (int m = rl; m < nm; m += 16) {
        const int e0 = lrp[p0 + m], e1 = lrp[p0 + m + 1];
        f32x4 acc = {};
        for (int e = e0; e < e1; ++e) {
            const int2 t = le[e];
            acc += __int_as_float(t.y) * rows[t.x][fg];
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, acc), ys,
                                               cl_rows[r0 + m] * 256u + 16u * fg, 0, 0);
    }
}


// ---- L2 read-bandwidth probe: every wave reads ITER b128 wave-loads from a region small
// enough to stay L2-resident.  ROWS = false: 1 KB contiguous per wave-load; ROWS = true: four
// pseudo-random 256-byte rows per wave-load (16 lanes each, the gather's shape).
template <bool ROWS, int ITER>
__global__ void __launch_bounds__(256) k_l2bw(const float* __restrict__ buf, uint32_t nrows, float* __restrict__ out) {
    const int lane = threadIdx.x & 63, rl = lane >> 4, fg = lane & 15;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t bs = rsrc(buf, nrows * 256u);
    f32x4 acc = {};
    uint32_t h = wave * 2654435761u + 12345u;
#pragma unroll 8
    for (int i = 0; i < ITER; ++i) {
        h = h * 1664525u + 1013904223u;
        uint32_t off;
        if (ROWS) {
            const uint32_t r = ((h >> 8) + rl * 40503u * (h | 1u)) % nrows;
            off = r * 256u + 16u * fg;
        } else {
            const uint32_t r = (h >> 8) % (nrows / 4);
            off = r * 1024u + 16u * lane;
        }
        acc += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(bs, off, 0, 0));
    }
    if (acc[0] == 1234.5f) out[0] = acc[1];
}

__global__ void __launch_bounds__(256) k_copy(const f32x4* __restrict__ s, f32x4* __restrict__ d, int n4) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) d[i] = s[i];
}

template <typename F>
float timeit(F f, int iters) {
    for (int i = 0; i < 3; ++i) f();
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / iters;
}

int main() {
    const int N = 100000, W = 317;
    // grid graph: right and down neighbours, a random 75 % of them kept (~3 neighbours per
    // node) + self loops; gcn normalisation
    std::mt19937 rng(0);
    std::vector<std::vector<int>> adj(N);
    for (int i = 0; i < N; ++i) {
        if ((i % W) + 1 < W && i + 1 < N && (rng() % 4) != 0) { adj[i].push_back(i + 1); adj[i + 1].push_back(i); }
        if (i + W < N && (rng() % 4) != 0) { adj[i].push_back(i + W); adj[i + W].push_back(i); }
    }
    std::vector<int> rp(N + 1, 0);
    std::vector<int> col;
    std::vector<float> deg(N);
    for (int i = 0; i < N; ++i) deg[i] = 1.f + adj[i].size();
    std::vector<int2> pr;
    for (int i = 0; i < N; ++i) {
        std::sort(adj[i].begin(), adj[i].end());
        for (int j : adj[i]) pr.push_back(int2{j, h_f2i(1.f / std::sqrt(deg[i] * deg[j]))});
        pr.push_back(int2{i, h_f2i(1.f / deg[i])});
        rp[i + 1] = static_cast<int>(pr.size());
    }
    const int nnz = rp[N];
    printf("N %d nnz %d (%.2f per row)\n", N, nnz, double(nnz) / N);
    int *d_rp;
    int2* d_pr;
    float *d_x, *d_y;
    CK(hipMalloc(&d_rp, 4 * (N + 1)));
    CK(hipMalloc(&d_pr, 8 * nnz));
    CK(hipMalloc(&d_x, 4ull * N * D));
    CK(hipMalloc(&d_y, 4ull * N * D));
    CK(hipMemcpy(d_rp, rp.data(), 4 * (N + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_pr, pr.data(), 8 * nnz, hipMemcpyHostToDevice));
    std::vector<float> hx(size_t(N) * D);
    for (auto& v : hx) v = float(rng() % 2001) / 1000.f - 1.f;
    CK(hipMemcpy(d_x, hx.data(), 4ull * N * D, hipMemcpyHostToDevice));
    // reference on the host
    std::vector<float> ref(size_t(N) * D, 0.f), hy(size_t(N) * D);
    for (int r = 0; r < N; ++r)
        for (int e = rp[r]; e < rp[r + 1]; ++e)
            for (int f = 0; f < D; ++f) ref[size_t(r) * D + f] += h_i2f(pr[e].y) * hx[size_t(pr[e].x) * D + f];
    const double bytes = 8.0 * N * D + 4.0 * (N + 1) + 8.0 * nnz;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto check = [&](const char* name, float us) {
        CK(hipMemcpy(hy.data(), d_y, 4ull * N * D, hipMemcpyDeviceToHost));
        double err = 0;
        for (size_t i = 0; i < hy.size(); ++i) err = std::max(err, double(std::fabs(hy[i] - ref[i])));
        printf("%-28s %8.2f us  %7.1f GB/s  maxerr %.2e\n", name, us, bytes / us / 1e3, err);
        CK(hipMemset(d_y, 0, 4ull * N * D));
    };
    const int iters = 200;
    {
        const int n4 = N * D / 4;
        float us = timeit([&] { k_copy<<<cus * 8, 256>>>((const f32x4*)d_x, (f32x4*)d_y, n4); }, iters);
        printf("%-28s %8.2f us  %7.1f GB/s (read + write)\n", "copy", us, 8.0 * N * D / us / 1e3);
    }

    {
        float* d_o;
        CK(hipMalloc(&d_o, 64));
        for (uint32_t nrows : {4096u, 8192u, 65536u}) {  // 1 MB, 2 MB (L2-resident per XCD), 16 MB
            constexpr int IT = 256;
            const int g = cus * 8;
            const double b = double(g) * 4 * IT * 1024;
            float us = timeit([&] { k_l2bw<false, IT><<<g, 256>>>(d_x, nrows, d_o); }, 50);
            printf("l2 probe contiguous %6u KB   %8.2f us  %7.1f GB/s\n", nrows / 4, us, b / us / 1e3);
            us = timeit([&] { k_l2bw<true, IT><<<g, 256>>>(d_x, nrows, d_o); }, 50);
            printf("l2 probe 256B rows  %6u KB   %8.2f us  %7.1f GB/s\n", nrows / 4, us, b / us / 1e3);
        }
    }
    const int t16 = (N + 15) / 16;
    for (int g : {t16 / 4, cus * 4, cus * 8}) {
        char nm[64];
        snprintf(nm, sizeof nm, "v1 ns3 grid %d", g);
        check(nm, timeit([&] { k_v1<3><<<g, 256>>>(d_rp, d_pr, d_x, d_y, N); }, iters));
        snprintf(nm, sizeof nm, "v1 ns6 grid %d", g);
        check(nm, timeit([&] { k_v1<6><<<g, 256>>>(d_rp, d_pr, d_x, d_y, N); }, iters));
        snprintf(nm, sizeof nm, "v1x ns3 grid %d", g);
        check(nm, timeit([&] { k_v1<3, true><<<g, 256>>>(d_rp, d_pr, d_x, d_y, N); }, iters));
        snprintf(nm, sizeof nm, "v1x ns6 grid %d", g);
        check(nm, timeit([&] { k_v1<6, true><<<g, 256>>>(d_rp, d_pr, d_x, d_y, N); }, iters));
    }
    for (int g : {cus * 4, cus * 8, cus * 16}) {
        char nm[64];
        snprintf(nm, sizeof nm, "v2 rw4 grid %d", g);
        check(nm, timeit([&] { k_v2<4, 24><<<g, 256>>>(d_rp, d_pr, d_x, d_y, N); }, iters));
        snprintf(nm, sizeof nm, "v2 rw8 grid %d", g);
        check(nm, timeit([&] { k_v2<8, 40><<<g, 256>>>(d_rp, d_pr, d_x, d_y, N); }, iters));
    }

    // ---- V3: BFS clusters of <= C nodes, their halos, cluster-local CSR
    for (int C : {128}) {
        std::vector<int> cid(N, -1), order;
        std::vector<int> cl_off{0}, cl_rows, cl_nm, mp0, lrp{0};
        std::vector<int2> le;
        int ncl = 0, maxr = 0;
        std::vector<int> q;
        std::vector<int> loc(N, -1);
        for (int s0 = 0; s0 < N; ++s0) {
            if (cid[s0] >= 0) continue;
            std::vector<int> mem;
            q.assign(1, s0);
            cid[s0] = ncl;
            for (size_t h = 0; h < q.size() && (int)mem.size() < C; ++h) {
                const int u = q[h];
                mem.push_back(u);
                for (int e = rp[u]; e < rp[u + 1]; ++e) {
                    const int w = pr[e].x;
                    if (cid[w] < 0 && (int)q.size() < C) { cid[w] = ncl; q.push_back(w); }
                }
            }
            for (size_t h = mem.size(); h < q.size(); ++h) cid[q[h]] = -1;  // queued past C: released
            std::sort(mem.begin(), mem.end());
            std::vector<int> halo;
            for (int u : mem) loc[u] = 0;
            for (int u : mem)
                for (int e = rp[u]; e < rp[u + 1]; ++e)
                    if (cid[pr[e].x] != ncl) halo.push_back(pr[e].x);
            std::sort(halo.begin(), halo.end());
            halo.erase(std::unique(halo.begin(), halo.end()), halo.end());
            for (size_t i = 0; i < mem.size(); ++i) loc[mem[i]] = (int)i;
            for (size_t i = 0; i < halo.size(); ++i) loc[halo[i]] = (int)(mem.size() + i);
            mp0.push_back((int)lrp.size() - 1);
            for (int u : mem) {
                for (int e = rp[u]; e < rp[u + 1]; ++e) le.push_back(int2{loc[pr[e].x], pr[e].y});
                lrp.push_back((int)le.size());
            }
            cl_rows.insert(cl_rows.end(), mem.begin(), mem.end());
            cl_rows.insert(cl_rows.end(), halo.begin(), halo.end());
            cl_off.push_back((int)cl_rows.size());
            cl_nm.push_back((int)mem.size());
            maxr = std::max(maxr, (int)(mem.size() + halo.size()));
            ++ncl;
        }
        printf("C %d: %d clusters, staged rows %zu (%.2f x N), max rows per cluster %d\n", C, ncl, cl_rows.size(),
               double(cl_rows.size()) / N, maxr);
        int *d_off, *d_rows, *d_nm, *d_mp0, *d_lrp;
        int2* d_le;
        CK(hipMalloc(&d_off, 4 * cl_off.size()));
        CK(hipMalloc(&d_rows, 4 * cl_rows.size()));
        CK(hipMalloc(&d_nm, 4 * cl_nm.size()));
        CK(hipMalloc(&d_mp0, 4 * mp0.size()));
        CK(hipMalloc(&d_lrp, 4 * lrp.size()));
        CK(hipMalloc(&d_le, 8 * le.size()));
        CK(hipMemcpy(d_off, cl_off.data(), 4 * cl_off.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_rows, cl_rows.data(), 4 * cl_rows.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_nm, cl_nm.data(), 4 * cl_nm.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_mp0, mp0.data(), 4 * mp0.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_lrp, lrp.data(), 4 * lrp.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_le, le.data(), 8 * le.size(), hipMemcpyHostToDevice));
        char nm[64];
        snprintf(nm, sizeof nm, "v3 C %d", C);
        if (maxr <= 256)
            check(nm, timeit([&] { k_v3<256><<<ncl, 256>>>(d_off, d_rows, d_nm, d_mp0, d_lrp, d_le, d_x, d_y, N); }, iters));
        else if (maxr <= 384)
            check(nm, timeit([&] { k_v3<384><<<ncl, 256>>>(d_off, d_rows, d_nm, d_mp0, d_lrp, d_le, d_x, d_y, N); }, iters));
        else
            printf("v3 C %d: %d rows do not fit\n", C, maxr);
    }
    return 0;
}
