// K5+K6+K7: fused GCN layer forward / backward on gfx950.
//
// Layout: node features fp32 [B][N][D], one single-graph CSR shared by all B
// windows (row r = b*N + n gathers rows b*N + col[e]).  When the CSR is small
// (L-TOWN-A: 20 KB) every workgroup stages it in LDS once and then walks it from
// there; large graphs (C5, 100k nodes) read it from L2.
//
// Work unit: a 16-row "wave tile" owned by ONE 64-lane wavefront.  The layer is
// computed transposed, y^T (D x 16 rows) = W (D x D) * (Ahat x)^T, on
// v_mfma_f32_16x16x4_f32 (exact fp32).  With the K index permuted as
// k = fk(ks, q) = 16*(ks>>2) + 4q + (ks&3), lane (j, q) of the wave gathers exactly
// the B-operand fragment it needs — features {16a + 4q .. 16a + 4q + 3} of row j —
// as float4 loads of the neighbour rows, and the accumulator comes out in the same
// per-lane layout, so the forward needs no LDS for operands or for the store:
//   1. CSR segmented reduce of row j over its entries in order (fp32 fma), 4 float4
//      loads per neighbour per lane (D = 64), neighbour rows are L2-resident;
//   2. D/16 x D/4 MFMAs with W held in registers (A operand), bias as the initial
//      accumulator;
//   3. ReLU / dropout epilogue and float4 row stores (each row's 256 B written by
//      four lanes of one instruction group).
// Waves never wait for each other inside the tile loop.
#include <algorithm>
#include "common.h"
#include "reduce.h"

namespace {

constexpr int kWaves = 8;      // waves per workgroup
constexpr int kTileRows = 16;  // rows per wave tile (MFMA N)
constexpr int64_t kCsrLdsMax = 48 * 1024;

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int fk(int ks, int q) { return 16 * (ks >> 2) + 4 * q + (ks & 3); }

template <int D>
struct Geo {
    static constexpr int A4 = D / 16;  // float4 groups per lane per row
    static constexpr int KS = D / 4;   // k-steps of one contraction
    static constexpr int MT = D / 16;  // 16-row output tiles
    static constexpr int S = D + 4;    // padded LDS row stride (floats)
};

// XCD-aware tile schedule.  Workgroups are dealt round-robin over the 8 XCDs, so
// blocks b and b+8 share one L2 (MI355X_MICROARCH.md, dispatch/XCD placement).  The
// tile range is cut into 8 contiguous chunks and the blocks of XCD group x = b % 8
// stride over chunk x: a window's rows (and the neighbour rows they gather) then
// stay in one L2 instead of being fetched into all eight.  Placement only changes
// speed: every tile is still visited exactly once for any dispatch order.
struct TileRange {
    int64_t first, end, stride;
};
__device__ __forceinline__ TileRange xcd_tiles(int64_t ntiles, int wave, int waves) {
    const int64_t G = gridDim.x, b = blockIdx.x;
    if (G < 8) return TileRange{b * waves + wave, ntiles, G * waves};
    const int64_t x = b % 8, k = b / 8;
    const int64_t nbx = (G - x + 7) / 8;
    const int64_t chunk = (ntiles + 7) / 8;
    const int64_t begin = x * chunk, end = min(ntiles, begin + chunk);
    return TileRange{begin + k * waves + wave, end, nbx * waves};
}

struct Csr {
    const int32_t* rp;
    const int32_t* col;
    const float* w;
};

// Stage rowptr / col / w into LDS (dynamic shared memory) for the whole block.
__device__ __forceinline__ Csr stage_csr(char* smem, const int32_t* __restrict__ rowptr,
                                         const int32_t* __restrict__ col, const float* __restrict__ w, int64_t N) {
    int32_t* srp = reinterpret_cast<int32_t*>(smem);
    const int32_t nnz = rowptr[N];
    int32_t* scol = srp + ((N + 1 + 3) & ~3LL);
    float* sw = reinterpret_cast<float*>(scol + ((nnz + 3) & ~3));
    for (int64_t i = threadIdx.x; i <= N; i += blockDim.x) srp[i] = rowptr[i];
    for (int32_t i = threadIdx.x; i < nnz; i += blockDim.x) {
        scol[i] = col[i];
        sw[i] = w[i];
    }
    __syncthreads();
    return Csr{srp, scol, sw};
}

// Coalesced row gather ("16 lanes per row"): lane (rl = lane>>4, fg = lane&15) owns
// feature float4 fg of rows 4k + rl of an 8-row group; each wave-instruction reads
// four whole 4*D-byte rows.  Two rows x two neighbours in flight per lane.  Row r sums
// w_e * src[b*N + col_e] over its CSR entries in order (fp32 fma).  MASK: gathered
// values are dy * scale * [m > 0] (ReLU/dropout backward of the gathered tensor).
// Measured on MI355X (tools/spmm_lab.hip, L-TOWN-A shape, B = 256): 4.3-4.5 TB/s for
// this layout vs 3.0 TB/s for quarter-row lanes; stream copy 6.4 TB/s.
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};

template <int D, bool MASK, typename Hook = NoHook>
__device__ __forceinline__ void gather8(const Csr& g, const float* __restrict__ src, const float* __restrict__ msk,
                                        float mscale, int64_t rbase, int64_t R, int64_t N, int lane,
                                        f32x4 (&acc)[2], Hook&& hook = Hook{}) {
    constexpr int LPR = D / 4;  // lanes per row
    constexpr int RPI = 64 / LPR;  // rows per instruction
    const int rl = lane / LPR, fg = lane % LPR;
    int e0[2], e1[2];
    int64_t off[2];
    int maxd = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int64_t r = rbase + RPI * k + rl;
        if (r < R) {
            const int64_t b = r / N, n = r - b * N;
            e0[k] = g.rp[n];
            e1[k] = g.rp[n + 1];
            off[k] = b * N * D + 4 * fg;
        } else {
            e0[k] = e1[k] = 0;
            off[k] = 4 * fg;
        }
        maxd = max(maxd, e1[k] - e0[k]);
    }
    // wave-uniform trip count: the hook (MFMA) must run with every lane active
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) maxd = max(maxd, __shfl_xor(maxd, o));
    maxd = __builtin_amdgcn_readfirstlane(maxd);
    for (int d = 0; d < maxd; d += 2) {
        f32x4 v[2][2];
        float ww[2][2];
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int e = e0[k] + d + u;
                const bool ok = e < e1[k];
                const int32_t s = ok ? g.col[e] : 0;
                ww[k][u] = ok ? g.w[e] : 0.f;
                const int64_t o = off[k] + static_cast<int64_t>(s) * D;
                v[k][u] = ld4(src + o);
                if constexpr (MASK) {
                    const f32x4 m = ld4(msk + o);
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[k][u][i] = m[i] > 0.f ? v[k][u][i] * mscale : 0.f;
                }
            }
        hook();  // independent work (e.g. the previous tile's MFMAs) under the load latency
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[k][i] = fmaf(ww[k][u], v[k][u][i], acc[k][i]);
    }
}

// Gather the 16-row tile at r0 into tl[row][feature] (row stride S).
template <int D, bool MASK, typename Hook = NoHook>
__device__ __forceinline__ void gather_tile(const Csr& g, const float* __restrict__ src,
                                            const float* __restrict__ msk, float mscale, int64_t r0, int64_t R,
                                            int64_t N, int lane, float* __restrict__ tl, Hook&& hook = Hook{}) {
    constexpr int LPR = D / 4, RPI = 64 / LPR;
    const int rl = lane / LPR, fg = lane % LPR;
#pragma unroll
    for (int pass = 0; pass < kTileRows / (2 * RPI); ++pass) {
        f32x4 acc[2];
        gather8<D, MASK>(g, src, msk, mscale, r0 + pass * 2 * RPI, R, N, lane, acc, hook);
#pragma unroll
        for (int k = 0; k < 2; ++k) st4(tl + (pass * 2 * RPI + RPI * k + rl) * Geo<D>::S + 4 * fg, acc[k]);
    }
}

// Store the 16-row tile tl[row][feature] to dst rows r0.. as whole rows.
template <int D>
__device__ __forceinline__ void store_tile(const float* __restrict__ tl, float* __restrict__ dst, int64_t r0,
                                           int64_t R, int lane) {
    constexpr int LPR = D / 4, RPI = 64 / LPR;
    const int rl = lane / LPR, fg = lane % LPR;
#pragma unroll
    for (int k = 0; k < kTileRows / RPI; ++k) {
        const int row = RPI * k + rl;
        if (r0 + row < R) st4(dst + (r0 + row) * D + 4 * fg, ld4(tl + row * Geo<D>::S + 4 * fg));
    }
}

// ------------------------------------------------------------------ forward
// y^T = W (Ahat x)^T: B operand = the gathered tile (LDS), A operand = W (LDS).
// Software pipeline per wave: the tile is double-buffered in LDS and the MFMA
// chunks of tile i run between issuing and consuming each gather round of tile
// i+1, so the matrix pipe works under the memory latency of the next gather.
constexpr int kFwdWaves = 12;  // one 768-thread workgroup per CU: 12 x 8.7 KB tiles + W + CSR in LDS

template <int D, bool CSR_LDS>
__global__ void __launch_bounds__(64 * kFwdWaves)
k_gcn_fwd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
          const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
          float* __restrict__ y, int64_t N, int64_t R, int64_t ntiles, int flags, float p_drop, float dscale,
          uint64_t seed, uint32_t salt, int64_t csr_bytes) {
    using G = Geo<D>;
    constexpr int TILE = kTileRows * G::S;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* wl = reinterpret_cast<float*>(smem + (CSR_LDS ? csr_bytes : 0));  // W [out][in], stride S
    float* tiles = wl + D * G::S;
    for (int i = threadIdx.x; i < D * D / 4; i += blockDim.x)
        st4(wl + (i / (D / 4)) * G::S + 4 * (i % (D / 4)), ld4(W + 4 * i));
    const Csr g = CSR_LDS ? stage_csr(smem, rowptr, col, wgt, N) : Csr{rowptr, col, wgt};
    if (!CSR_LDS) __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    float* buf0 = tiles + wave * 2 * TILE;
    const uint32_t key = lg_dropout_key(seed, salt);
    f32x4 bv[G::MT];
#pragma unroll
    for (int mt = 0; mt < G::MT; ++mt)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) bv[mt][reg] = (flags & LG_F_BIAS) ? bias[16 * mt + 4 * q + reg] : 0.f;

    const TileRange tr = xcd_tiles(ntiles, wave, kFwdWaves);
    if (tr.first < tr.end) gather_tile<D, false>(g, x, nullptr, 1.f, tr.first * kTileRows, R, N, lane, buf0);
    int cur = 0;
    for (int64_t tile = tr.first; tile < tr.end; tile += tr.stride, cur ^= 1) {
        float* cb = buf0 + cur * TILE;
        float* nb = buf0 + (cur ^ 1) * TILE;
        wave_lds_sync();
        f32x4 o[G::MT];
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) o[mt] = bv[mt];
        int chunk = 0;
        auto mfma_chunk = [&]() {
            if (chunk < G::KS / 4) {
                const f32x4 bt = ld4(cb + j * G::S + 16 * chunk + 4 * q);  // (Ahat x)[row j][16c + 4q + i]
#pragma unroll
                for (int mt = 0; mt < G::MT; ++mt) {
                    const f32x4 wa = ld4(wl + (16 * mt + j) * G::S + 16 * chunk + 4 * q);  // W[16mt + j][..]
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[mt] = mfma(wa[i], bt[i], o[mt]);
                }
                ++chunk;
            }
        };
        const int64_t next = tile + tr.stride;
        if (next < tr.end) gather_tile<D, false>(g, x, nullptr, 1.f, next * kTileRows, R, N, lane, nb, mfma_chunk);
        while (chunk < G::KS / 4) mfma_chunk();
        const int64_t r0 = tile * kTileRows, r = r0 + j;
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) {
            f32x4 v = o[mt];
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                float t = v[reg];
                if (flags & LG_F_RELU) t = fmaxf(t, 0.f);
                if (flags & LG_F_DROPOUT) t = lg_dropout(t, p_drop, dscale, key, r * D + 16 * mt + 4 * q + reg);
                v[reg] = t;
            }
            o[mt] = v;
        }
        wave_lds_sync();
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) st4(cb + j * G::S + 16 * mt + 4 * q, o[mt]);
        wave_lds_sync();
        store_tile<D>(cb, y, r0, R, lane);
    }
}

// ------------------------------------------------------------------ backward
// dz = MASK_IN ? dy*scale_in*[y>0] : dy ; t = Ahat^T dz ; dx = t W ; dW += t^T x ; db += sum dz
template <int D, bool MASK_IN, bool CSR_LDS>
__global__ void __launch_bounds__(64 * kWaves, 2)
k_gcn_bwd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
          const float* __restrict__ dy, const float* __restrict__ yv, const float* __restrict__ x,
          const float* __restrict__ W, float* __restrict__ dxo, float* __restrict__ slab, int64_t N, int64_t R,
          int64_t ntiles, int mask_out, float scale_in, float scale_out, int64_t csr_bytes) {
    using G = Geo<D>;
    constexpr int LPR = D / 4, RPI = 64 / LPR;
    constexpr int SW = D + 4;  // W rows in LDS, conflict-free column reads
    constexpr int WBUF = 2 * kTileRows * G::S;
    constexpr int L = D * D + D;
    static_assert(kWaves * WBUF >= L, "reduction buffer must fit in the tile buffers");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Csr g = CSR_LDS ? stage_csr(smem, rowptr, col, wgt, N) : Csr{rowptr, col, wgt};
    float* lds = reinterpret_cast<float*>(smem + (CSR_LDS ? csr_bytes : 0));
    float* wl = lds + kWaves * WBUF;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const int rl = lane / LPR, fg = lane % LPR;
    float* tl = lds + wave * WBUF;      // t tile [row][feature], later dx
    float* xl = tl + kTileRows * G::S;  // x tile [row][feature]
    for (int i = threadIdx.x; i < D * D; i += blockDim.x) wl[(i / D) * SW + (i % D)] = W[i];
    __syncthreads();

    f32x4 dw[G::MT][G::MT];  // dW tile (mo, ni): rows o = 16mo + 4q + reg, cols i = 16ni + j
#pragma unroll
    for (int a = 0; a < G::MT; ++a)
#pragma unroll
        for (int b = 0; b < G::MT; ++b) dw[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dbacc = f32x4{0.f, 0.f, 0.f, 0.f};  // features 4fg..4fg+3, summed over this lane's rows

    const TileRange tr = xcd_tiles(ntiles, wave, kWaves);
    for (int64_t tile = tr.first; tile < tr.end; tile += tr.stride) {
        const int64_t r0 = tile * kTileRows;
        gather_tile<D, MASK_IN>(g, dy, yv, scale_in, r0, R, N, lane, tl);
        // own rows (coalesced): dz for db, x for dW and the output mask
#pragma unroll
        for (int k = 0; k < kTileRows / RPI; ++k) {
            const int row = RPI * k + rl;
            const int64_t r = r0 + row;
            f32x4 xv = f32x4{0.f, 0.f, 0.f, 0.f};
            if (r < R) {
                const int64_t off = r * D + 4 * fg;
                f32x4 dz = ld4(dy + off);
                if constexpr (MASK_IN) {
                    const f32x4 m = ld4(yv + off);
#pragma unroll
                    for (int i = 0; i < 4; ++i) dz[i] = m[i] > 0.f ? dz[i] * scale_in : 0.f;
                }
                dbacc += dz;
                xv = ld4(x + off);
            }
            st4(xl + row * G::S + 4 * fg, xv);
        }
        wave_lds_sync();
        // dW[o][i] += sum_rows t[row][o] x[row][i]   (rows = 4q + kk on the K index)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int row = 4 * q + kk;
            float ta[G::MT], xb[G::MT];
#pragma unroll
            for (int m = 0; m < G::MT; ++m) {
                ta[m] = tl[row * G::S + 16 * m + j];
                xb[m] = xl[row * G::S + 16 * m + j];
            }
#pragma unroll
            for (int mo = 0; mo < G::MT; ++mo)
#pragma unroll
                for (int ni = 0; ni < G::MT; ++ni) dw[mo][ni] = mfma(ta[mo], xb[ni], dw[mo][ni]);
        }
        // dx^T[i][row] = sum_o W[o][i] t[row][o] : A = W^T (LDS), B = t tile (LDS)
        f32x4 o[G::MT];
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) o[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < G::KS / 4; ++a) {
            const f32x4 bt = ld4(tl + j * G::S + 16 * a + 4 * q);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ko = 16 * a + 4 * q + i;
#pragma unroll
                for (int mt = 0; mt < G::MT; ++mt) o[mt] = mfma(wl[ko * SW + 16 * mt + j], bt[i], o[mt]);
            }
        }
        if (mask_out) {
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt) {
                const f32x4 xm = ld4(xl + j * G::S + 16 * mt + 4 * q);
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) o[mt][reg] = xm[reg] > 0.f ? o[mt][reg] * scale_out : 0.f;
            }
        }
        wave_lds_sync();
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) st4(tl + j * G::S + 16 * mt + 4 * q, o[mt]);
        wave_lds_sync();
        store_tile<D>(tl, dxo, r0, R, lane);
        wave_lds_sync();
    }

    // ---- per-block reduction of dW / db (fixed wave order -> deterministic)
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) dbacc[i] += __shfl_xor(dbacc[i], off);
    __syncthreads();
    float* red = lds;  // reuse the tile buffers
    for (int i = threadIdx.x; i < L; i += blockDim.x) red[i] = 0.f;
    for (int wv = 0; wv < kWaves; ++wv) {
        __syncthreads();
        if (wave == wv) {
#pragma unroll
            for (int mo = 0; mo < G::MT; ++mo)
#pragma unroll
                for (int ni = 0; ni < G::MT; ++ni)
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg)
                        red[(16 * mo + 4 * q + reg) * D + 16 * ni + j] += dw[mo][ni][reg];
            if (lane < LPR)
#pragma unroll
                for (int i = 0; i < 4; ++i) red[D * D + 4 * lane + i] += dbacc[i];
        }
    }
    __syncthreads();
    float* out = slab + static_cast<int64_t>(blockIdx.x) * L;
    for (int i = threadIdx.x; i < L; i += blockDim.x) out[i] = red[i];
}

// ------------------------------------------------------------------ plain propagate
template <int D, bool CSR_LDS>
__global__ void __launch_bounds__(256)
k_spmm(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
       const float* __restrict__ x, float* __restrict__ y, int64_t N, int64_t R, int64_t ntiles) {
    constexpr int LPR = D / 4, RPI = 64 / LPR;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Csr g = CSR_LDS ? stage_csr(smem, rowptr, col, wgt, N) : Csr{rowptr, col, wgt};
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int rl = lane / LPR, fg = lane % LPR;
    const TileRange tr = xcd_tiles(ntiles, wave, 4);  // a "tile" here is 2*RPI rows
    for (int64_t tile = tr.first; tile < tr.end; tile += tr.stride) {
        const int64_t rb = tile * 2 * RPI;
        f32x4 acc[2];
        gather8<D, false>(g, x, nullptr, 1.f, rb, R, N, lane, acc);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int64_t r = rb + RPI * k + rl;
            if (r < R) st4(y + r * D + 4 * fg, acc[k]);
        }
    }
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// LDS bytes to stage the CSR (rowptr + col + w, each padded to 16 B), or 0 if too big.
inline int64_t csr_lds_bytes(int64_t N, int64_t nnz_cap) {
    const int64_t b = 4 * ((N + 1 + 3) & ~3LL) + 8 * ((nnz_cap + 3) & ~3LL);
    return b <= kCsrLdsMax ? b : 0;
}

int bwd_grid(int64_t ntiles, int64_t dyn_lds) {
    const int64_t want = ceil_div(ntiles, kWaves);
    const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(2, (160 * 1024) / dyn_lds));
    const int64_t cap = per_cu * static_cast<int64_t>(lg_num_cus());
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(want, cap)));
}

int bwd_grid_max() { return 2 * lg_num_cus(); }

}  // namespace

extern "C" int lg_gcn_fwd(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, const float* W,
                          const float* bias, float* y, int64_t B, int64_t N, int64_t D, int64_t nnz_cap, int flags,
                          float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream) {
    if (B < 0 || N <= 0 || nnz_cap < 0) return LG_EINVAL;
    if (!rowptr || !col || !w || !x || !W || !y || x == y) return LG_EINVAL;
    if ((flags & LG_F_BIAS) && !bias) return LG_EINVAL;
    if ((flags & LG_F_DROPOUT) && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    const int64_t R = B * N;
    if (R == 0) return LG_OK;
    const int64_t ntiles = ceil_div(R, kTileRows);
    const int64_t csr = csr_lds_bytes(N, nnz_cap);
    const int64_t dyn = csr + static_cast<int64_t>(sizeof(float)) * (D + 2 * kFwdWaves * kTileRows) * (D + 4);
    const unsigned grid = static_cast<unsigned>(
        std::max<int64_t>(1, std::min<int64_t>(ceil_div(ntiles, kFwdWaves), lg_num_cus())));
    const float scale = (flags & LG_F_DROPOUT) ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
#define LG_FWD(DD, CL)                                                                                        \
    do {                                                                                                      \
        if (dyn > 64 * 1024 &&                                                                                \
            hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gcn_fwd<DD, CL>),                            \
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(dyn)) != hipSuccess) \
            return LG_EHIP;                                                                                   \
        k_gcn_fwd<DD, CL><<<grid, 64 * kFwdWaves, dyn, s>>>(rowptr, col, w, x, W, bias, y, N, R, ntiles, flags, \
                                                        dropout_p, scale, seed, salt, csr);                   \
    } while (0)
    if (D == 64) {
        if (csr) LG_FWD(64, true); else LG_FWD(64, false);
    } else {
        if (csr) LG_FWD(32, true); else LG_FWD(32, false);
    }
#undef LG_FWD
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_spmm(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, float* y,
                       int64_t B, int64_t N, int64_t D, int64_t nnz_cap, lg_stream_t stream) {
    if (B < 0 || N <= 0 || nnz_cap < 0) return LG_EINVAL;
    if (!rowptr || !col || !w || !x || !y || x == y) return LG_EINVAL;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    const int64_t R = B * N;
    if (R == 0) return LG_OK;
    const int64_t ntiles = ceil_div(R, 2 * (64 / (D / 4)));
    const int64_t lds = csr_lds_bytes(N, nnz_cap);
    const int64_t per_cu = lds ? std::max<int64_t>(1, std::min<int64_t>(8, (160 * 1024) / lds)) : 8;
    const unsigned grid =
        static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(ntiles, 4), per_cu * lg_num_cus())));
    hipStream_t s = lg_stream(stream);
#define LG_SPMM(DD, CL) k_spmm<DD, CL><<<grid, 256, CL ? lds : 0, s>>>(rowptr, col, w, x, y, N, R, ntiles)
    if (D == 64) {
        if (lds) LG_SPMM(64, true); else LG_SPMM(64, false);
    } else {
        if (lds) LG_SPMM(32, true); else LG_SPMM(32, false);
    }
#undef LG_SPMM
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int64_t lg_gcn_bwd_workspace_bytes(int64_t D) {
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    return static_cast<int64_t>(bwd_grid_max()) * (D * D + D) * static_cast<int64_t>(sizeof(float));
}

extern "C" int lg_gcn_bwd(const int32_t* rowptr_t, const int32_t* col_t, const float* w_t, const float* dy,
                          const float* y, const float* x, const float* W, float* dx_out, float* dW, float* db,
                          int64_t B, int64_t N, int64_t D, int64_t nnz_cap, int flags, float scale_in,
                          float scale_out, void* workspace, lg_stream_t stream) {
    if (B < 0 || N <= 0 || nnz_cap < 0) return LG_EINVAL;
    if (!rowptr_t || !col_t || !w_t || !dy || !x || !W || !dx_out || !dW || !workspace) return LG_EINVAL;
    if ((flags & LG_F_MASK_IN) && !y) return LG_EINVAL;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    const int64_t R = B * N;
    hipStream_t s = lg_stream(stream);
    const int64_t ntiles = ceil_div(R, kTileRows);
    float* slab = static_cast<float*>(workspace);
    const int mask_out = (flags & LG_F_MASK_OUT) ? 1 : 0;
    const bool mask_in = (flags & LG_F_MASK_IN) != 0;
    const int64_t csr = csr_lds_bytes(N, nnz_cap);
    const int64_t tiles_lds = static_cast<int64_t>(sizeof(float)) *
                              (kWaves * 2 * kTileRows * (D + 4) + D * (D + 4));
    const int grid = bwd_grid(ntiles, csr + tiles_lds);
#define LG_BWD(DD, MI, CL)                                                                                        \
    do {                                                                                                          \
        const int64_t dyn = (CL ? csr : 0) + tiles_lds;                                                           \
        if (dyn > 64 * 1024 &&                                                                                    \
            hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gcn_bwd<DD, MI, CL>),                            \
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(dyn)) != hipSuccess) \
            return LG_EHIP;                                                                                       \
        k_gcn_bwd<DD, MI, CL><<<grid, 64 * kWaves, dyn, s>>>(rowptr_t, col_t, w_t, dy, y, x, W, dx_out, slab, N, \
                                                             R, ntiles, mask_out, scale_in, scale_out, csr);      \
    } while (0)
    if (D == 64) {
        if (mask_in) {
            if (csr) LG_BWD(64, true, true); else LG_BWD(64, true, false);
        } else {
            if (csr) LG_BWD(64, false, true); else LG_BWD(64, false, false);
        }
    } else {
        if (mask_in) {
            if (csr) LG_BWD(32, true, true); else LG_BWD(32, true, false);
        } else {
            if (csr) LG_BWD(32, false, true); else LG_BWD(32, false, false);
        }
    }
#undef LG_BWD
    LG_RET_IF_LAUNCH_FAILED();
    const int64_t L = D * D + D;
    int rc = lg_launch_slab_reduce(slab, grid, L, D * D, dW, s);
    if (rc == LG_OK && db) rc = lg_launch_slab_reduce(slab + D * D, grid, L, D, db, s);
    return rc;
}
