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

constexpr int kWaves = 4;      // waves per workgroup
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

// Row j of the tile: acc[a][i] = sum_e w_e * src[(b*N + col_e)][16a + 4q + i]  (in CSR order).
// MASK: the gathered values are dy * scale * [m > 0] (ReLU/dropout backward).
template <int D, bool MASK>
__device__ __forceinline__ void gather_row(const Csr& g, const float* __restrict__ src, const float* __restrict__ msk,
                                           float mscale, int64_t r, bool valid, int64_t N, int q,
                                           f32x4 (&acc)[Geo<D>::A4]) {
#pragma unroll
    for (int a = 0; a < Geo<D>::A4; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (!valid) return;
    const int64_t b = r / N, n = r - b * N;
    const int32_t e0 = g.rp[n], e1 = g.rp[n + 1];
    const float* base = src + b * N * D + 4 * q;
    const float* mbase = MASK ? msk + b * N * D + 4 * q : nullptr;
    int32_t e = e0;
    for (; e + 1 < e1; e += 2) {  // two neighbours in flight
        const int32_t s0 = g.col[e], s1 = g.col[e + 1];
        const float w0 = g.w[e], w1 = g.w[e + 1];
        f32x4 v0[Geo<D>::A4], v1[Geo<D>::A4];
#pragma unroll
        for (int a = 0; a < Geo<D>::A4; ++a) {
            v0[a] = ld4(base + static_cast<int64_t>(s0) * D + 16 * a);
            v1[a] = ld4(base + static_cast<int64_t>(s1) * D + 16 * a);
        }
        if constexpr (MASK) {
#pragma unroll
            for (int a = 0; a < Geo<D>::A4; ++a) {
                const f32x4 m0 = ld4(mbase + static_cast<int64_t>(s0) * D + 16 * a);
                const f32x4 m1 = ld4(mbase + static_cast<int64_t>(s1) * D + 16 * a);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    v0[a][i] = m0[i] > 0.f ? v0[a][i] * mscale : 0.f;
                    v1[a][i] = m1[i] > 0.f ? v1[a][i] * mscale : 0.f;
                }
            }
        }
#pragma unroll
        for (int a = 0; a < Geo<D>::A4; ++a)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[a][i] = fmaf(w1, v1[a][i], fmaf(w0, v0[a][i], acc[a][i]));
    }
    if (e < e1) {
        const int32_t s0 = g.col[e];
        const float w0 = g.w[e];
#pragma unroll
        for (int a = 0; a < Geo<D>::A4; ++a) {
            f32x4 v = ld4(base + static_cast<int64_t>(s0) * D + 16 * a);
            if constexpr (MASK) {
                const f32x4 m = ld4(mbase + static_cast<int64_t>(s0) * D + 16 * a);
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = m[i] > 0.f ? v[i] * mscale : 0.f;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[a][i] = fmaf(w0, v[i], acc[a][i]);
        }
    }
}

// ------------------------------------------------------------------ forward
template <int D, bool CSR_LDS>
__global__ void __launch_bounds__(64 * kWaves, 4)
k_gcn_fwd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
          const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
          float* __restrict__ y, int64_t N, int64_t R, int64_t ntiles, int flags, float p_drop, float dscale,
          uint64_t seed, uint32_t salt, int64_t csr_bytes) {
    using G = Geo<D>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* wl = reinterpret_cast<float*>(smem + (CSR_LDS ? csr_bytes : 0));  // W [out][in], stride S
    for (int i = threadIdx.x; i < D * D / 4; i += blockDim.x) st4(wl + (i / (D / 4)) * G::S + 4 * (i % (D / 4)),
                                                                  ld4(W + 4 * i));
    const Csr g = CSR_LDS ? stage_csr(smem, rowptr, col, wgt, N) : Csr{rowptr, col, wgt};
    if (!CSR_LDS) __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    f32x4 bv[G::MT];
#pragma unroll
    for (int mt = 0; mt < G::MT; ++mt)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) bv[mt][reg] = (flags & LG_F_BIAS) ? bias[16 * mt + 4 * q + reg] : 0.f;

    const TileRange tr = xcd_tiles(ntiles, wave, kWaves);
    for (int64_t tile = tr.first; tile < tr.end; tile += tr.stride) {
        const int64_t r = tile * kTileRows + j;
        const bool valid = r < R;
        f32x4 acc[G::A4];
        gather_row<D, false>(g, x, nullptr, 1.f, r, valid, N, q, acc);
        asm volatile("" ::: "memory");  // keep the W reads below in the loop (no 64-VGPR hoist)
        f32x4 o[G::MT];
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) o[mt] = bv[mt];
#pragma unroll
        for (int a = 0; a < G::KS / 4; ++a)
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt) {
                // A operand W[16mt + j][fk(4a + i, q)] = W[16mt + j][16a + 4q + i]
                const f32x4 wa = ld4(wl + (16 * mt + j) * G::S + 16 * a + 4 * q);
#pragma unroll
                for (int i = 0; i < 4; ++i) o[mt] = mfma(wa[i], acc[a][i], o[mt]);
            }
        if (valid) {
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt) {
                f32x4 v = o[mt];
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) {
                    float t = v[reg];
                    if (flags & LG_F_RELU) t = fmaxf(t, 0.f);
                    if (flags & LG_F_DROPOUT) t = lg_dropout(t, p_drop, dscale, seed, salt, r * D + 16 * mt + 4 * q + reg);
                    v[reg] = t;
                }
                st4(y + r * D + 16 * mt + 4 * q, v);
            }
        }
    }
}

// ------------------------------------------------------------------ backward
// dz = MASK_IN ? dy*scale_in*[y>0] : dy ; t = Ahat^T dz ; dx = t W ; dW += t^T x ; db += sum dz
template <int D, bool MASK_IN, bool CSR_LDS>
__global__ void __launch_bounds__(64 * kWaves)
k_gcn_bwd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
          const float* __restrict__ dy, const float* __restrict__ yv, const float* __restrict__ x,
          const float* __restrict__ W, float* __restrict__ dxo, float* __restrict__ slab, int64_t N, int64_t R,
          int64_t ntiles, int mask_out, float scale_in, float scale_out, int64_t csr_bytes) {
    using G = Geo<D>;
    constexpr int SW = D + 4;               // W rows in LDS, conflict-free column reads
    constexpr int WBUF = 2 * kTileRows * G::S;
    constexpr int L = D * D + D;
    static_assert(kWaves * WBUF >= L, "reduction buffer must fit in the tile buffers");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Csr g = CSR_LDS ? stage_csr(smem, rowptr, col, wgt, N) : Csr{rowptr, col, wgt};
    float* lds = reinterpret_cast<float*>(smem + (CSR_LDS ? csr_bytes : 0));
    float* wl = lds + kWaves * WBUF;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    float* tl = lds + wave * WBUF;   // t tile [row][feature]
    float* xl = tl + kTileRows * G::S;  // x tile [row][feature]
    for (int i = threadIdx.x; i < D * D; i += blockDim.x) wl[(i / D) * SW + (i % D)] = W[i];
    __syncthreads();

    f32x4 dw[G::MT][G::MT];  // dW tile (mo, ni): rows o = 16mo + 4q + reg, cols i = 16ni + j
#pragma unroll
    for (int a = 0; a < G::MT; ++a)
#pragma unroll
        for (int b = 0; b < G::MT; ++b) dw[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dbacc[G::A4];
#pragma unroll
    for (int a = 0; a < G::A4; ++a) dbacc[a] = f32x4{0.f, 0.f, 0.f, 0.f};

    const TileRange tr = xcd_tiles(ntiles, wave, kWaves);
    for (int64_t tile = tr.first; tile < tr.end; tile += tr.stride) {
        const int64_t r = tile * kTileRows + j;
        const bool valid = r < R;
        f32x4 t[G::A4];
        gather_row<D, MASK_IN>(g, dy, yv, scale_in, r, valid, N, q, t);
        f32x4 xv[G::A4];
#pragma unroll
        for (int a = 0; a < G::A4; ++a) {
            xv[a] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (valid) {
                const int64_t off = r * D + 16 * a + 4 * q;
                f32x4 dz = ld4(dy + off);
                if constexpr (MASK_IN) {
                    const f32x4 m = ld4(yv + off);
#pragma unroll
                    for (int i = 0; i < 4; ++i) dz[i] = m[i] > 0.f ? dz[i] * scale_in : 0.f;
                }
                dbacc[a] += dz;
                xv[a] = ld4(x + off);
            }
            st4(tl + j * G::S + 16 * a + 4 * q, t[a]);
            st4(xl + j * G::S + 16 * a + 4 * q, xv[a]);
        }
        // dx^T[i][row] = sum_o W[o][i] t[row][o]  : A = W^T from LDS, B = t (lane-local)
        f32x4 o[G::MT];
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) o[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) {
            const float bt = t[ks >> 2][ks & 3];
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt) o[mt] = mfma(wl[fk(ks, q) * SW + 16 * mt + j], bt, o[mt]);
        }
        if (valid) {
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt) {
                f32x4 v = o[mt];
                if (mask_out) {
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) v[reg] = xv[mt][reg] > 0.f ? v[reg] * scale_out : 0.f;
                }
                st4(dxo + r * D + 16 * mt + 4 * q, v);
            }
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
        wave_lds_sync();
    }

    // ---- per-block reduction of dW / db (fixed wave order -> deterministic)
#pragma unroll
    for (int off = 1; off < 16; off <<= 1)
#pragma unroll
        for (int a = 0; a < G::A4; ++a)
#pragma unroll
            for (int i = 0; i < 4; ++i) dbacc[a][i] += __shfl_xor(dbacc[a][i], off);
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
            if (j == 0)
#pragma unroll
                for (int a = 0; a < G::A4; ++a)
#pragma unroll
                    for (int i = 0; i < 4; ++i) red[D * D + 16 * a + 4 * q + i] += dbacc[a][i];
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
    using G = Geo<D>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Csr g = CSR_LDS ? stage_csr(smem, rowptr, col, wgt, N) : Csr{rowptr, col, wgt};
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const TileRange tr = xcd_tiles(ntiles, wave, 4);
    for (int64_t tile = tr.first; tile < tr.end; tile += tr.stride) {
        const int64_t r = tile * kTileRows + j;
        const bool valid = r < R;
        f32x4 acc[G::A4];
        gather_row<D, false>(g, x, nullptr, 1.f, r, valid, N, q, acc);
        if (valid) {
#pragma unroll
            for (int a = 0; a < G::A4; ++a) st4(y + r * D + 16 * a + 4 * q, acc[a]);
        }
    }
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// LDS bytes to stage the CSR (rowptr + col + w, each padded to 16 B), or 0 if too big.
inline int64_t csr_lds_bytes(int64_t N, int64_t nnz_cap) {
    const int64_t b = 4 * ((N + 1 + 3) & ~3LL) + 8 * ((nnz_cap + 3) & ~3LL);
    return b <= kCsrLdsMax ? b : 0;
}

int bwd_grid(int64_t ntiles) {
    const int64_t want = ceil_div(ntiles, kWaves);
    const int64_t cap = 2 * static_cast<int64_t>(lg_num_cus());
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
    const int64_t dyn = csr + static_cast<int64_t>(sizeof(float)) * D * (D + 4);
    const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(8, (160 * 1024) / dyn));
    const unsigned grid =
        static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(ntiles, kWaves), per_cu * lg_num_cus())));
    const float scale = (flags & LG_F_DROPOUT) ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
#define LG_FWD(DD, CL)                                                                                             \
    k_gcn_fwd<DD, CL><<<grid, 64 * kWaves, dyn, s>>>(rowptr, col, w, x, W, bias, y, N, R, ntiles, flags, dropout_p, \
                                                    scale, seed, salt, csr)
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
    const int64_t ntiles = ceil_div(R, kTileRows);
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
    const int grid = bwd_grid(ntiles);
    float* slab = static_cast<float*>(workspace);
    const int mask_out = (flags & LG_F_MASK_OUT) ? 1 : 0;
    const bool mask_in = (flags & LG_F_MASK_IN) != 0;
    const int64_t csr = csr_lds_bytes(N, nnz_cap);
    const int64_t tiles_lds = static_cast<int64_t>(sizeof(float)) *
                              (kWaves * 2 * kTileRows * (D + 4) + D * (D + 4));
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
