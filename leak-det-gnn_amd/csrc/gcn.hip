// K5+K6+K7: fused GCN layer forward / backward on gfx950.
//
// Layout: node features fp32 [B][N][D], one single-graph CSR shared by all B
// windows (row r = b*N + n gathers rows b*N + col[e]).
//
// Work unit: a 16-row "wave tile" owned by ONE 64-lane wavefront, start to end:
//   1. CSR gather + segmented reduce, D/4 lanes per row, one float4 per lane, rows
//      read as whole 4*D-byte lines (coalesced); up to 4 rows per lane in flight.
//   2. the 16 x D tile goes to the wave's private LDS slice (padded rows),
//   3. 16 x D x D product on MFMA v_mfma_f32_16x16x4_f32 (exact fp32 fma chain),
//   4. epilogue (bias / ReLU / dropout or the backward masks), transposed back
//      through LDS and stored as full rows (1 KiB per wave-instruction at D=64).
// Waves never wait for each other inside the tile loop (no workgroup barrier),
// so the gather of one wave overlaps the MFMA phase of its neighbours.
#include "common.h"
#include "reduce.h"

namespace {

constexpr int kWaves = 4;         // waves per workgroup
constexpr int kTileRows = 16;     // rows per wave tile (MFMA M)

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int D>
struct Geo {
    static constexpr int LPR = D / 4;                 // lanes per row (float4 each)
    static constexpr int RPI = 64 / LPR;              // rows per wave-instruction
    static constexpr int PASSES = kTileRows / RPI;    // row groups per lane per tile
    static constexpr int KQ = D / 4;                  // k-steps per MFMA chain
    static constexpr int NT = D / 16;                 // 16-wide column tiles
    static constexpr int S = D + 4;                   // padded LDS row stride (floats)
    static constexpr int TILE = kTileRows * S;        // floats per wave tile buffer
};

// Gather + segmented reduce of the PASSES rows this lane owns in the tile at r0.
// Row r sums  wgt[e] * load(b*N + col[e])  over its CSR entries in order.
template <int D, bool MASK>
__device__ __forceinline__ void gather_rows(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                            const float* __restrict__ wgt, const float* __restrict__ src,
                                            const float* __restrict__ msk, float mscale, int64_t r0, int64_t R,
                                            int64_t N, int lane, f32x4 (&acc)[Geo<D>::PASSES]) {
    using G = Geo<D>;
    const int rl = lane / G::LPR, fg = lane % G::LPR;
    int beg[G::PASSES], deg[G::PASSES];
    int64_t base[G::PASSES];
    int maxdeg = 0;
#pragma unroll
    for (int p = 0; p < G::PASSES; ++p) {
        acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int64_t r = r0 + p * G::RPI + rl;
        if (r < R) {
            const int64_t b = r / N, n = r - b * N;
            beg[p] = rowptr[n];
            deg[p] = rowptr[n + 1] - beg[p];
            base[p] = b * N;
        } else {
            beg[p] = 0;
            deg[p] = 0;
            base[p] = 0;
        }
        maxdeg = max(maxdeg, deg[p]);
    }
    for (int k = 0; k < maxdeg; ++k) {
#pragma unroll
        for (int p = 0; p < G::PASSES; ++p) {
            if (k < deg[p]) {
                const int32_t s = col[beg[p] + k];
                const float ww = wgt[beg[p] + k];
                const int64_t off = (base[p] + s) * D + 4 * fg;
                f32x4 v = ld4(src + off);
                if constexpr (MASK) {
                    const f32x4 m = ld4(msk + off);
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[i] = m[i] > 0.f ? v[i] * mscale : 0.f;
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[p][i] = fmaf(ww, v[i], acc[p][i]);
            }
        }
    }
}

// ------------------------------------------------------------------ forward
template <int D>
__global__ void __launch_bounds__(64 * kWaves)
k_gcn_fwd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
          const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
          float* __restrict__ y, int64_t N, int64_t R, int64_t ntiles, int flags, float p_drop, float dscale,
          uint64_t seed, uint32_t salt) {
    using G = Geo<D>;
    __shared__ __attribute__((aligned(16))) float lds[kWaves * G::TILE];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* my = lds + wave * G::TILE;
    const int j = lane & 15, q = lane >> 4;
    const int rl = lane / G::LPR, fg = lane % G::LPR;

    // B operand of y = a W^T: B[k][c] = W[c][k]; lane (c = 16n + j, k-group q) keeps
    // W[16n+j][KQ*q .. KQ*q+KQ-1] for the whole kernel.
    float bw[G::NT][G::KQ];
#pragma unroll
    for (int n = 0; n < G::NT; ++n)
#pragma unroll
        for (int k4 = 0; k4 < G::KQ; k4 += 4) {
            const f32x4 v = ld4(W + (16 * n + j) * D + G::KQ * q + k4);
#pragma unroll
            for (int i = 0; i < 4; ++i) bw[n][k4 + i] = v[i];
        }
    float bv[G::NT];
#pragma unroll
    for (int n = 0; n < G::NT; ++n) bv[n] = (flags & LG_F_BIAS) ? bias[16 * n + j] : 0.f;

    for (int64_t tile = static_cast<int64_t>(blockIdx.x) * kWaves + wave; tile < ntiles;
         tile += static_cast<int64_t>(gridDim.x) * kWaves) {
        const int64_t r0 = tile * kTileRows;
        f32x4 acc[G::PASSES];
        gather_rows<D, false>(rowptr, col, wgt, x, nullptr, 1.f, r0, R, N, lane, acc);
#pragma unroll
        for (int p = 0; p < G::PASSES; ++p) st4(my + (p * G::RPI + rl) * G::S + 4 * fg, acc[p]);
        wave_lds_sync();

        f32x4 o[G::NT];
#pragma unroll
        for (int n = 0; n < G::NT; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k4 = 0; k4 < G::KQ; k4 += 4) {
            const f32x4 a = ld4(my + j * G::S + G::KQ * q + k4);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int n = 0; n < G::NT; ++n) o[n] = mfma16x16x4(a[i], bw[n][k4 + i], o[n]);
        }
        wave_lds_sync();

        // epilogue: o[n][reg] = out[row 4q+reg][col 16n+j]
#pragma unroll
        for (int n = 0; n < G::NT; ++n)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int row = 4 * q + reg, c = 16 * n + j;
                float v = o[n][reg] + bv[n];
                if (flags & LG_F_RELU) v = fmaxf(v, 0.f);
                if (flags & LG_F_DROPOUT) v = lg_dropout(v, p_drop, dscale, seed, salt, (r0 + row) * D + c);
                my[row * G::S + c] = v;
            }
        wave_lds_sync();
#pragma unroll
        for (int p = 0; p < G::PASSES; ++p) {
            const int lr = p * G::RPI + rl;
            const int64_t r = r0 + lr;
            if (r < R) st4(y + r * D + 4 * fg, ld4(my + lr * G::S + 4 * fg));
        }
        wave_lds_sync();
    }
}

// ------------------------------------------------------------------ backward
// dz = MASK_IN ? dy*scale_in*[y>0] : dy ; t = Ahat^T dz ; dx = t W ; dW += t^T x ; db += sum dz
template <int D, bool MASK_IN>
__global__ void __launch_bounds__(64 * kWaves)
k_gcn_bwd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
          const float* __restrict__ dy, const float* __restrict__ yv, const float* __restrict__ x,
          const float* __restrict__ W, float* __restrict__ dxo, float* __restrict__ slab, int64_t N, int64_t R,
          int64_t ntiles, int mask_out, float scale_in, float scale_out) {
    using G = Geo<D>;
    constexpr int SW = D + 1;  // W rows padded: conflict-free column reads
    constexpr int WBUF = 2 * G::TILE;
    constexpr int L = D * D + D;
    static_assert(kWaves * WBUF >= L, "reduction buffer must fit in the tile buffers");
    __shared__ __attribute__((aligned(16))) float lds[kWaves * WBUF + D * SW];
    float* wl = lds + kWaves * WBUF;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* tl = lds + wave * WBUF;  // t tile, then dx tile
    float* xl = tl + G::TILE;       // x tile
    const int j = lane & 15, q = lane >> 4;
    const int rl = lane / G::LPR, fg = lane % G::LPR;

    for (int i = threadIdx.x; i < D * D; i += blockDim.x) wl[(i / D) * SW + (i % D)] = W[i];
    __syncthreads();

    f32x4 dw[G::NT][G::NT];  // dW tile (mo, ni): rows o = 16mo + 4q + reg, cols i = 16ni + j
#pragma unroll
    for (int a = 0; a < G::NT; ++a)
#pragma unroll
        for (int b = 0; b < G::NT; ++b) dw[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dbacc = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int64_t tile = static_cast<int64_t>(blockIdx.x) * kWaves + wave; tile < ntiles;
         tile += static_cast<int64_t>(gridDim.x) * kWaves) {
        const int64_t r0 = tile * kTileRows;
        f32x4 acc[G::PASSES];
        gather_rows<D, MASK_IN>(rowptr, col, wgt, dy, yv, scale_in, r0, R, N, lane, acc);
#pragma unroll
        for (int p = 0; p < G::PASSES; ++p) {
            const int lr = p * G::RPI + rl;
            const int64_t r = r0 + lr;
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
            st4(tl + lr * G::S + 4 * fg, acc[p]);
            st4(xl + lr * G::S + 4 * fg, xv);
        }
        wave_lds_sync();

        // dx = t W : A[row][k=o] = t[row][o], B[k=o][c] = W[o][c]
        f32x4 o[G::NT];
#pragma unroll
        for (int n = 0; n < G::NT; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k4 = 0; k4 < G::KQ; k4 += 4) {
            const f32x4 a = ld4(tl + j * G::S + G::KQ * q + k4);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ko = G::KQ * q + k4 + i;
#pragma unroll
                for (int n = 0; n < G::NT; ++n) o[n] = mfma16x16x4(a[i], wl[ko * SW + 16 * n + j], o[n]);
            }
        }
        // dW += t^T x : A[o][k=row] = t[row][o], B[k=row][i] = x[row][i]; row = 4q + ks
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int row = 4 * q + ks;
            float ta[G::NT], xb[G::NT];
#pragma unroll
            for (int m = 0; m < G::NT; ++m) {
                ta[m] = tl[row * G::S + 16 * m + j];
                xb[m] = xl[row * G::S + 16 * m + j];
            }
#pragma unroll
            for (int mo = 0; mo < G::NT; ++mo)
#pragma unroll
                for (int ni = 0; ni < G::NT; ++ni) dw[mo][ni] = mfma16x16x4(ta[mo], xb[ni], dw[mo][ni]);
        }
        wave_lds_sync();

#pragma unroll
        for (int n = 0; n < G::NT; ++n)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int row = 4 * q + reg, c = 16 * n + j;
                float v = o[n][reg];
                if (mask_out) v = xl[row * G::S + c] > 0.f ? v * scale_out : 0.f;
                tl[row * G::S + c] = v;
            }
        wave_lds_sync();
#pragma unroll
        for (int p = 0; p < G::PASSES; ++p) {
            const int lr = p * G::RPI + rl;
            const int64_t r = r0 + lr;
            if (r < R) st4(dxo + r * D + 4 * fg, ld4(tl + lr * G::S + 4 * fg));
        }
        wave_lds_sync();
    }

    // ---- per-block reduction of dW / db (fixed wave order -> deterministic)
    // db: lanes sharing a feature group are lane % LPR; fold rows together.
#pragma unroll
    for (int off = G::LPR; off < 64; off <<= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) dbacc[i] += __shfl_xor(dbacc[i], off);
    __syncthreads();
    float* red = lds;  // reuse tile buffers
    for (int i = threadIdx.x; i < L; i += blockDim.x) red[i] = 0.f;
    for (int wv = 0; wv < kWaves; ++wv) {
        __syncthreads();
        if (wave == wv) {
#pragma unroll
            for (int mo = 0; mo < G::NT; ++mo)
#pragma unroll
                for (int ni = 0; ni < G::NT; ++ni)
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg)
                        red[(16 * mo + 4 * q + reg) * D + 16 * ni + j] += dw[mo][ni][reg];
            if (lane < G::LPR)
#pragma unroll
                for (int i = 0; i < 4; ++i) red[D * D + 4 * lane + i] += dbacc[i];
        }
    }
    __syncthreads();
    float* out = slab + static_cast<int64_t>(blockIdx.x) * L;
    for (int i = threadIdx.x; i < L; i += blockDim.x) out[i] = red[i];
}

// ------------------------------------------------------------------ plain propagate
template <int D>
__global__ void __launch_bounds__(256)
k_spmm(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
       const float* __restrict__ x, float* __restrict__ y, int64_t N, int64_t R, int64_t ntiles) {
    using G = Geo<D>;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int rl = lane / G::LPR, fg = lane % G::LPR;
    for (int64_t tile = static_cast<int64_t>(blockIdx.x) * 4 + wave; tile < ntiles;
         tile += static_cast<int64_t>(gridDim.x) * 4) {
        const int64_t r0 = tile * kTileRows;
        f32x4 acc[G::PASSES];
        gather_rows<D, false>(rowptr, col, wgt, x, nullptr, 1.f, r0, R, N, lane, acc);
#pragma unroll
        for (int p = 0; p < G::PASSES; ++p) {
            const int64_t r = r0 + p * G::RPI + rl;
            if (r < R) st4(y + r * D + 4 * fg, acc[p]);
        }
    }
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

int bwd_grid(int64_t ntiles) {
    const int64_t want = ceil_div(ntiles, kWaves);
    const int64_t cap = 2 * static_cast<int64_t>(lg_num_cus());
    return static_cast<int>(want < cap ? (want > 0 ? want : 1) : cap);
}

int bwd_grid_max() { return 2 * lg_num_cus(); }

}  // namespace

extern "C" int lg_gcn_fwd(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, const float* W,
                          const float* bias, float* y, int64_t B, int64_t N, int64_t D, int flags, float dropout_p,
                          uint64_t seed, uint32_t salt, lg_stream_t stream) {
    if (B < 0 || N <= 0) return LG_EINVAL;
    if (!rowptr || !col || !w || !x || !W || !y || x == y) return LG_EINVAL;
    if ((flags & LG_F_BIAS) && !bias) return LG_EINVAL;
    if ((flags & LG_F_DROPOUT) && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    const int64_t R = B * N;
    if (R == 0) return LG_OK;
    const int64_t ntiles = ceil_div(R, kTileRows);
    const int64_t cap = 8LL * lg_num_cus();
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(ntiles, kWaves), cap));
    const float scale = (flags & LG_F_DROPOUT) ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
    switch (D) {
        case 64:
            k_gcn_fwd<64><<<grid, 64 * kWaves, 0, s>>>(rowptr, col, w, x, W, bias, y, N, R, ntiles, flags, dropout_p,
                                                       scale, seed, salt);
            break;
        case 32:
            k_gcn_fwd<32><<<grid, 64 * kWaves, 0, s>>>(rowptr, col, w, x, W, bias, y, N, R, ntiles, flags, dropout_p,
                                                       scale, seed, salt);
            break;
        default:
            return LG_EUNSUPPORTED;
    }
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_spmm(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, float* y,
                       int64_t B, int64_t N, int64_t D, lg_stream_t stream) {
    if (B < 0 || N <= 0) return LG_EINVAL;
    if (!rowptr || !col || !w || !x || !y || x == y) return LG_EINVAL;
    const int64_t R = B * N;
    if (R == 0) return LG_OK;
    const int64_t ntiles = ceil_div(R, kTileRows);
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(ntiles, 4), 8LL * lg_num_cus()));
    hipStream_t s = lg_stream(stream);
    switch (D) {
        case 64: k_spmm<64><<<grid, 256, 0, s>>>(rowptr, col, w, x, y, N, R, ntiles); break;
        case 32: k_spmm<32><<<grid, 256, 0, s>>>(rowptr, col, w, x, y, N, R, ntiles); break;
        default: return LG_EUNSUPPORTED;
    }
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int64_t lg_gcn_bwd_workspace_bytes(int64_t D) {
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    return static_cast<int64_t>(bwd_grid_max()) * (D * D + D) * static_cast<int64_t>(sizeof(float));
}

extern "C" int lg_gcn_bwd(const int32_t* rowptr_t, const int32_t* col_t, const float* w_t, const float* dy,
                          const float* y, const float* x, const float* W, float* dx_out, float* dW, float* db,
                          int64_t B, int64_t N, int64_t D, int flags, float scale_in, float scale_out,
                          void* workspace, lg_stream_t stream) {
    if (B < 0 || N <= 0) return LG_EINVAL;
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
#define LG_BWD_LAUNCH(DD, MI)                                                                                     \
    k_gcn_bwd<DD, MI><<<grid, 64 * kWaves, 0, s>>>(rowptr_t, col_t, w_t, dy, y, x, W, dx_out, slab, N, R, ntiles, \
                                                   mask_out, scale_in, scale_out)
    if (D == 64) {
        if (mask_in) LG_BWD_LAUNCH(64, true); else LG_BWD_LAUNCH(64, false);
    } else {
        if (mask_in) LG_BWD_LAUNCH(32, true); else LG_BWD_LAUNCH(32, false);
    }
#undef LG_BWD_LAUNCH
    LG_RET_IF_LAUNCH_FAILED();
    const int64_t L = D * D + D;
    int rc = lg_launch_slab_reduce(slab, grid, L, D * D, dW, s);
    if (rc == LG_OK && db) rc = lg_launch_slab_reduce(slab + D * D, grid, L, D, db, s);
    return rc;
}
