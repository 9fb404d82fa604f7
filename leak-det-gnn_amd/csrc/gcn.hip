// K5+K6+K7: fused GCN layer forward / backward and the plain propagate, gfx950.
//
// Layout: node features fp32 [B][N][D] (row r = b*N + n), one single-graph CSR
// (rowptr / col / w, self loop last in each row) shared by all B windows: row r
// gathers rows b*N + col[e].  When the CSR fits (L-TOWN-A: 20 KB) every workgroup
// stages it in LDS once; large graphs (C5, 100k nodes) read it through L2.
//
// Work unit: a 16-row "wave tile" owned by one wavefront, tiles dealt XCD-aware
// (xcd_tiles) to a persistent grid.  Per tile:
//   gather   16 lanes per row (D = 64), lane = one float4 of features; all 16 rows
//            in one round with U neighbours each, so K*U float4 loads per lane are
//            in flight; neighbour rows are read with buffer loads whose offset is
//            pushed out of range for padded slots (the hardware returns 0 and
//            issues no memory request), so the loop has no branches and all CSR
//            reads of a round are issued before any row load;
//   MFMA     the layer is computed transposed, y^T (D x 16) = W (D x D) (Ahat x)^T
//            on v_mfma_f32_16x16x4_f32 (exact fp32); A = W from LDS, B = the
//            gathered tile from LDS; the k-chunks of tile i run between the row
//            loads of tile i+1 and their use (software pipeline, one LDS tile per
//            wave: the next tile is held in registers until the MFMAs are done);
//   epilogue bias (initial accumulator), ReLU as max(t, floor), counter-hash
//            dropout, then rows are written back whole through the LDS tile.
// Backward: dz = MASK_IN ? dy*scale*[y>0] : dy; t = Ahat^T dz (transposed CSR);
// dx = t W (MFMA), dW = t^T x and db = sum dz accumulated per wave, reduced per
// block in a fixed order, then across blocks by the shared slab reducer.
// All offsets are 32-bit byte offsets: the API splits launches over windows so that
// each launch's [rows][D] tensors stay below 4 GiB.
#include <algorithm>
#include "common.h"
#include "reduce.h"

namespace {

constexpr int kTileRows = 16;  // rows per wave tile (MFMA N)
constexpr int kBwdWaves = 8;
constexpr int kSpmmWaves = 4;
constexpr int64_t kCsrLdsMax = 48 * 1024;
constexpr uint32_t kOob = 0xFFFFFFF0u;             // beyond every descriptor: loads read 0, stores drop
constexpr int64_t kMaxLaunchBytes = 0xFFFFFF00LL;  // per-launch tensor size limit (32-bit offsets)

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int D>
struct Geo {
    static constexpr int LPR = D / 4;           // lanes per row in the gather
    static constexpr int RPI = 64 / LPR;        // rows per wave instruction
    static constexpr int K = kTileRows / RPI;   // row groups per tile
    static constexpr int KS = D / 4;            // k-steps of one contraction
    static constexpr int CH = KS / 4;           // k-chunks (4 k-steps, one float4 of B)
    static constexpr int MT = D / 16;           // 16-row output tiles
    static constexpr int S = D + 4;             // padded LDS row stride (floats)
    static constexpr int TILE = kTileRows * S;  // floats per LDS tile
};

// fp32 rows [rows][D] behind a buffer descriptor (built from kernel arguments, so it
// lives in SGPRs).  ok == false turns the access into a no-op (load returns 0).
template <int D>
struct Rows {
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ f32x4 ld(uint32_t row, int fg, bool ok) const {
        const uint32_t off = ok ? row * (4u * D) + 16u * fg : kOob;
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
    __device__ __forceinline__ void st(uint32_t row, int fg, bool ok, f32x4 v) const {
        const uint32_t off = ok ? row * (4u * D) + 16u * fg : kOob;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v), rs,
                                               off, 0, 0);
    }
};
template <int D>
__device__ __forceinline__ Rows<D> rows_of(const float* p, uint32_t rows) {
    return Rows<D>{__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), static_cast<short>(0),
                                                     static_cast<int>(rows * (4u * D)), 0x00020000)};
}

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

// Single-graph CSR.  Global form: rowptr / col / w arrays.  LDS form (PAIRS): rowptr
// [0, N+1), padded to an even word count, then one (col, w) pair per entry, so a
// neighbour slot costs one 64-bit LDS read; `col` then points at the pairs.
struct Csr {
    const int32_t* rp;
    const int32_t* col;
    const float* w;
};
template <bool PAIRS>
__device__ __forceinline__ void csr_at(const Csr& g, int e, int32_t& c, float& w) {
    if constexpr (PAIRS) {
        const int2 v = *reinterpret_cast<const int2*>(g.col + 2 * e);
        c = v.x;
        w = __int_as_float(v.y);
    } else {
        c = g.col[e];
        w = g.w[e];
    }
}

// CSR words in LDS (pair layout), or 0 when it does not fit.
inline int64_t csr_lds_bytes(int64_t N, int64_t nnz_cap) {
    const int64_t b = 4 * (((N + 2) & ~int64_t{1}) + 2 * nnz_cap);
    return b <= kCsrLdsMax ? b : 0;
}

// Stage the CSR into LDS in the pair layout: every thread issues all of its loads
// (clamped indices, no branches) before its first LDS store, so the prologue costs one
// memory round trip per 8*blockDim words instead of one per word-loop iteration.
// Caller syncs.
__device__ __forceinline__ Csr stage_csr(uint32_t* s, const int32_t* __restrict__ rowptr,
                                         const int32_t* __restrict__ col, const float* __restrict__ w, uint32_t N) {
    const uint32_t n1 = N + 1, n1p = (N + 2) & ~1u, nnz = static_cast<uint32_t>(rowptr[N]), total = n1p + 2 * nnz;
    const uint32_t* rp = reinterpret_cast<const uint32_t*>(rowptr);
    const uint32_t* cp = reinterpret_cast<const uint32_t*>(col);
    const uint32_t* wp = reinterpret_cast<const uint32_t*>(w);
    constexpr int PER = 8;
    for (uint32_t base = 0; base < total; base += blockDim.x * PER) {
        uint32_t v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t i = min(base + u * blockDim.x + threadIdx.x, total - 1);
            const uint32_t j = i - n1p, e = j >> 1;
            // one mask-selected address and one load (no branches, so all PER loads are in
            // flight); the pad word between rowptr and the pairs copies rowptr[N] (never read)
            const uint32_t ec = min(e, nnz > 0 ? nnz - 1 : 0u);
            const uint64_t mr = 0 - static_cast<uint64_t>(i < n1p);
            const uint64_t mw = 0 - static_cast<uint64_t>(i >= n1p && (j & 1));
            const uint64_t mc = ~(mr | mw);
            const uint64_t ad = (reinterpret_cast<uint64_t>(rp + min(i, n1 - 1)) & mr) |
                                (reinterpret_cast<uint64_t>(wp + ec) & mw) | (reinterpret_cast<uint64_t>(cp + ec) & mc);
            v[u] = *reinterpret_cast<const uint32_t*>(ad);
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t i = base + u * blockDim.x + threadIdx.x;
            if (i < total) s[i] = v[u];
        }
    }
    return Csr{reinterpret_cast<const int32_t*>(s), reinterpret_cast<const int32_t*>(s + n1p), nullptr};
}


struct NoHook {
    __device__ __forceinline__ void operator()(int, int) const {}
};

// Whole-tile gather: acc[k] = row (r0 + RPI*k + rl), features 4fg..4fg+3, summed over
// the row's CSR entries in order (fp32 fma; w * v[s] per entry).  MASK: gathered values
// are v * mscale * [m > 0] (ReLU / dropout backward of the gathered tensor).  The trip
// count is the tile's wave-uniform max degree so hook(round, rounds) — independent
// work such as the previous tile's MFMAs — runs with every lane active, between the
// issue of a round's loads and their use.
template <int D, bool MASK, int U, bool PAIRS, typename Hook = NoHook>
__device__ __forceinline__ void gather16(const Csr& g, const Rows<D>& src, const Rows<D>& msk, float mscale,
                                         uint32_t r0, uint32_t R, const lg_fastdiv& fdN, int lane,
                                         f32x4 (&acc)[Geo<D>::K], Hook&& hook = Hook{}) {
    using G = Geo<D>;
    const int rl = lane / G::LPR, fg = lane % G::LPR;
    int e0[G::K], e1[G::K];
    uint32_t base[G::K];
    int maxd = 0;
    // node of the tile's first row by one (wave-uniform) division; the other rows add
    // their offset (< 16) and wrap once (N >= 16; tiny graphs divide per row)
    const uint32_t n0 = r0 - lg_div(r0, fdN) * fdN.d;
#pragma unroll
    for (int k = 0; k < G::K; ++k) {
        acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        const uint32_t r = r0 + G::RPI * k + rl;
        const bool valid = r < R;
        const uint32_t rr = valid ? r : 0u;
        uint32_t n;
        if (fdN.d >= 16) {
            const uint32_t t = n0 + G::RPI * k + rl;
            n = valid ? (t >= fdN.d ? t - fdN.d : t) : 0u;
        } else {
            n = rr - lg_div(rr, fdN) * fdN.d;
        }
        e0[k] = g.rp[n];
        e1[k] = valid ? g.rp[n + 1] : e0[k];
        base[k] = rr - n;
        maxd = max(maxd, e1[k] - e0[k]);
    }
    // rounds = wave max of ceil(maxd / U): a few ballots (SALU) instead of a shuffle tree
    int rounds = 0;
    while (__builtin_amdgcn_ballot_w64(maxd > rounds * U) != 0) ++rounds;
    // CSR entries of round rd + 1 are read (LDS) while round rd's rows are in flight, so
    // the LDS latency is off the round's critical path (read -> address -> load issue).
    int32_t s[G::K][U];
    float ww[G::K][U];
    bool ok[G::K][U];
    auto read_entries = [&](int rd) {
#pragma unroll
        for (int k = 0; k < G::K; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = e0[k] + rd * U + u;
                ok[k][u] = e < e1[k];
                const int ei = ok[k][u] ? e : 0;  // maxd > 0 implies nnz > 0, so entry 0 exists
                csr_at<PAIRS>(g, ei, s[k][u], ww[k][u]);
            }
    };
    if (rounds > 0) read_entries(0);
    for (int rd = 0; rd < rounds; ++rd) {
        f32x4 v[G::K][U], m[G::K][U];
#pragma unroll
        for (int k = 0; k < G::K; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                v[k][u] = src.ld(base[k] + static_cast<uint32_t>(s[k][u]), fg, ok[k][u]);
                if constexpr (MASK) m[k][u] = msk.ld(base[k] + static_cast<uint32_t>(s[k][u]), fg, ok[k][u]);
            }
        float wv[G::K][U];
#pragma unroll
        for (int k = 0; k < G::K; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u) wv[k][u] = ok[k][u] ? ww[k][u] : 0.f;
        if (rd + 1 < rounds) read_entries(rd + 1);
        hook(rd, rounds);
#pragma unroll
        for (int k = 0; k < G::K; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                f32x4 t = v[k][u];
                if constexpr (MASK) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) t[i] = m[k][u][i] > 0.f ? t[i] * mscale : 0.f;
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[k][i] = fmaf(wv[k][u], t[i], acc[k][i]);
            }
    }
}

template <int D>
__device__ __forceinline__ void put_tile(float* __restrict__ tl, const f32x4 (&acc)[Geo<D>::K], int lane) {
    using G = Geo<D>;
    const int rl = lane / G::LPR, fg = lane % G::LPR;
#pragma unroll
    for (int k = 0; k < G::K; ++k) st4(tl + (G::RPI * k + rl) * G::S + 4 * fg, acc[k]);
}

// Write the 16-row LDS tile tl[row][feature] to rows r0.. as whole rows.
template <int D>
__device__ __forceinline__ void store_tile(const float* __restrict__ tl, const Rows<D>& dst, uint32_t r0, uint32_t R,
                                           int lane) {
    using G = Geo<D>;
    const int rl = lane / G::LPR, fg = lane % G::LPR;
    f32x4 v[G::K];
#pragma unroll
    for (int k = 0; k < G::K; ++k) v[k] = ld4(tl + (G::RPI * k + rl) * G::S + 4 * fg);
#pragma unroll
    for (int k = 0; k < G::K; ++k) {
        const uint32_t r = r0 + G::RPI * k + rl;
        dst.st(r, fg, r < R, v[k]);
    }
}

// ------------------------------------------------------------------ forward
template <int D, int NW, bool CSR_LDS, bool DROP>
__global__ void __launch_bounds__(64 * NW)
k_gcn_fwd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
          const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
          float* __restrict__ y, uint32_t N, lg_fastdiv fdN, uint32_t R, int64_t ntiles, float relu_floor,
          float p_drop, float dscale, uint64_t seed, uint32_t salt, uint64_t row_offset, int csr_words) {
    using G = Geo<D>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* wl = reinterpret_cast<float*>(smem) + (CSR_LDS ? ((csr_words + 3) & ~3) : 0);  // W [out][in], stride S
    float* bl = wl + D * G::S;                                                          // bias [D]
    float* tiles = bl + D;
    const Rows<D> xs = rows_of<D>(x, R), ys = rows_of<D>(y, R);

    // prologue: W and bias loads first, then the CSR staging, then the LDS stores
    constexpr int W4 = D * D / 4, WPER = (W4 + 64 * NW - 1) / (64 * NW);
    f32x4 wv[WPER];
#pragma unroll
    for (int u = 0; u < WPER; ++u) wv[u] = ld4(W + 4 * min<int>(u * 64 * NW + threadIdx.x, W4 - 1));
    const float bb = (bias && threadIdx.x < D) ? bias[threadIdx.x] : 0.f;
    const Csr g = CSR_LDS ? stage_csr(reinterpret_cast<uint32_t*>(smem), rowptr, col, wgt, N)
                          : Csr{rowptr, col, wgt};
    // dropout's 1 / (1 - p) is folded into W and b: relu(s z) = s relu(z) for s > 0
    const float fold = DROP ? dscale : 1.0f;
#pragma unroll
    for (int u = 0; u < WPER; ++u) {
        const int i = u * 64 * NW + threadIdx.x;
        if (i < W4) st4(wl + (i / (D / 4)) * G::S + 4 * (i % (D / 4)), wv[u] * fold);
    }
    if (threadIdx.x < D) bl[threadIdx.x] = bb * fold;
    __syncthreads();

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    float* tl = tiles + wave * G::TILE;
    const uint32_t key = lg_dropout_key_dev(seed, salt);

    const TileRange tr = xcd_tiles(ntiles, wave, NW);
    f32x4 acc[G::K];
    if (tr.first < tr.end) {
        gather16<D, false, 2, CSR_LDS>(g, xs, xs, 1.f, static_cast<uint32_t>(tr.first * kTileRows), R, fdN, lane, acc);
        put_tile<D>(tl, acc, lane);
    }
    for (int64_t tile = tr.first; tile < tr.end; tile += tr.stride) {
        wave_lds_sync();
        f32x4 o[G::MT];
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) o[mt] = ld4(bl + 16 * mt + 4 * q);
        int chunk = 0;
        auto mfma_chunk = [&]() {
            const f32x4 bt = ld4(tl + j * G::S + 16 * chunk + 4 * q);  // (Ahat x)[row j][16c + 4q + i]
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt) {
                const f32x4 wa = ld4(wl + (16 * mt + j) * G::S + 16 * chunk + 4 * q);  // W[16mt + j][..]
#pragma unroll
                for (int i = 0; i < 4; ++i) o[mt] = mfma(wa[i], bt[i], o[mt]);
            }
            ++chunk;
        };
        // spread the k-chunks over the next tile's gather rounds
        auto hook = [&](int rd, int rounds) {
            const int target = (G::CH * (rd + 1) + rounds - 1) / rounds;
            while (chunk < target) mfma_chunk();
        };
        const int64_t next = tile + tr.stride;
        const bool more = next < tr.end;
        if (more)
            gather16<D, false, 2, CSR_LDS>(g, xs, xs, 1.f, static_cast<uint32_t>(next * kTileRows), R, fdN, lane, acc,
                                           hook);
        while (chunk < G::CH) mfma_chunk();

        const uint32_t r0 = static_cast<uint32_t>(tile * kTileRows);
        // row-stream dropout (common.h): seeded by the global row (launch splits do not
        // change it) and the lane group q; each xorshift step decides two channels
        // (16-bit halves against rint(p 2^16)), in (mt, reg) order
        uint32_t st = 0, thr = 0;
        if constexpr (DROP) {
            st = lg_row_stream_seed(key, row_offset + r0 + j, static_cast<uint32_t>(q));
            thr = lg_keep_threshold16(p_drop);
        }
        const uint32_t r = r0 + j;
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) {
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                float t = fmaxf(o[mt][reg], relu_floor);
                if constexpr (DROP) {
                    if ((reg & 1) == 0) st = lg_xorshift32(st);
                    const uint32_t u16 = (reg & 1) ? (st >> 16) : (st & 0xFFFFu);
                    t = u16 >= thr ? t : 0.0f;
                }
                o[mt][reg] = t;
            }
            // D fragment: row r0 + j, channels 16 mt + 4q .. +3 -> one float4 per block
            ys.st(r, 4 * mt + q, r < R, o[mt]);
        }
        if (more) {
            wave_lds_sync();
            put_tile<D>(tl, acc, lane);
        }
    }
}

// ------------------------------------------------------------------ backward
// dz = MASK_IN ? dy*scale_in*[y>0] : dy ; t = Ahat^T dz ; dx = t W ; dW += t^T x ; db += sum dz
// NB: also sum dx_out over the rows whose node has node_slot < 0 (the node-init bias
// gradient, detector.py:184-190: rows without a sensor are relu(bias) + dropout).
template <int D, bool MASK_IN, bool CSR_LDS, bool NB>
__global__ void __launch_bounds__(64 * kBwdWaves, 2)
k_gcn_bwd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
          const float* __restrict__ dy, const float* __restrict__ yv, const float* __restrict__ x,
          const float* __restrict__ W, const int32_t* __restrict__ node_slot, float* __restrict__ dxo,
          float* __restrict__ slab, uint32_t N, lg_fastdiv fdN, uint32_t R, int64_t ntiles, int mask_out,
          float scale_in, float scale_out, int csr_words, int accumulate) {
    using G = Geo<D>;
    constexpr int SW = D + 4;  // W rows in LDS, conflict-free column reads
    constexpr int WBUF = 2 * G::TILE;
    constexpr int L = D * D + 2 * D;  // slab row: dW, db, d(node bias)
    static_assert(kBwdWaves * WBUF >= L, "reduction buffer must fit in the tile buffers");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Rows<D> dys = rows_of<D>(dy, R), ms = rows_of<D>(MASK_IN ? yv : dy, R), xs = rows_of<D>(x, R),
                  dxs = rows_of<D>(dxo, R);
    float* lds = reinterpret_cast<float*>(smem) + (CSR_LDS ? ((csr_words + 3) & ~3) : 0);
    float* wl = lds + kBwdWaves * WBUF;
    constexpr int W4 = D * D / 4, WPER = (W4 + 64 * kBwdWaves - 1) / (64 * kBwdWaves);
    f32x4 wv[WPER];
#pragma unroll
    for (int u = 0; u < WPER; ++u) wv[u] = ld4(W + 4 * min<int>(u * 64 * kBwdWaves + threadIdx.x, W4 - 1));
    const Csr g = CSR_LDS ? stage_csr(reinterpret_cast<uint32_t*>(smem), rowptr, col, wgt, N)
                          : Csr{rowptr, col, wgt};
#pragma unroll
    for (int u = 0; u < WPER; ++u) {
        const int i = u * 64 * kBwdWaves + threadIdx.x;
        if (i < W4) st4(wl + (i / (D / 4)) * SW + 4 * (i % (D / 4)), wv[u]);
    }
    __syncthreads();

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const int rl = lane / G::LPR, fg = lane % G::LPR;
    float* tl = lds + wave * WBUF;  // t tile [row][feature], later dx
    float* xl = tl + G::TILE;       // x tile [row][feature]

    f32x4 dw[G::MT][G::MT];  // dW tile (mo, ni): rows o = 16mo + 4q + reg, cols i = 16ni + j
#pragma unroll
    for (int a = 0; a < G::MT; ++a)
#pragma unroll
        for (int b = 0; b < G::MT; ++b) dw[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dbacc = f32x4{0.f, 0.f, 0.f, 0.f};  // features 4fg..4fg+3, summed over this lane's rows
    f32x4 nbacc[NB ? G::MT : 1];              // NB: features 16mt + 4q + reg over this lane's rows j
#pragma unroll
    for (int mt = 0; mt < (NB ? G::MT : 1); ++mt) nbacc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

    const TileRange tr = xcd_tiles(ntiles, wave, kBwdWaves);
    for (int64_t tile = tr.first; tile < tr.end; tile += tr.stride) {
        const uint32_t r0 = static_cast<uint32_t>(tile * kTileRows);
        // own rows (coalesced): dz for db, x for dW and the output mask — issued first
        f32x4 dz[G::K], mz[G::K], xv[G::K];
#pragma unroll
        for (int k = 0; k < G::K; ++k) {
            const uint32_t r = r0 + G::RPI * k + rl;
            dz[k] = dys.ld(r, fg, r < R);
            if constexpr (MASK_IN) mz[k] = ms.ld(r, fg, r < R);
            xv[k] = xs.ld(r, fg, r < R);
        }
        f32x4 acc[G::K];
        gather16<D, MASK_IN, 1, CSR_LDS>(g, dys, ms, scale_in, r0, R, fdN, lane, acc);
        put_tile<D>(tl, acc, lane);
#pragma unroll
        for (int k = 0; k < G::K; ++k) {
            if constexpr (MASK_IN) {
#pragma unroll
                for (int i = 0; i < 4; ++i) dz[k][i] = mz[k][i] > 0.f ? dz[k][i] * scale_in : 0.f;
            }
            dbacc += dz[k];
            st4(xl + (G::RPI * k + rl) * G::S + 4 * fg, xv[k]);
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
        for (int a = 0; a < G::CH; ++a) {
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
        if constexpr (NB) {
            const uint32_t r = r0 + j;
            const uint32_t rr = r < R ? r : 0u;
            const bool bias_row = r < R && node_slot[rr - lg_div(rr, fdN) * fdN.d] < 0;
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt)
                if (bias_row) nbacc[mt] += o[mt];
        }
        wave_lds_sync();
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) st4(tl + j * G::S + 16 * mt + 4 * q, o[mt]);
        wave_lds_sync();
        store_tile<D>(tl, dxs, r0, R, lane);
        wave_lds_sync();
    }
    if constexpr (NB) {  // fold the 16 row lanes j of each (q, reg)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1)
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt)
#pragma unroll
                for (int i = 0; i < 4; ++i) nbacc[mt][i] += __shfl_xor(nbacc[mt][i], off);
    }

    // ---- per-block reduction of dW / db (fixed wave order -> deterministic)
#pragma unroll
    for (int off = G::LPR; off < 64; off <<= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) dbacc[i] += __shfl_xor(dbacc[i], off);
    __syncthreads();
    float* red = lds;  // reuse the tile buffers
    for (int i = threadIdx.x; i < L; i += blockDim.x) red[i] = 0.f;
    for (int wv2 = 0; wv2 < kBwdWaves; ++wv2) {
        __syncthreads();
        if (wave == wv2) {
#pragma unroll
            for (int mo = 0; mo < G::MT; ++mo)
#pragma unroll
                for (int ni = 0; ni < G::MT; ++ni)
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg)
                        red[(16 * mo + 4 * q + reg) * D + 16 * ni + j] += dw[mo][ni][reg];
            if (lane < G::LPR)
#pragma unroll
                for (int i = 0; i < 4; ++i) red[D * D + 4 * lane + i] += dbacc[i];
            if (NB && j == 0)
#pragma unroll
                for (int mt = 0; mt < G::MT; ++mt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) red[D * D + D + 16 * mt + 4 * q + i] += nbacc[mt][i];
        }
    }
    __syncthreads();
    float* out = slab + static_cast<int64_t>(blockIdx.x) * L;
    if (accumulate)
        for (int i = threadIdx.x; i < L; i += blockDim.x) out[i] += red[i];
    else
        for (int i = threadIdx.x; i < L; i += blockDim.x) out[i] = red[i];
}

// ------------------------------------------------------------------ plain propagate
template <int D, bool CSR_LDS>
__global__ void __launch_bounds__(64 * kSpmmWaves)
k_spmm(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ wgt,
       const float* __restrict__ x, float* __restrict__ y, uint32_t N, lg_fastdiv fdN, uint32_t R, int64_t ntiles) {
    using G = Geo<D>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Csr g = CSR_LDS ? stage_csr(reinterpret_cast<uint32_t*>(smem), rowptr, col, wgt, N)
                          : Csr{rowptr, col, wgt};
    __syncthreads();
    const Rows<D> xs = rows_of<D>(x, R), ys = rows_of<D>(y, R);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, rl = lane / G::LPR, fg = lane % G::LPR;
    const TileRange tr = xcd_tiles(ntiles, wave, kSpmmWaves);
    for (int64_t tile = tr.first; tile < tr.end; tile += tr.stride) {
        const uint32_t r0 = static_cast<uint32_t>(tile * kTileRows);
        f32x4 acc[G::K];
        gather16<D, false, 2, CSR_LDS>(g, xs, xs, 1.f, r0, R, fdN, lane, acc);
#pragma unroll
        for (int k = 0; k < G::K; ++k) {
            const uint32_t r = r0 + G::RPI * k + rl;
            ys.st(r, fg, r < R, acc[k]);
        }
    }
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Windows per launch so that one launch's [rows][D] fp32 tensor stays below 4 GiB.
inline int64_t windows_per_launch(int64_t N, int64_t D) { return kMaxLaunchBytes / (4 * D * N); }

// Persistent grid: as many blocks as are co-resident (registers and LDS both count),
// capped at `cap_per_cu` per CU and at the work available.
template <typename Kern>
int resident_grid(Kern kernel, int threads, int64_t dyn_lds, int64_t want, int cap_per_cu) {
    int per_cu = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, static_cast<size_t>(dyn_lds)) !=
            hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    const int64_t cap = std::min(cap_per_cu, per_cu) * static_cast<int64_t>(lg_num_cus());
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(want, cap)));
}

template <typename Kern>
bool allow_lds(Kern kernel, int64_t dyn) {
    return dyn <= 64 * 1024 || hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   static_cast<int>(dyn)) == hipSuccess;
}

constexpr int kFwdWaves = 16;

template <int D, bool CL, bool DROP>
int launch_fwd(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, const float* W,
               const float* bias, float* y, int64_t Bc, int64_t N, int64_t csr_bytes, float relu_floor, float p,
               float scale, uint64_t seed, uint32_t salt, uint64_t row_offset, hipStream_t s) {
    using G = Geo<D>;
    const int64_t R = Bc * N, ntiles = ceil_div(R, kTileRows);
    const int64_t csr_words = CL ? csr_bytes / 4 : 0;
    const int64_t dyn = 4 * (((csr_words + 3) & ~3LL) + D * G::S + D + kFwdWaves * G::TILE);
    auto kern = k_gcn_fwd<D, kFwdWaves, CL, DROP>;
    if (!allow_lds(kern, dyn)) return LG_EHIP;
    const int grid = resident_grid(kern, 64 * kFwdWaves, dyn, ceil_div(ntiles, kFwdWaves), 2);
    lg_launch(kern, grid, 64 * kFwdWaves, dyn, s, rowptr, col, w, x, W, bias, y, static_cast<uint32_t>(N),
                                            lg_make_fastdiv(static_cast<uint32_t>(N)), static_cast<uint32_t>(R),
                                            ntiles, relu_floor, p, scale, seed, salt, row_offset,
                                            static_cast<int>(csr_words));
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

template <int D>
int fwd_dispatch(bool cl, bool drop, const int32_t* rowptr, const int32_t* col, const float* w, const float* x,
                 const float* W, const float* bias, float* y, int64_t Bc, int64_t N, int64_t csr_bytes,
                 float relu_floor, float p, float scale, uint64_t seed, uint32_t salt, uint64_t row_offset,
                 hipStream_t s) {
#define LG_FWD_ARGS rowptr, col, w, x, W, bias, y, Bc, N, csr_bytes, relu_floor, p, scale, seed, salt, row_offset, s
    if (cl) return drop ? launch_fwd<D, true, true>(LG_FWD_ARGS) : launch_fwd<D, true, false>(LG_FWD_ARGS);
    return drop ? launch_fwd<D, false, true>(LG_FWD_ARGS) : launch_fwd<D, false, false>(LG_FWD_ARGS);
#undef LG_FWD_ARGS
}

template <int D, bool MI, bool CL, bool NB>
int launch_bwd(const int32_t* rowptr_t, const int32_t* col_t, const float* w_t, const float* dy, const float* y,
               const float* x, const float* W, const int32_t* node_slot, float* dx, float* slab, int64_t Bc,
               int64_t N, int64_t csr_bytes, int mask_out, float scale_in, float scale_out, int accumulate,
               int* grid_io, hipStream_t s) {
    using G = Geo<D>;
    const int64_t R = Bc * N, ntiles = ceil_div(R, kTileRows);
    const int64_t csr_words = CL ? csr_bytes / 4 : 0;
    const int64_t dyn = 4 * (((csr_words + 3) & ~3LL) + kBwdWaves * 2 * G::TILE + D * (D + 4));
    auto kern = k_gcn_bwd<D, MI, CL, NB>;
    if (!allow_lds(kern, dyn)) return LG_EHIP;
    // every chunk of a split launch uses the first chunk's grid (the slab rows it accumulates into)
    if (*grid_io == 0) *grid_io = resident_grid(kern, 64 * kBwdWaves, dyn, ceil_div(ntiles, kBwdWaves), 2);
    lg_launch(kern, *grid_io, 64 * kBwdWaves, dyn, s, rowptr_t, col_t, w_t, dy, y, x, W, node_slot, dx, slab,
                                                static_cast<uint32_t>(N),
                                                lg_make_fastdiv(static_cast<uint32_t>(N)), static_cast<uint32_t>(R),
                                                ntiles, mask_out, scale_in, scale_out, static_cast<int>(csr_words),
                                                accumulate);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

template <int D, bool NB>
int bwd_dispatch_nb(bool mi, bool cl, const int32_t* rowptr_t, const int32_t* col_t, const float* w_t,
                    const float* dy, const float* y, const float* x, const float* W, const int32_t* node_slot,
                    float* dx, float* slab, int64_t Bc, int64_t N, int64_t csr_bytes, int mask_out, float scale_in,
                    float scale_out, int accumulate, int* grid_io, hipStream_t s) {
#define LG_BWD_ARGS                                                                                                 \
    rowptr_t, col_t, w_t, dy, y, x, W, node_slot, dx, slab, Bc, N, csr_bytes, mask_out, scale_in, scale_out, accumulate, \
        grid_io, s
    if (mi) return cl ? launch_bwd<D, true, true, NB>(LG_BWD_ARGS) : launch_bwd<D, true, false, NB>(LG_BWD_ARGS);
    return cl ? launch_bwd<D, false, true, NB>(LG_BWD_ARGS) : launch_bwd<D, false, false, NB>(LG_BWD_ARGS);
#undef LG_BWD_ARGS
}

template <int D>
int bwd_dispatch(bool mi, bool cl, const int32_t* rowptr_t, const int32_t* col_t, const float* w_t, const float* dy,
                 const float* y, const float* x, const float* W, const int32_t* node_slot, float* dx, float* slab,
                 int64_t Bc, int64_t N, int64_t csr_bytes, int mask_out, float scale_in, float scale_out,
                 int accumulate, int* grid_io, hipStream_t s) {
    if (node_slot)
        return bwd_dispatch_nb<D, true>(mi, cl, rowptr_t, col_t, w_t, dy, y, x, W, node_slot, dx, slab, Bc, N,
                                        csr_bytes, mask_out, scale_in, scale_out, accumulate, grid_io, s);
    return bwd_dispatch_nb<D, false>(mi, cl, rowptr_t, col_t, w_t, dy, y, x, W, node_slot, dx, slab, Bc, N, csr_bytes,
                                     mask_out, scale_in, scale_out, accumulate, grid_io, s);
}

template <int D, bool CL>
int launch_spmm(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, float* y, int64_t Bc,
                int64_t N, int64_t csr_bytes, hipStream_t s) {
    const int64_t R = Bc * N, ntiles = ceil_div(R, kTileRows);
    const int64_t dyn = CL ? csr_bytes : 0;
    auto kern = k_spmm<D, CL>;
    const int grid = resident_grid(kern, 64 * kSpmmWaves, dyn, ceil_div(ntiles, kSpmmWaves), 8);
    lg_launch(kern, grid, 64 * kSpmmWaves, dyn, s, rowptr, col, w, x, y, static_cast<uint32_t>(N),
                                             lg_make_fastdiv(static_cast<uint32_t>(N)), static_cast<uint32_t>(R),
                                             ntiles);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

int bwd_grid_max() { return 2 * lg_num_cus(); }

}  // namespace

extern "C" int lg_gcn_fwd(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, const float* W,
                          const float* bias, float* y, int64_t B, int64_t N, int64_t D, int64_t nnz_cap, int flags,
                          float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream) {
    if (B < 0 || N <= 0 || nnz_cap < 0) return LG_EINVAL;
    if (!rowptr || !col || !w || !x || !W || !y || x == y) return LG_EINVAL;
    if ((flags & LG_F_BIAS) && !bias) return LG_EINVAL;
    const bool drop = (flags & LG_F_DROPOUT) != 0;
    if (drop && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    if (B == 0) return LG_OK;
    const int64_t wpl = windows_per_launch(N, D);
    if (wpl < 1) return LG_EUNSUPPORTED;
    const int64_t csr = csr_lds_bytes(N, nnz_cap);
    const float relu_floor = (flags & LG_F_RELU) ? 0.f : -__builtin_huge_valf();
    const float scale = drop ? 1.0f / (1.0f - dropout_p) : 1.0f;
    const float* bp = (flags & LG_F_BIAS) ? bias : nullptr;
    hipStream_t s = lg_stream(stream);
    for (int64_t b0 = 0; b0 < B; b0 += wpl) {
        const int64_t Bc = std::min(wpl, B - b0), off = b0 * N * D;
        const uint64_t row_off = static_cast<uint64_t>(b0 * N);
        const int rc = D == 64 ? fwd_dispatch<64>(csr != 0, drop, rowptr, col, w, x + off, W, bp, y + off, Bc, N, csr,
                                                  relu_floor, dropout_p, scale, seed, salt, row_off, s)
                               : fwd_dispatch<32>(csr != 0, drop, rowptr, col, w, x + off, W, bp, y + off, Bc, N, csr,
                                                  relu_floor, dropout_p, scale, seed, salt, row_off, s);
        if (rc != LG_OK) return rc;
    }
    return LG_OK;
}

extern "C" int lg_spmm(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, float* y,
                       int64_t B, int64_t N, int64_t D, int64_t nnz_cap, lg_stream_t stream) {
    if (B < 0 || N <= 0 || nnz_cap < 0) return LG_EINVAL;
    if (!rowptr || !col || !w || !x || !y || x == y) return LG_EINVAL;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    if (B == 0) return LG_OK;
    const int64_t wpl = windows_per_launch(N, D);
    if (wpl < 1) return LG_EUNSUPPORTED;
    const int64_t csr = csr_lds_bytes(N, nnz_cap);
    hipStream_t s = lg_stream(stream);
    for (int64_t b0 = 0; b0 < B; b0 += wpl) {
        const int64_t Bc = std::min(wpl, B - b0), off = b0 * N * D;
        int rc;
        if (D == 64)
            rc = csr ? launch_spmm<64, true>(rowptr, col, w, x + off, y + off, Bc, N, csr, s)
                     : launch_spmm<64, false>(rowptr, col, w, x + off, y + off, Bc, N, csr, s);
        else
            rc = csr ? launch_spmm<32, true>(rowptr, col, w, x + off, y + off, Bc, N, csr, s)
                     : launch_spmm<32, false>(rowptr, col, w, x + off, y + off, Bc, N, csr, s);
        if (rc != LG_OK) return rc;
    }
    return LG_OK;
}

// ------------------------------------------------------------------ propagate, any width
// y[n][c] = sum over row n's CSR entries (entry order) of w[e] x[col[e]][c] (+ bias[c]) for any
// column count C: GCNConv's general path (in_channels != out_channels, or widths other than the
// fused kernels' 32 / 64; models/gcn.py).  A thread owns four consecutive columns of one row
// (VEC, when C and both row strides are multiples of 4 and the bases 16-byte aligned) or one
// column; consecutive threads take consecutive columns, so a row's reads and writes coalesce.
template <bool VEC, typename IX>  // IX: uint32_t when N * C < 2^32 (no 64-bit division per item)
__global__ void __launch_bounds__(256) k_spmm_cols(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                   const float* __restrict__ w, const float* __restrict__ x,
                                                   int64_t ldx, const float* __restrict__ bias, float* __restrict__ y,
                                                   int64_t ldy, int64_t N, int64_t C) {
    constexpr int V = VEC ? 4 : 1;
    const IX CV = static_cast<IX>(C / V), total = static_cast<IX>(N) * CV;
    for (IX i = static_cast<IX>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += static_cast<IX>(gridDim.x) * blockDim.x) {
        const IX nq = i / CV;
        const int64_t n = nq, c = static_cast<int64_t>(i - nq * CV) * V;
        const int e0 = rowptr[n], e1 = rowptr[n + 1];
        if constexpr (VEC) {
            f32x4 acc = bias ? ld4(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
            f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
            for (int e = e0; e < e1; ++e) {
                const f32x4 v = ld4(x + static_cast<int64_t>(col[e]) * ldx + c);
                const float we = w[e];
#pragma unroll
                for (int k = 0; k < 4; ++k) s[k] = fmaf(we, v[k], s[k]);
            }
            st4(y + n * ldy + c, s + acc);
        } else {
            float s = 0.f;
            for (int e = e0; e < e1; ++e) s = fmaf(w[e], x[static_cast<int64_t>(col[e]) * ldx + c], s);
            y[n * ldy + c] = s + (bias ? bias[c] : 0.f);
        }
    }
}

extern "C" int lg_spmm_cols(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, int64_t ldx,
                            const float* bias, float* y, int64_t ldy, int64_t N, int64_t C, lg_stream_t stream) {
    if (N < 0 || C < 0 || ldx < C || ldy < C) return LG_EINVAL;
    if (N == 0 || C == 0) return LG_OK;
    if (!rowptr || !col || !w || !x || !y || x == y) return LG_EINVAL;
    hipStream_t s = lg_stream(stream);
    const bool vec = C % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(y) % 16 == 0 && (!bias || reinterpret_cast<uintptr_t>(bias) % 16 == 0);
    const int64_t items = N * (vec ? C / 4 : C);
    const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((items + 255) / 256, 64LL * lg_num_cus())));
    const bool i32 = items + 256LL * grid < (int64_t{1} << 32);
    if (vec) {
        if (i32) lg_launch(k_spmm_cols<true, uint32_t>, grid, 256, 0, s, rowptr, col, w, x, ldx, bias, y, ldy, N, C);
        else lg_launch(k_spmm_cols<true, int64_t>, grid, 256, 0, s, rowptr, col, w, x, ldx, bias, y, ldy, N, C);
    } else {
        if (i32) lg_launch(k_spmm_cols<false, uint32_t>, grid, 256, 0, s, rowptr, col, w, x, ldx, bias, y, ldy, N, C);
        else lg_launch(k_spmm_cols<false, int64_t>, grid, 256, 0, s, rowptr, col, w, x, ldx, bias, y, ldy, N, C);
    }
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int64_t lg_gcn_bwd_workspace_bytes(int64_t D) {
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    return static_cast<int64_t>(bwd_grid_max()) * (D * D + 2 * D) * static_cast<int64_t>(sizeof(float));
}

extern "C" int lg_gcn_bwd(const int32_t* rowptr_t, const int32_t* col_t, const float* w_t, const float* dy,
                          const float* y, const float* x, const float* W, float* dx_out, float* dW, float* db,
                          const int32_t* node_slot, float* dnode_bias, int64_t B, int64_t N, int64_t D,
                          int64_t nnz_cap, int flags, float scale_in, float scale_out, void* workspace, int64_t ws_bytes,
                          lg_stream_t stream) {
    if (B < 0 || N <= 0 || nnz_cap < 0) return LG_EINVAL;
    if (!rowptr_t || !col_t || !w_t || !dy || !x || !W || !dx_out || !dW || !workspace) return LG_EINVAL;
    if ((node_slot == nullptr) != (dnode_bias == nullptr)) return LG_EINVAL;
    const bool mask_in = (flags & LG_F_MASK_IN) != 0;
    if (mask_in && !y) return LG_EINVAL;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    const int64_t wpl = windows_per_launch(N, D);
    if (wpl < 1) return LG_EUNSUPPORTED;
    // the launch grid is at most bwd_grid_max() workgroups, one slab row each
    if (ws_bytes < lg_gcn_bwd_workspace_bytes(D)) return LG_EINVAL;
    hipStream_t s = lg_stream(stream);
    float* slab = static_cast<float*>(workspace);
    const int mask_out = (flags & LG_F_MASK_OUT) ? 1 : 0;
    const int64_t csr = csr_lds_bytes(N, nnz_cap);
    int grid = 0;
    // B == 0 still runs one (empty) launch so the slab holds zeros
    for (int64_t b0 = 0; b0 < std::max<int64_t>(B, 1); b0 += wpl) {
        const int64_t Bc = std::min(wpl, B - b0), off = b0 * N * D;
        const float* yc = y ? y + off : nullptr;
        const int accumulate = b0 > 0 ? 1 : 0;
        const int rc = D == 64 ? bwd_dispatch<64>(mask_in, csr != 0, rowptr_t, col_t, w_t, dy + off, yc, x + off, W,
                                                  node_slot, dx_out + off, slab, Bc, N, csr, mask_out, scale_in,
                                                  scale_out, accumulate, &grid, s)
                               : bwd_dispatch<32>(mask_in, csr != 0, rowptr_t, col_t, w_t, dy + off, yc, x + off, W,
                                                  node_slot, dx_out + off, slab, Bc, N, csr, mask_out, scale_in,
                                                  scale_out, accumulate, &grid, s);
        if (rc != LG_OK) return rc;
    }
    const int64_t L = D * D + 2 * D;
    const LgSlabSeg segs[3] = {{0, D * D, dW}, {D * D, D, db}, {D * D + D, D, dnode_bias}};
    return lg_launch_slab_reduce_multi(slab, grid, L, segs, 3, nullptr, nullptr, s);
}
