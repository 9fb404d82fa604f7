// Frozen-predictor residual builder: one dilated causal conv layer of
// NormalPredictorTCN (reference models/predictor.py:17-52) over the shared-window row
// plan of models/tcn_plan.py, fused with its bias, LayerNorm, ReLU and (conv2) the
// block's residual add.  SURVEY §8 f rank 1.
//
// Rows: a layer's output for one segment is rows_out rows of C = 128 channels
// ([nseg][rows_out][C], row-major); output row r reads three input rows
// (taps t, t-d, t-2d, or zero) and, for conv2, one block-input row (residual), all
// given as segment-local row numbers by the plan table plan[r] = (tap0, tap1, tap2,
// res), -1 = zero / none.  The conv is then a row-gathered GEMM
//   y[r] = sum_tap sum_ci x[tap_r][ci] W[co][ci][2 - tap] + b[co],   K = 3C = 384,
// computed in exact fp32 on v_mfma_f32_16x16x4_f32 (LayerNorm needs whole rows, so a
// workgroup owns all 128 output channels of its rows).
//
// Weight-stationary, one 16-row tile at a time, persistent grid:
//   * wave w of 4 owns output channels [32w, 32w + 32): its 32 x 384 weight slice
//     sits in 192 VGPRs for the whole kernel, pre-packed by lg_tcn_pack_weight into
//     fragment order so it loads as 48 coalesced float4;
//   * the tile's gathered rows arrive in LDS by LDS-DMA (buffer_load ... lds, no VGPR
//     staging): K chunk q (16 k) of the 16 rows is one 1 KiB piece whose lane l holds
//     row l % 16, k = 16q + 4(l / 16) .. +3 — exactly the A fragment of four k-steps,
//     so the MFMA loop reads it back with one linear, conflict-free ds_read_b128 per
//     lane and chunk (the packed weights use the same permuted k order); the tile's
//     16 residual rows ride along as 8 more pieces; zero taps / missing rows are
//     out-of-range buffer offsets, which read zeros;
//   * two LDS tile buffers: tile j+1's pieces are issued during tile j's MFMAs;
//   * epilogue: bias (initial accumulator), two-pass LayerNorm over the 128 channels
//     (DPP inside a wave, Chan's merge of the 4 waves' partials through LDS),
//     ReLU, + residual, store; tile j's normalisation and stores run inside tile
//     j+1's K loop, between its MFMAs.
// All K-loop LDS reads are inline asm with explicit lgkmcnt waits: a compiler-visible
// ds_read after an LDS-DMA gets a conservative vmcnt(0), which would serialise the
// next tile's gather with this tile's MFMAs.
// Tiles are dealt XCD-aware (contiguous tile ranges per XCD group, so the rows a
// segment's tiles share stay in one L2).
// Measured (MI355X, B = 256 segments, widest layer): 70-72 us = 88-91 TFLOP/s, 0.56-0.58
// of the fp32 MFMA peak; the K loop runs at the MFMA rate, the remainder is the
// epilogue / side work a single wave per SIMD cannot fully overlap (tools/tcn_prof.cpp).
#include <algorithm>
#include <utility>
#include "common.h"

namespace {

constexpr int kC = 128;             // channels (NormalPredictorTCN hidden_channels default)
constexpr int kK = 3 * kC;          // contraction: 3 taps x C
constexpr int kQ = kK / 16;         // 16-k chunks
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kPieces = kQ / kWaves;    // tap pieces issued per wave and tile
constexpr int kResPieces = kC / 16 / kWaves;  // residual pieces per wave and tile
constexpr int kTileFloats = (kQ + kC / 16) * 256;  // 16 rows x (384 k of taps + 128 residual channels)
constexpr uint32_t kOobOff = 0xFFFF0000u;  // beyond every descriptor (launches stay below 2 GiB per tensor)
constexpr int kPlanMaxRows = 2048;      // LDS-resident plan table (32 KiB)


typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// K-loop LDS reads in inline asm.  A compiler-visible ds_read would be preceded by
// s_waitcnt vmcnt(0) (hipcc cannot tell the in-flight LDS-DMA of the NEXT tile from
// the tile being read), which would serialise the gather with the MFMAs; hidden in
// asm, the reads are ordered by explicit lgkmcnt waits that take the loaded
// registers as in/out operands, so no MFMA can be scheduled above its wait.
template <int OFF>
__device__ __forceinline__ f32x4 ds_read16(uint32_t addr) {
    f32x4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return v;
}
// LDS returns in order, so lgkmcnt(1) retires every LDS read but the newest one (the
// kernel issues no scalar loads inside the tile loop, whose out-of-order returns would
// otherwise count here).
__device__ __forceinline__ void lgkm_wait_but1(f32x4& a) { asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(a)); }
__device__ __forceinline__ void lgkm_wait_all(f32x4& a) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a)); }

template <typename F, int... I>
__device__ __forceinline__ void static_for(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}

__device__ __forceinline__ uint32_t lds_addr(const float* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) float*)p));
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// Sum over the 16 lanes of a DPP row (= one MFMA output column group), result in every
// lane: xor 1, xor 2 (quad_perm), then half-row and row mirrors — VALU only, no LDS.
__device__ __forceinline__ float sum16(float v) {
    v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);  // row_half_mirror
    v += dpp<0x140>(v);  // row_mirror
    return v;
}

struct TileRange {
    uint32_t first, end, stride;
};
// Blocks b and b + 8 share an XCD (round-robin dispatch): XCD group x walks the x-th
// contiguous eighth of the tiles.  Only placement changes; every tile is visited once.
__device__ __forceinline__ TileRange xcd_tiles(uint32_t ntiles) {
    const uint32_t G = gridDim.x, b = blockIdx.x;
    if (G < 8) return TileRange{b, ntiles, G};
    const uint32_t x = b % 8, k = b / 8, nbx = (G - x + 7) / 8, chunk = (ntiles + 7) / 8;
    const uint32_t begin = x * chunk, end = min(ntiles, begin + chunk);
    return TileRange{begin + k, end, nbx};
}

struct ConvArgs {
    const float* in;      // [nseg * rows_in][C]
    const float* blk;     // [nseg * rows_blk][C] or null
    const int4* plan;     // [rows_out] (tap0, tap1, tap2, res)
    const float* wpk;     // packed weight, fragment order
    const float* bias;
    const float* ln_w;
    const float* ln_b;
    float* out;           // [nseg * rows_out][C]
    float eps;
    uint32_t total_rows;  // nseg * rows_out
    uint32_t rows_in, rows_blk, rows_out;
    lg_fastdiv seg_of;    // row -> segment (divisor rows_out)
    uint32_t ntiles;
    uint32_t in_bytes;    // nseg * rows_in * C * 4 (< 2 GiB per launch)
    uint32_t blk_bytes;   // nseg * rows_blk * C * 4, 0 without a residual
};

typedef int i32x4 __attribute__((ext_vector_type(4)));

// Side-work LDS reads inside the K loop, also in asm (see ds_read16): issued in chunk q,
// retired by the lgkmcnt(1) wait at the end of chunk q + 1 (LDS returns in order and a
// newer ring read is outstanding by then), tied there and consumed from chunk q + 2.
__device__ __forceinline__ f32x4 ds_read16v(uint32_t addr) {
    f32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}
__device__ __forceinline__ i32x4 ds_read16i(uint32_t addr) {
    i32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}
__device__ __forceinline__ int ds_read4i(uint32_t addr) {
    int v;
    asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}
template <typename T>
__device__ __forceinline__ void tie(T& v) {
    asm volatile("" : "+v"(v));
}

// Output rows through a buffer descriptor: a row past the end gets an out-of-range
// offset and the hardware drops the store (no branch in the MFMA stream).
__device__ __forceinline__ void store_out(__amdgpu_buffer_rsrc_t rs, uint32_t row, bool ok, int col, float v) {
    const uint32_t off = ok ? (row * kC + col) * 4u : 0xFFFFFFF0u;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rs, off, 0, 0);
}

// Finished accumulators of one tile, carried into the next tile's K loop where their
// LayerNorm / ReLU / residual epilogue runs between the MFMAs.
struct Pending {
    float v0[4], v1[4];   // conv + bias, channels 32w + c16 and 32w + 16 + c16, rows 4g + i
    float res[4][2];
    uint32_t tile;
    int par;
    bool live;
};


__global__ __launch_bounds__(kThreads) void k_tcn_conv(ConvArgs a) {
    // tiles[b]: pieces 0..23 = the gathered tap rows (A fragments), pieces 24..31 = the
    // tile's 16 residual rows (block input) in the same fragment layout
    __shared__ __attribute__((aligned(16))) float tiles[2][kTileFloats];
    __shared__ __attribute__((aligned(16))) float red[2][16][2][kWaves];  // [tile parity][row][mean, M2][wave]
    extern __shared__ int4 plan_s[];

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
    for (uint32_t i = threadIdx.x; i < a.rows_out; i += kThreads) plan_s[i] = a.plan[i];

    f32x4 wr[kQ][2];
#pragma unroll
    for (int q = 0; q < kQ; ++q)
#pragma unroll
        for (int c = 0; c < 2; ++c) wr[q][c] = ld4(a.wpk + ((((w * kQ + q) * 2 + c) * 64) + lane) * 4);
    float bias[2], gam[2], bet[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int co = 32 * w + 16 * c + c16;
        bias[c] = a.bias[co];
        gam[c] = a.ln_w[co];
        bet[c] = a.ln_b[co];
    }
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        a.out, static_cast<short>(0), static_cast<int>(a.total_rows * (4u * kC)), 0x00020000);
    const __amdgpu_buffer_rsrc_t irs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.in), static_cast<short>(0), static_cast<int>(a.in_bytes), 0x00020000);
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.blk), static_cast<short>(0), static_cast<int>(a.blk_bytes), 0x00020000);
    const uint32_t plan_lds = lds_addr(reinterpret_cast<const float*>(plan_s));
    const uint32_t red_lds = lds_addr(&red[0][0][0][0]);
    __syncthreads();  // plan table staged

    // ---- LDS-DMA of one tile: this wave's 6 tap pieces (q = 6w + u: tap q / 8,
    // channels 16 (q % 8) + 4 (l / 16) .. +3 of row l % 16) and 2 residual pieces
    // (channels 16 (2w + v) + 4 (l / 16) .. +3).  Byte offsets into `in` / `blk`; a zero
    // tap, a missing residual or a row past the end reads out of range, i.e. zeros.
    uint32_t doff[kPieces + kResPieces];
    auto dma_offsets = [&](bool ok, uint32_t seg, i32x4 p) {
        const uint32_t row_in = seg * a.rows_in, row_blk = seg * a.rows_blk;
        const uint32_t o0 = ok && p.x >= 0 ? (row_in + p.x) * (4u * kC) : kOobOff;
        const uint32_t o1 = ok && p.y >= 0 ? (row_in + p.y) * (4u * kC) : kOobOff;
        const uint32_t o2 = ok && p.z >= 0 ? (row_in + p.z) * (4u * kC) : kOobOff;
        const uint32_t orr = ok && p.w >= 0 ? (row_blk + p.w) * (4u * kC) : kOobOff;
#pragma unroll
        for (int u = 0; u < kPieces; ++u) {
            const int q = w * kPieces + u;
            const int tap = q >> 3;  // wave-uniform; mask selects keep this out of scratch
            const uint32_t ot = (o0 & (0u - (tap == 0))) | (o1 & (0u - (tap == 1))) | (o2 & (0u - (tap == 2)));
            doff[u] = ot + (16 * (q & 7) + 4 * g) * 4;
        }
#pragma unroll
        for (int v = 0; v < kResPieces; ++v) doff[kPieces + v] = orr + (16 * (kResPieces * w + v) + 4 * g) * 4;
    };
    auto issue_piece = [&](float* buf, int u) {  // u < kPieces: tap piece, else residual piece
        if (u < kPieces)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(irs, (lds_ptr_t)(buf + (w * kPieces + u) * 256), 16, doff[u], 0,
                                                     0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                brs, (lds_ptr_t)(buf + (kQ + kResPieces * w + (u - kPieces)) * 256), 16, doff[u], 0, 0, 0);
    };
    // plan row of this lane's DMA row (l % 16) in tile `tile`; ok = a real row
    auto dma_row = [&](uint32_t tile, bool& ok, uint32_t& seg) -> uint32_t {
        const uint32_t row = tile * 16 + (lane & 15);
        ok = tile < a.ntiles && row < a.total_rows;
        const uint32_t rc = ok ? row : 0u;
        seg = lg_div(rc, a.seg_of);
        return rc - seg * a.rows_out;
    };

    // Schedule (one barrier per tile, two LDS tile buffers): tile j's K loop reads
    // tiles[j % 2] while the pieces of tile j+1 are issued into tiles[(j+1) % 2], one
    // per chunk over the first chunks of the loop (that buffer held tile j-1, which
    // every wave finished before barrier j-1).  Each wave retires its pieces (vmcnt)
    // before barrier j, so tile j+1 has landed for everyone after it.  Between two K
    // loops only the LayerNorm partial sums and the barrier run; tile j-1's
    // normalisation and stores, the read of tile j's residual rows and tile j+2's DMA
    // offsets are side work inside tile j's K loop.  The loop never waits on its own
    // output stores (vmcnt counts stores on gfx9): they retire during later MFMAs.
    const TileRange tr = xcd_tiles(a.ntiles);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t t = tr.first + k * tr.stride;
        bool ok;
        uint32_t seg;
        const uint32_t pr = dma_row(t, ok, seg);
        dma_offsets(ok && t < tr.end, seg, *reinterpret_cast<const i32x4*>(&plan_s[pr]));
        if (k == 0 && t < tr.end)
#pragma unroll
            for (int u = 0; u < kPieces + kResPieces; ++u) issue_piece(tiles[0], u);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    Pending pd;
    pd.live = false;
    pd.tile = 0;
    pd.par = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) pd.v0[i] = pd.v1[i] = pd.res[i][0] = pd.res[i][1] = 0.f;

    float lsc[4][2], lsh[4][2];  // folded LayerNorm affine of the pending rows: y = v * lsc + lsh
    f32x4 rsum[4], rm2[4];       // the 4 waves' (mean, M2) partials of the pending tile's rows 4g+i
    auto read_stats = [&]() {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t ad = red_lds + ((pd.par * 16 + 4 * g + i) * 2 * kWaves) * 4;
            rsum[i] = ds_read16v(ad);
            rm2[i] = ds_read16v(ad + 16);
        }
    };
    auto tie_stats = [&]() {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            tie(rsum[i]);
            tie(rm2[i]);
        }
    };
    auto ln_stats = [&](int i) {  // Chan's parallel merge of the four waves' (mean, M2)
        const f32x4 m = rsum[i], q2 = rm2[i];
        const float mu = 0.25f * ((m[0] + m[1]) + (m[2] + m[3]));
        const float e0 = m[0] - mu, e1 = m[1] - mu, e2 = m[2] - mu, e3 = m[3] - mu;
        const float M2 = ((q2[0] + q2[1]) + (q2[2] + q2[3])) + 32.0f * ((e0 * e0 + e1 * e1) + (e2 * e2 + e3 * e3));
        const float rs = rsqrtf(M2 * (1.0f / kC) + a.eps);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            lsc[i][c] = rs * gam[c];
            lsh[i][c] = bet[c] - mu * lsc[i][c];
        }
    };
    auto finish_row = [&](int i) {
        const uint32_t orow = pd.tile * 16 + 4 * g + i;
        const bool ok = pd.live && orow < a.total_rows;
        const float y0 = fmaxf(fmaf(pd.v0[i], lsc[i][0], lsh[i][0]), 0.f) + pd.res[i][0];
        const float y1 = fmaxf(fmaf(pd.v1[i], lsc[i][1], lsh[i][1]), 0.f) + pd.res[i][1];
        store_out(ors, orow, ok, 32 * w + c16, y0);
        store_out(ors, orow, ok, 32 * w + 16 + c16, y1);
    };

    int buf = 0;
    for (uint32_t tile = tr.first; tile < tr.end; tile += tr.stride, buf ^= 1) {
        float res[4][2];
        i32x4 dplan;
        bool dok = false;
        uint32_t dseg = 0;
        // K loop: chunk q's A fragment (1 KiB piece q of the tile) is read two chunks
        // ahead into a 3-register ring; the wait after step q's MFMAs retires chunk q + 1
        // (and every older LDS read).  Side work is hooked between chunks.
        const uint32_t abase = lds_addr(tiles[buf]) + lane * 16;
        // residual of this lane's (row 4g+i, channel 32w + 16c + c16) in the fragment
        // layout of pieces 24..31
        const uint32_t rbase = lds_addr(tiles[buf]) + (kQ + 2 * w) * 1024 + (16 * (c16 >> 2) + 4 * g) * 16 +
                               (c16 & 3) * 4;
        f32x4 acc0 = {bias[0], bias[0], bias[0], bias[0]};
        f32x4 acc1 = {bias[1], bias[1], bias[1], bias[1]};
        f32x4 ring[3];
        ring[0] = ds_read16<0>(abase);
        ring[1] = ds_read16<1024>(abase);
        lgkm_wait_all(ring[0]);
        static_for(
            [&](auto qc) {
                constexpr int q = decltype(qc)::value;
                if constexpr (q + 2 < kQ) ring[(q + 2) % 3] = ds_read16<(q + 2) * 1024>(abase);
                const f32x4 av = ring[q % 3];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc0 = mfma(av[j], wr[q][0][j], acc0);
                    acc1 = mfma(av[j], wr[q][1][j], acc1);
                }
                // ---- side work ----
#ifndef TCN_NOHOOK
                if constexpr (q < kPieces + kResPieces) issue_piece(tiles[buf ^ 1], q);  // tile j+1
                if constexpr (q == 0) read_stats();
                if constexpr (q >= 2 && q <= 5) ln_stats(q - 2);
                if constexpr (q >= 3 && q <= 6) finish_row(q - 3);
                if constexpr (q == 8) {
                    const uint32_t pr = dma_row(tile + 2 * tr.stride, dok, dseg);
                    dok = dok && tile + 2 * tr.stride < tr.end;  // else all pieces read zeros (unused)
                    dplan = ds_read16i(plan_lds + pr * 16);
                }
                if constexpr (q == 10) dma_offsets(dok, dseg, dplan);
                if constexpr (q == 14) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        res[i][0] = __builtin_bit_cast(float, ds_read4i(rbase + i * 16));
                        res[i][1] = __builtin_bit_cast(float, ds_read4i(rbase + 1024 + i * 16));
                    }
                }
#endif
                // ---- waits ----
                if constexpr (q + 2 < kQ)
                    lgkm_wait_but1(ring[(q + 1) % 3]);  // chunk q + 2 may stay in flight
                else if constexpr (q + 1 < kQ)
                    lgkm_wait_all(ring[(q + 1) % 3]);
#ifndef TCN_NOHOOK
                if constexpr (q == 1) tie_stats();
                if constexpr (q == 9) tie(dplan);
                if constexpr (q == 10)
#pragma unroll
                    for (int u = 0; u < kPieces + kResPieces; ++u) tie(doff[u]);  // computed here, not sunk
                if constexpr (q == 15)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        tie(res[i][0]);
                        tie(res[i][1]);
                    }
#endif
            },
            std::make_integer_sequence<int, kQ>{});
        // LayerNorm partials of this tile: each wave reduces its 32 channels exactly
        // (two-pass mean / M2 inside the wave, DPP only); the four waves' (mean, M2)
        // are merged by ln_stats with Chan's parallel formula.
        float mw[4], m2[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) mw[i] = sum16(acc0[i] + acc1[i]) * (1.0f / 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float d0 = acc0[i] - mw[i], d1 = acc1[i] - mw[i];
            m2[i] = sum16(d0 * d0 + d1 * d1);
        }
        if (c16 == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                red[buf][4 * g + i][0][w] = mw[i];
                red[buf][4 * g + i][1][w] = m2[i];
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            pd.v0[i] = acc0[i];
            pd.v1[i] = acc1[i];
            pd.res[i][0] = res[i][0];
            pd.res[i][1] = res[i][1];
        }
        pd.tile = tile;
        pd.par = buf;
        pd.live = true;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile j+1
        __syncthreads();
    }
    if (pd.live) {
        read_stats();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        tie_stats();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            ln_stats(i);
            finish_row(i);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outstanding at exit
}

// Packed weight: wpk[w][q][c][lane][j] = W[co][ci][2 - tap] with co = 32w + 16c + lane % 16,
// k = 16q + 4(lane / 16) + j, tap = k / C, ci = k % C.
__global__ void k_tcn_pack_weight(const float* __restrict__ weight, float* __restrict__ wpk) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= static_cast<uint32_t>(kC * kK)) return;
    const uint32_t j = i & 3, lane = (i >> 2) & 63, c = (i >> 8) & 1, q = (i >> 9) % kQ, w = (i >> 9) / kQ;
    const uint32_t co = 32 * w + 16 * c + (lane & 15), k = 16 * q + 4 * (lane >> 4) + j;
    const uint32_t tap = k / kC, ci = k % kC;
    wpk[i] = weight[(co * kC + ci) * 3 + (2 - tap)];
}

}  // namespace

extern "C" {

int64_t lg_tcn_packed_weight_floats(int64_t C) { return C == kC ? int64_t{kC} * kK : 0; }

int lg_tcn_pack_weight(const float* weight, float* packed, int64_t C, lg_stream_t stream) {
    if (C != kC) return LG_EUNSUPPORTED;
    if (weight == nullptr || packed == nullptr) return LG_EINVAL;
    const int n = kC * kK;
    k_tcn_pack_weight<<<(n + 255) / 256, 256, 0, lg_stream(stream)>>>(weight, packed);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

int lg_tcn_conv_fwd(const float* in, const float* blk, const int32_t* plan, const float* packed_weight,
                    const float* bias, const float* ln_w, const float* ln_b, float eps, float* out, int64_t nseg,
                    int64_t rows_in, int64_t rows_blk, int64_t rows_out, int64_t C, lg_stream_t stream) {
    if (C != kC) return LG_EUNSUPPORTED;
    if (nseg < 0 || rows_in <= 0 || rows_out <= 0 || rows_out > kPlanMaxRows || (blk != nullptr && rows_blk <= 0))
        return LG_EINVAL;
    if (in == nullptr || plan == nullptr || packed_weight == nullptr || bias == nullptr || ln_w == nullptr ||
        ln_b == nullptr || out == nullptr)
        return LG_EINVAL;
    if (nseg == 0) return LG_OK;
    if (nseg * rows_in >= kLgMaxRows || nseg * std::max<int64_t>(rows_blk, 0) >= kLgMaxRows) return LG_EUNSUPPORTED;
    // output rows are stored through a buffer descriptor (32-bit byte offsets): split
    // the segments so that each launch's output stays below 4 GiB
    // rows are addressed through buffer descriptors (32-bit byte offsets, out-of-range
    // offsets read zero / drop the store): split the segments so that each launch's
    // tensors stay below 2 GiB
    const int64_t widest = std::max(std::max(rows_out, rows_in), std::max<int64_t>(rows_blk, 0));
    const int64_t seg_cap = std::max<int64_t>(1, (int64_t{1} << 31) / (widest * kC * 4));
    const size_t dyn = static_cast<size_t>(rows_out) * sizeof(int4);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_tcn_conv, kThreads, dyn) != hipSuccess || per_cu < 1)
        per_cu = 1;
    for (int64_t s0 = 0; s0 < nseg; s0 += seg_cap) {
        const int64_t ns = std::min(seg_cap, nseg - s0);
        const int64_t total = ns * rows_out;
        ConvArgs a;
        a.in = in + s0 * rows_in * kC;
        a.blk = blk != nullptr ? blk + s0 * rows_blk * kC : nullptr;
        a.plan = reinterpret_cast<const int4*>(plan);
        a.wpk = packed_weight;
        a.bias = bias;
        a.ln_w = ln_w;
        a.ln_b = ln_b;
        a.out = out + s0 * rows_out * kC;
        a.eps = eps;
        a.total_rows = static_cast<uint32_t>(total);
        a.rows_in = static_cast<uint32_t>(rows_in);
        a.rows_blk = static_cast<uint32_t>(std::max<int64_t>(rows_blk, 0));
        a.rows_out = static_cast<uint32_t>(rows_out);
        a.seg_of = lg_make_fastdiv(static_cast<uint32_t>(rows_out));
        a.ntiles = static_cast<uint32_t>((total + 15) / 16);
        a.in_bytes = static_cast<uint32_t>(ns * rows_in * kC * 4);
        a.blk_bytes = blk != nullptr ? static_cast<uint32_t>(ns * rows_blk * kC * 4) : 0u;
        const int64_t grid = std::min<int64_t>(a.ntiles, int64_t{per_cu} * lg_num_cus());
        k_tcn_conv<<<static_cast<unsigned>(grid), kThreads, dyn, lg_stream(stream)>>>(a);
        if (hipGetLastError() != hipSuccess) return LG_EHIP;
    }
    return LG_OK;
}

}  // extern "C"
