// Fused GCN layer forward / backward in the NODE-MAJOR layout of the LeakDetector trunk.
//
// Layout: node features [N][B][D] (row r = n*B + b): the B windows of one node are
// contiguous.  Every window carries the same graph, so a 16-row tile is ONE node n and 16
// consecutive windows b0..b0+15 (a "window group"), and its aggregation
//     (Ahat x)[n][b0..b0+15][:] = sum_{m in N(n)} w_nm x[m][b0..b0+15][:]
// reads one contiguous 16 x D block per neighbour (4 KiB at D = 64):
//   * the CSR entry (m, w_nm) is wave-uniform (scalar loads of (col, w) pairs),
//   * the degree is uniform (no padded neighbour slots),
//   * row loads are buffer loads with a scalar base and a per-lane constant offset —
//     no per-lane index or address arithmetic; a ragged last window group masks rows.
// Compared with the window-major kernels (gcn.hip) this removes most of the per-row VALU
// work that bounded them (measured: 35.7 -> 24.4 us per train-mode layer at B = 256, and
// 0.57 of the HBM peak at B = 1024).
//
// Forward: aggregate -> LDS -> MFMA B operand, y^T = W (Ahat x)^T on
// v_mfma_f32_16x16x4_f32 (exact fp32), bias as the initial accumulator, ReLU, row-stream
// dropout with the 1/(1-p) scale folded into W and b, rows written back through LDS as
// one contiguous block with plain (cacheable) stores: the next launch (the next layer, the
// heads) reads y, and a non-temporal store sent it past the Infinity Cache — measured, the
// layer reading a non-temporally written input ran 28-31 us instead of 20 us.
// Backward: t = Ahat^T dz (transposed CSR, dz = dy * s * [y > 0] when MASK_IN), dx = t W
// (MFMA, masked by the input's [x > 0] * s), dW += t^T x and db += sum dz accumulated per
// wave and reduced per block in a fixed order (deterministic), then by the slab reducer.
// Tiles are ordered window-group-major and dealt XCD-aware.
#include <algorithm>
#include <type_traits>
#include "common.h"
#include "reduce.h"
#include "split_bf16.h"

namespace {

constexpr int kNmBwdWaves3 = 4;

__device__ __forceinline__ f32x4 mfma_nm(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void wave_sync_nm() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    asm volatile("" ::: "memory");
}

template <int D>
struct NmGeo {
    static constexpr int LPR = D / 4;     // lanes per row (one float4 each)
    static constexpr int RPI = 64 / LPR;  // rows per wave instruction
    static constexpr int K = 16 / RPI;    // instructions per 16-row block
    static constexpr int CH = D / 16;     // MFMA k chunks = output blocks
    static constexpr int S = D + 4;       // LDS row stride (floats)
    static constexpr int TILE = 16 * S;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t nm_rsrc(const float* p, uint64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), static_cast<short>(0), static_cast<int>(bytes),
                                             0x00020000);
}

// 16-byte buffer stores read their data VGPRs after issue: keep those registers unwritten for a
// few wait states.  Measured on k_gcn_bwd_pc (tools/bpc_check.py; profiles/r03/r03q-r03t): the
// compiler reused a store's data registers for VALU results 0-1 instructions after the
// buffer_store_dwordx4 and dwords 0-1 of some lanes went out overwritten (~1 % of dx rows).
// Call after the last store of a tile with all of its data values.
template <int K>
__device__ __forceinline__ void lg_store_guard(const f32x4 (&v)[K]) {
    if constexpr (K == 4) asm volatile("s_nop 7" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
    else if constexpr (K == 2) asm volatile("s_nop 7" ::"v"(v[0]), "v"(v[1]));
    else asm volatile("s_nop 7" ::"v"(v[0]));
}

// Tile -> (node, window group) and the XCD-aware persistent schedule over groups * N tiles.
struct NmSched {
    int64_t first, end, stride;
};
__device__ __forceinline__ NmSched nm_sched(int64_t ntiles, int wave, int waves) {
    const int64_t G = gridDim.x, b = blockIdx.x;
    if (G < 8) return NmSched{b * waves + wave, ntiles, G * waves};
    const int64_t x = b % 8, k = b / 8, nbx = (G - x + 7) / 8, chunk = (ntiles + 7) / 8;
    return NmSched{x * chunk + k * waves + wave, std::min<int64_t>(ntiles, x * chunk + chunk), nbx * waves};
}

// ------------------------------------------------------------------ forward, node-table pipeline
// k_gcn_fwd_nm2's math with the CSR read from the node table (graph.hip k_nm_table): one
// 64-byte record per node holds (e0, e1) and its first kLgNmInline (col, w) pairs, read by
// a single scalar load.  nm2 walked rowptr -> pair -> pair ... as dependent scalar round
// trips before each tile's row loads could issue, and the MFMA transform waited behind
// them (SMEM and LDS share lgkmcnt).  Here the record of tile i+1 is requested at the top
// of tile i and lands while tile i's rows are waited for and accumulated, so tile i+1's
// NPF neighbour blocks issue at once, right before tile i's transform.  (A record carried
// across the loop back edge in SGPRs is copied there, and the copy waits for the load.)
#ifndef LG_NM3_NPF
#define LG_NM3_NPF 3  // lab builds override (-DLG_NM3_NPF=n); 3 measured best of 2-5 (tools/exp_r02an.sh)
#endif
constexpr int kNm3Npf = LG_NM3_NPF;

struct NmRec {  // one node-table record (wave-uniform, SGPRs)
    int e0, e1, self, node;
    int2 p[kLgNmInline];
};

__device__ __forceinline__ NmRec nm_rec(const int32_t* __restrict__ tab, uint32_t n) {
    const int4* t = reinterpret_cast<const int4*>(tab) + 4 * static_cast<size_t>(n);
    const int4 a = t[0], b = t[1], c = t[2], d = t[3];
    NmRec r;
    r.e0 = a.x;
    r.e1 = a.y;
    r.p[0] = int2{a.z, a.w};
    r.p[1] = int2{b.x, b.y};
    r.p[2] = int2{b.z, b.w};
    r.p[3] = int2{c.x, c.y};
    r.p[4] = int2{c.z, c.w};
    r.p[5] = int2{d.x, d.y};
    r.self = d.z;
    r.node = d.w;
    return r;
}
static_assert(kLgNmInline == 6, "nm_rec unpacks six inline pairs");

template <int D, bool SPLIT, int WAVES>
struct Nm3Lds {  // dynamic LDS layout (floats)
    static constexpr int SB = D + 8;
    static constexpr int WF = SPLIT ? (3 * D * SB) / 2 : D * NmGeo<D>::S;
    static constexpr int TILES = WF + D;
    static constexpr int TILE = NmGeo<D>::TILE;
    static constexpr size_t BYTES = 4 * static_cast<size_t>(TILES + WAVES * TILE);
    // float offset of 16-byte chunk c of row r in a wave's tile
    static __device__ __forceinline__ int tix(int r, int c) { return r * NmGeo<D>::S + 4 * c; }
};

#if defined(LG_NM3_STAMPS) || defined(LG_PC_PROBE)
// kernel-lab timeline (LG_NM3_STAMPS builds only): per wave, slot 0 realtime at start, 1 clock
// at start, 2 after the W staging barrier, 3 + 3 t .. 5 + 3 t for tile t < 6 (rows
// accumulated, transform done, stores issued), 21 clock at end, 22 realtime at end, 23 hw id.
// LG_PC_PROBE builds (k_gcn_fwd_pc only): the same slots 0, 1, 2, 21, 22, 23 and the wave's
// tile count in slot 3, all held in registers and stored once at the wave's end, so the
// kernel runs at product speed (the per-tile stamps' s_memtime waits on lgkmcnt, which also
// drains the record prefetch and the LDS traffic: that build runs 2.9x slow).
constexpr int kNm3Stamps = 24;
__device__ uint64_t g_nm3_stamps[8192 * kNm3Stamps];
#endif
#ifdef LG_NM3_STAMPS
#define LG_NM3_STAMP(slot, v)                                                                      \
    do {                                                                                           \
        if (lane == 0) g_nm3_stamps[(static_cast<size_t>(blockIdx.x) * WAVES + wave) * kNm3Stamps + (slot)] = (v); \
    } while (0)
#else
#define LG_NM3_STAMP(slot, v) \
    do {                      \
    } while (0)
#endif

// acc += w * v on packed fp32 (v_pk_fma_f32: two lanes' worth of fma per instruction,
// each element the same IEEE fma as fmaf)
__device__ __forceinline__ void pk_fma4(f32x4& a, float w, const f32x4& v) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 ww = {w, w};
    const f2 lo = __builtin_elementwise_fma(ww, f2{v[0], v[1]}, f2{a[0], a[1]});
    const f2 hi = __builtin_elementwise_fma(ww, f2{v[2], v[3]}, f2{a[2], a[3]});
    a = f32x4{lo[0], lo[1], hi[0], hi[1]};
}

// Output mask of a layer (ymask, lg_gcn_fwd_nm_bits): per 16-row tile (node n, window
// group g) one uint16 per lane of the gather layout, bit 4 k + i = [y > 0] of the lane's
// slot k, element i; 128 bytes per tile at ((n * ngroups + g) * 64 + lane) * 2.  The
// backward reads it instead of gathering y (1/32 of the bytes).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t nm_mask_rsrc(const uint16_t* p, uint32_t N, uint32_t ngroups) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p), static_cast<short>(0),
                                             static_cast<int>(static_cast<uint64_t>(N) * ngroups * 128u), 0x00020000);
}
__device__ __forceinline__ uint32_t nm_mask_off(uint32_t n, uint32_t grp, uint32_t ngroups, int lane) {
    return (n * ngroups + grp) * 128u + 2u * static_cast<uint32_t>(lane);
}

// Out-of-range offsets of the nm3 addressing: a lane offset of a masked row is kNm3RowOob
// and an absent neighbour's block base is kNm3BlkOob, so lane + base lands past
// num_records (<= kNm3MaxBytes) with ONE v_add per load and no wrap-around.
constexpr uint32_t kNm3RowOob = 0x80000000u;
constexpr uint32_t kNm3BlkOob = 0x7FFFF000u;
constexpr uint64_t kNm3MaxBytes = 0x7FFFF000u;

// BF (LG_F_BF16, the bf16 node-MLP tier): the transform's single hi x hi product.
template <int D, bool DROP, bool RELU, bool SPLIT, int WAVES, bool BF = false>
__global__ void __launch_bounds__(64 * WAVES, WAVES >= 5 ? 4 : 1)
k_gcn_fwd_nm3(const int32_t* __restrict__ tab, const int2* __restrict__ pairs, const float* __restrict__ x,
              const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ y, uint32_t N,
              uint32_t B, uint32_t ngroups, lg_fastdiv fdN, float p_drop, float dscale, uint64_t seed,
              uint32_t salt, uint16_t* __restrict__ ymask) {
    using G = NmGeo<D>;
    using LY = Nm3Lds<D, SPLIT, WAVES>;
    constexpr int SB = LY::SB;
    constexpr int NPF = kNm3Npf;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* wl = reinterpret_cast<float*>(smem);         // fp32: W [out][in] * fold, stride S
    uint16_t* wsl = reinterpret_cast<uint16_t*>(smem);  // SPLIT: 3 x [out][in] bf16, stride SB
    float* bl = wl + LY::WF;                            // bias * fold
    float* tiles = wl + LY::TILES;

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const int rl = lane / G::LPR, fg = lane % G::LPR;
#ifdef LG_NM3_STAMPS
    LG_NM3_STAMP(0, __builtin_amdgcn_s_memrealtime());
    LG_NM3_STAMP(1, __builtin_amdgcn_s_memtime());
#endif
    float* tl = tiles + wave * LY::TILE;
    const uint64_t bytes = static_cast<uint64_t>(N) * B * (4u * D);
    const __amdgpu_buffer_rsrc_t xrs = nm_rsrc(x, bytes), yrs = nm_rsrc(y, bytes);
    const __amdgpu_buffer_rsrc_t mrs = nm_mask_rsrc(ymask, N, ngroups);
    uint32_t loff[G::K];  // byte offset in a 16-row block of this lane's slot k (row RPI k + rl)
#pragma unroll
    for (int k = 0; k < G::K; ++k) loff[k] = (G::RPI * k + rl) * (4u * D) + 16u * fg;
    const NmSched sc = nm_sched(static_cast<int64_t>(ngroups) * N, wave, WAVES);
    const int64_t tend = sc.end;

    auto tile_coords = [&](int64_t tile, uint32_t& n, uint32_t& b0, uint32_t& nb) {
        const bool valid = tile < tend;
        const uint32_t t32 = static_cast<uint32_t>(valid ? tile : 0);
        const uint32_t grp = lg_div(t32, fdN);
        n = t32 - grp * N;
        b0 = grp * 16;
        nb = valid ? min(16u, B - b0) : 0u;
    };
    // tile in flight: its record, coordinates, lane offsets and first NPF neighbour blocks
    f32x4 pf[NPF][G::K];
    uint32_t lo[G::K];  // loff, or kNm3RowOob for rows past the tile's window count
    NmRec cur;
    uint32_t cn, cb0;
    auto issue = [&](const NmRec& r, uint32_t n, uint32_t b0, uint32_t nb) {
        n = static_cast<uint32_t>(r.node);  // tiles run in the table's schedule order (slot -> node)
        cur = r;
        cn = n;
        cb0 = b0;
#pragma unroll
        for (int k = 0; k < G::K; ++k) lo[k] = (G::RPI * k + rl) < static_cast<int>(nb) ? loff[k] : kNm3RowOob;
#pragma unroll
        for (int i = 0; i < NPF; ++i) {
            const bool have = r.e0 + i < r.e1;
            const uint32_t base = have ? (static_cast<uint32_t>(r.p[i].x) * B + b0) * (4u * D) : kNm3BlkOob;
#pragma unroll
            for (int k = 0; k < G::K; ++k)
                pf[i][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, lo[k] + base, 0, 0));
        }
    };
    // a present neighbour's block (the rows past the prefetched ones)
    auto ldblk = [&](uint32_t base, uint32_t lk) -> f32x4 {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, lk + base, 0, 0));
    };
    const int64_t t0 = sc.first;
    // W (x dropout scale fold) and bias to LDS
    constexpr int W4 = D * D / 4, WPER = (W4 + 64 * WAVES - 1) / (64 * WAVES);
    f32x4 wv[WPER];
    float bb = 0.f;
    auto load_w = [&]() {
#pragma unroll
        for (int u = 0; u < WPER; ++u) wv[u] = ld4(W + 4 * min<int>(u * 64 * WAVES + threadIdx.x, W4 - 1));
        bb = (bias && threadIdx.x < D) ? bias[threadIdx.x] : 0.f;
    };
    {
        uint32_t n0, b00, nb00;
        tile_coords(t0, n0, b00, nb00);
        issue(nm_rec(tab, N + n0), n0, b00, nb00);  // schedule section
    }
    load_w();
    {
        const float fold = DROP ? dscale : 1.0f;  // relu(s z) = s relu(z), s > 0
#pragma unroll
        for (int u = 0; u < WPER; ++u) {
            const int i = u * 64 * WAVES + threadIdx.x;
            if (i >= W4) continue;
            const int o = i / (D / 4), c4 = 4 * (i % (D / 4));
            // the product rounded to fp32 before the split, as every other staging path stores it
            // (the empty asm keeps -ffp-contract from fusing it into the split's residual)
            f32x4 w = wv[u] * fold;
            asm volatile("" : "+v"(w));
            if constexpr (SPLIT) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    uint32_t p0, p1, p2;
                    split3_pair(w[2 * h], w[2 * h + 1], p0, p1, p2);
                    const int e = o * SB + c4 + 2 * h;
                    *reinterpret_cast<uint32_t*>(wsl + e) = p0;
                    *reinterpret_cast<uint32_t*>(wsl + D * SB + e) = p1;
                    *reinterpret_cast<uint32_t*>(wsl + 2 * D * SB + e) = p2;
                }
            } else {
                st4(wl + o * G::S + c4, w);
            }
        }
        if (threadIdx.x < D) bl[threadIdx.x] = bb * fold;
    }
    __syncthreads();

    const uint32_t key = lg_dropout_key_dev(seed, salt);
    const uint32_t thr = lg_keep_threshold16(p_drop);

    int tcount = 0;
    (void)tcount;
    LG_NM3_STAMP(2, __builtin_amdgcn_s_memtime());
    for (int64_t tile = t0; tile < tend; tile += sc.stride) {
        const uint32_t n = cn, b0 = cb0;
        const int e0 = cur.e0, e1 = cur.e1;
        uint32_t tlo[G::K];
#pragma unroll
        for (int k = 0; k < G::K; ++k) tlo[k] = lo[k];
        // the next tile's record goes in flight while this tile's rows are waited for
        uint32_t nn, nb0, nnb;
        tile_coords(tile + sc.stride, nn, nb0, nnb);
        const NmRec nxt = nm_rec(tab, N + nn);
        asm volatile("" ::: "memory");  // keep the request here: the compiler would sink it to its use
        // CSR order from 0: the first term is the product itself (an absent first neighbour
        // loaded zeros, and its weight is taken as 0), the rest fma'd in
        f32x4 acc[G::K];
        {
            const float w = e0 < e1 ? __int_as_float(cur.p[0].y) : 0.f;
#pragma unroll
            for (int k = 0; k < G::K; ++k) acc[k] = pf[0][k] * w;
        }
#pragma unroll
        for (int i = 1; i < NPF; ++i) {
            if (e0 + i < e1) {
                const float w = __int_as_float(cur.p[i].y);
#pragma unroll
                for (int k = 0; k < G::K; ++k) pk_fma4(acc[k], w, pf[i][k]);
            }
        }
        // neighbours past the prefetched ones (degree > NPF): inline pairs, then the pair array
        if (e0 + NPF < e1) {
            int2 ip[kLgNmInline - NPF];
#pragma unroll
            for (int i = 0; i < kLgNmInline - NPF; ++i) ip[i] = cur.p[NPF + i];
#pragma unroll
            for (int i = 0; i < kLgNmInline - NPF; ++i) {
                if (e0 + NPF + i < e1) {
                    const uint32_t ba = (static_cast<uint32_t>(ip[i].x) * B + b0) * (4u * D);
                    f32x4 va[G::K];
#pragma unroll
                    for (int k = 0; k < G::K; ++k) va[k] = ldblk(ba, tlo[k]);
                    const float wa = __int_as_float(ip[i].y);
#pragma unroll
                    for (int k = 0; k < G::K; ++k) pk_fma4(acc[k], wa, va[k]);
                }
            }
            int e = e0 + kLgNmInline;
            for (; e + 1 < e1; e += 2) {
                const int2 pa = pairs[e], pb = pairs[e + 1];
                const uint32_t ba = (static_cast<uint32_t>(pa.x) * B + b0) * (4u * D);
                const uint32_t bbs = (static_cast<uint32_t>(pb.x) * B + b0) * (4u * D);
                f32x4 va[G::K], vb[G::K];
#pragma unroll
                for (int k = 0; k < G::K; ++k) {
                    va[k] = ldblk(ba, tlo[k]);
                    vb[k] = ldblk(bbs, tlo[k]);
                }
                const float wa = __int_as_float(pa.y), wb = __int_as_float(pb.y);
#pragma unroll
                for (int k = 0; k < G::K; ++k) {
                    pk_fma4(acc[k], wa, va[k]);
                    pk_fma4(acc[k], wb, vb[k]);
                }
            }
            if (e < e1) {
                const int2 pa = pairs[e];
                const uint32_t ba = (static_cast<uint32_t>(pa.x) * B + b0) * (4u * D);
                f32x4 va[G::K];
#pragma unroll
                for (int k = 0; k < G::K; ++k) va[k] = ldblk(ba, tlo[k]);
                const float wa = __int_as_float(pa.y);
#pragma unroll
                for (int k = 0; k < G::K; ++k) pk_fma4(acc[k], wa, va[k]);
            }
        }
#ifdef LG_NM3_STAMPS
        if (tcount < 6) LG_NM3_STAMP(3 + 3 * tcount, __builtin_amdgcn_s_memtime());
#endif
        // next tile's blocks go in flight under this tile's transform (its record landed meanwhile)
        issue(nxt, nn, nb0, nnb);
        __builtin_amdgcn_sched_barrier(0);

        // gather layout -> LDS -> MFMA B operand
        wave_sync_nm();
#pragma unroll
        for (int k = 0; k < G::K; ++k) st4(tl + LY::tix(G::RPI * k + rl, fg), acc[k]);
        wave_sync_nm();
        f32x4 o[G::CH];
#pragma unroll
        for (int mt = 0; mt < G::CH; ++mt) o[mt] = ld4(bl + 16 * mt + 4 * q);
        if constexpr (SPLIT) {
#pragma unroll
            for (int s2 = 0; s2 < D / 32; ++s2) {
                lg_bf16x8 b0f, b1f, b2f;
                split3_x8(ld4(tl + LY::tix(j, 8 * s2 + 2 * q)), ld4(tl + LY::tix(j, 8 * s2 + 2 * q + 1)), b0f, b1f,
                          b2f);
#pragma unroll
                for (int mt = 0; mt < G::CH; ++mt) {
                    const int ew = (16 * mt + j) * SB + 32 * s2 + 8 * q;
                    const lg_bf16x8 a0 = *reinterpret_cast<const lg_bf16x8*>(wsl + ew);
                    const lg_bf16x8 a1 = *reinterpret_cast<const lg_bf16x8*>(wsl + D * SB + ew);
                    const lg_bf16x8 a2 = *reinterpret_cast<const lg_bf16x8*>(wsl + 2 * D * SB + ew);
                    if constexpr (BF) {
                        o[mt] = mfma_bf(a0, b0f, o[mt]);
                        continue;
                    }
                    o[mt] = mfma_bf(a2, b0f, o[mt]);
                    o[mt] = mfma_bf(a1, b1f, o[mt]);
                    o[mt] = mfma_bf(a0, b2f, o[mt]);
                    o[mt] = mfma_bf(a1, b0f, o[mt]);
                    o[mt] = mfma_bf(a0, b1f, o[mt]);
                    o[mt] = mfma_bf(a0, b0f, o[mt]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int c = 0; c < G::CH; ++c) {
                const f32x4 bt = ld4(tl + LY::tix(j, 4 * c + q));
#pragma unroll
                for (int mt = 0; mt < G::CH; ++mt) {
                    const f32x4 wa = ld4(wl + (16 * mt + j) * G::S + 16 * c + 4 * q);
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[mt] = mfma_nm(wa[i], bt[i], o[mt]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#ifdef LG_NM3_STAMPS
        if (tcount < 6) LG_NM3_STAMP(4 + 3 * tcount, __builtin_amdgcn_s_memtime());
#endif
        // epilogue: ReLU, row-stream dropout seeded with the window-major row id (b0 + j) N + n,
        // both as ONE select per element (no fmaxf: its NaN canonicalisation costs a VALU op)
        uint32_t st = 0;
        if constexpr (DROP) st = lg_row_stream_seed(key, static_cast<uint64_t>(b0 + j) * N + n, q);
#pragma unroll
        for (int mt = 0; mt < G::CH; ++mt) {
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const float v = o[mt][reg];
                bool keep = true;
                if constexpr (DROP) {
                    if ((reg & 1) == 0) st = lg_xorshift32(st);
                    const uint32_t u16 = (reg & 1) ? (st >> 16) : (st & 0xFFFFu);
                    keep = u16 >= thr;
                }
                if constexpr (RELU) keep = keep && v > 0.f;
                o[mt][reg] = keep ? v : 0.0f;
            }
        }
        const uint32_t ob = (n * B + b0) * (4u * D);
        wave_sync_nm();
#pragma unroll
        for (int mt = 0; mt < G::CH; ++mt) st4(tl + LY::tix(j, 4 * mt + q), o[mt]);
        wave_sync_nm();
        uint32_t bits = 0;  // [y > 0] of this lane's 4 K elements (bit 4 k + i), for ymask
#pragma unroll
        for (int k = 0; k < G::K; ++k) {
            const f32x4 v = ld4(tl + LY::tix(G::RPI * k + rl, fg));
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                                   yrs, tlo[k] + ob, 0, kLgActAux);
#pragma unroll
            for (int i = 0; i < 4; ++i) bits |= (v[i] > 0.f ? 1u : 0u) << (4 * k + i);
        }
        if (ymask)
            __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(bits), mrs, nm_mask_off(n, b0 >> 4, ngroups, lane),
                                                  0, kLgActAux);
#ifdef LG_NM3_STAMPS
        if (tcount < 6) LG_NM3_STAMP(5 + 3 * tcount, __builtin_amdgcn_s_memtime());
        ++tcount;
#endif
    }
#ifdef LG_NM3_STAMPS
    LG_NM3_STAMP(21, __builtin_amdgcn_s_memtime());
    LG_NM3_STAMP(22, __builtin_amdgcn_s_memrealtime());
    LG_NM3_STAMP(23, (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11))) << 32) |
                         static_cast<uint64_t>(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11))));
#endif
}

// ------------------------------------------------------------------ forward, producer / consumer waves
// The fused layer split by ROLE inside one workgroup per CU.  In nm3/nm5 every wave
// alternates a memory phase (wait for its gathered blocks, accumulate) with a compute phase
// (transpose, split, MFMAs, epilogue).  A per-wave timeline (kernel-lab stamps) showed each
// tile's compute phase as a ~3k-cycle latency chain (LDS round trips, the MFMA chain, VALU
// dependencies) that 2-3 waves per SIMD could not hide, while each wave's loads for the next
// tile were in flight only during it.  Here:
//   * kPcProd PRODUCER waves gather and accumulate (Ahat x) tiles — two tiles' neighbour
//     blocks in flight in registers — and hand each finished tile to a consumer through an
//     LDS ring of R tile slots (16 x D fp32, XOR-swizzled at D = 64);
//   * NC CONSUMER waves per producer (tiles t = c, c + NC, ...) read a slot in the MFMA B
//     layout, run the transform with W's fragments held in registers for the whole launch,
//     bias / ReLU / dropout, write y back through the same slot, store it and free the slot.
// Hand-off: per producer a `ready` tile counter, per consumer a `done` counter, in LDS
// (release stores, acquire polls with s_sleep, workgroup scope); slot t % R is rewritten only
// after its previous tile's consumer counted it done.  Every poll is bounded (a broken
// protocol would end the launch with wrong results instead of a hang).
// Transform: the 3-way bf16 split (bit-identical to k_gcn_fwd_nm3) or, F16, the 2-way fp16
// split with power-of-two scaling (split_bf16.h; 3 MFMAs per product instead of 6).
#ifndef LG_PC_RING
#define LG_PC_RING 4
#endif
// Neighbour blocks per tile in the producers' two-tile prefetch.  A tile with more neighbours
// issues the rest when it is accumulated, and waiting for those youngest loads waits for the
// other buffer's tile too (vmcnt counts in order): at 3, the 32 % of L-TOWN-A's tiles with a
// fourth neighbour (degree 4 with the self loop) exposed a full memory round trip each.  4
// (168 VGPRs, 3 waves per SIMD) leaves that to the 3.5 % of degree 5-6 (r06c, isolated, same
// box: layer 1 21.5-22.8 -> 20.2-21.0 us; in the step 21.1-21.2 -> 20.7-21.0, r06e).  The X0
// layer (2-byte mask words per neighbour) measured best at 4 too: 6 (no rest-of-row path at all)
// took 25.5 us in the step against 24.4-24.8 (r06e), its wider issue costing more than the 3.5 %
// of degree-5/6 tiles' round trip.
#ifndef LG_PC_NPF
#define LG_PC_NPF 4
#endif
#ifndef LG_PC_NPF_X0
#define LG_PC_NPF_X0 4
#endif
constexpr int kPcRing = LG_PC_RING;
// consumer waves per producer wave (4 producers per workgroup)
#ifndef LG_PC_NC
#define LG_PC_NC 2
#endif
constexpr int kPcNC = LG_PC_NC;
// producer waves per workgroup
#ifndef LG_PC_PROD
#define LG_PC_PROD 4
#endif
constexpr int kPcProdN = LG_PC_PROD;
static_assert(kPcProdN <= 16 && kPcProdN * (1 + LG_PC_NC) <= 16, "ready[16]; at most 16 waves");
// The node-table records of a workgroup's first kPcRecs tiles are staged in LDS with W, so a
// producer's record is an LDS read after its tile draw instead of a scalar load from L2 (whose
// latency sat between drawing tile t + 2 and issuing its loads, every tile); later tiles (large
// graphs) read theirs with nm_rec.
#ifndef LG_PC_RECS
#define LG_PC_RECS 256
#endif
constexpr int kPcRecs = LG_PC_RECS;
// 1: the workgroup-wide barrier at the start only covers the hand-off counters; the CONSUMER
// waves stage W (and the bias, the max |W|) among themselves behind an LDS counter, so the
// producers start gathering at once instead of waiting ~1.3 us for W's loads (probe, r05h/i).
// The node-table records then come from scalar loads (nothing else to stage).  0: one barrier
// after W and the records are staged by the whole workgroup.
#ifndef LG_PC_WSPLIT
#define LG_PC_WSPLIT 1
#endif
constexpr bool kPcWsplit = LG_PC_WSPLIT != 0;
// lab: the split W staging on the dense layers too (LG_PC_WS_DENSE), and with it the node-table
// records staged by the producer waves instead of read from L2 per tile (LG_PC_PREC)
#ifndef LG_PC_WS_DENSE
#define LG_PC_WS_DENSE 0
#endif
#ifndef LG_PC_PREC
#define LG_PC_PREC 0
#endif
// lab: tiles dealt to a workgroup's producers statically (p, p + 4, ...) with their records
// by scalar loads a step ahead, instead of an LDS counter and LDS-staged records
#ifndef LG_PC_STATIC
#define LG_PC_STATIC 0
#endif
// producer wave priority (s_setprio; 0: the default, equal to the consumers').  Measured (r05m,
// isolated train mode, two rounds): 2 and 3 within the box's noise of 0 (20.5-21.3 us each)
#ifndef LG_PC_PRIO
#define LG_PC_PRIO 0
#endif
// 1: the producers' prefetch loads are issued through inline asm and waited for with explicit
// vmcnt counts (the other buffer's loads stay in flight).  The compiler's own wait insertion
// lost track of the unrolled pair's two buffers (the loop it builds is irreducible) and waited
// for every load in flight at each tile's accumulate — one tile of prefetch instead of two
// (r05j: 10.7 us for the launch with neither loads nor consumer work, 15.1 with the loads).
// Its waits for loads it does see stay correct: the asm loads are older, and vmcnt counts in
// order.  0: the builtin loads (A/B).
#ifndef LG_PC_EARLY
#define LG_PC_EARLY 1
#endif
#ifndef LG_PC_ASMLOAD
#define LG_PC_ASMLOAD 1
#endif
__device__ __forceinline__ f32x4 pc_load_b128(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
#if LG_PC_ASMLOAD
    f32x4 v;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(v) : "v"(voff), "s"(rs), "s"(soff));
    return v;
#else
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
#endif
}
__device__ __forceinline__ uint32_t pc_load_u16(__amdgpu_buffer_rsrc_t rs, uint32_t voff) {
#if LG_PC_ASMLOAD
    uint32_t v;
    asm volatile("buffer_load_ushort %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(rs));
    return v;
#else
    return __builtin_amdgcn_raw_buffer_load_b16(rs, voff, 0, 0);
#endif
}
// wait until at most N of this wave's vector memory loads are in flight (asm loads only)
template <int N>
__device__ __forceinline__ void pc_vm_wait() {
#if LG_PC_ASMLOAD
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N));
#endif
}
template <typename T>
__device__ __forceinline__ void pc_pin(T& v) {  // v is read only after the waits above it
#if LG_PC_ASMLOAD
    asm volatile("" : "+v"(v));
#else
    (void)v;
#endif
}
// lab: work moved from the consumer waves (the pipeline's bound) to the producers: the tile's
// largest |value| for the f16 scale (LG_PC_PMAX, dense layers; word 10 of the slot metadata) and
// the dropout row-stream seeds (LG_PC_PSEED, one per consumer lane, in LDS beside the slot);
// LG_PC_CPRIO: consumer wave priority (s_setprio)
#ifndef LG_PC_PMAX
#define LG_PC_PMAX 0
#endif
#ifndef LG_PC_PSEED
#define LG_PC_PSEED 0
#endif
#ifndef LG_PC_CPRIO
#define LG_PC_CPRIO 0
#endif
// ring-slot metadata: n, b0, nb, X0's sensor entries (count, then up to kPcSens (slot, w) pairs)
constexpr int kPcSens = 3;
constexpr int kPcMeta = 16;
static_assert(4 + 2 * kPcSens <= kPcMeta, "meta words");

template <int D, int kPcProd, int NC>
struct PcLds {  // floats
    static constexpr bool SWZ = D == 64;
    static constexpr int TILE = SWZ ? 16 * D : NmGeo<D>::TILE;
    static constexpr int WS = D + 4;
    static constexpr int WOFF = 0;                                  // W [out][in] * fold (fp32), bias * fold
    static constexpr int XOFF = D * WS + D;                         // per-wave max|W| bits (F16)
    static constexpr int FOFF = XOFF + 16;                          // ready[16], done[kPcProd * NC], fin[4], ctr
    static constexpr int MOFF = FOFF + 16 + kPcProd * NC + kPcProd + 4;  // per (producer, slot): kPcMeta words
    static constexpr int COFF = MOFF + kPcMeta * kPcProd * kPcRing;  // kPcRecs node-table records (16 words)
    static constexpr int SOFF = COFF + 16 * kPcRecs;                  // LG_PC_PSEED: per (producer, slot) 64 row-stream seeds
    static constexpr int ROFF = SOFF + (LG_PC_PSEED ? 64 * kPcProd * kPcRing : 0);  // the rings
    static constexpr size_t BYTES = 4 * static_cast<size_t>(ROFF + kPcProd * kPcRing * TILE);
    static __device__ __forceinline__ int tix(int r, int c) { return SWZ ? r * D + 4 * (c ^ r) : r * NmGeo<D>::S + 4 * c; }
};
static_assert(kPcRing >= kPcNC, "a ring slot per consumer at least");

__device__ __forceinline__ uint32_t pc_load_acq(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void pc_store_rel(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The hand-off polls are bounded (a broken protocol ends the launch instead of hanging the
// GPU); a poll that runs out sets a bit of g_pc_spin_err (1: a producer's or a W-staging wait,
// 2: a consumer's wait for its tile), which lg_spin_errors reads back -- the launch's results
// are then invalid.  The tests assert it stays 0 (tests/conftest.py, after every GPU module).
__device__ uint32_t g_pc_spin_err;
// lab (LG_PC_DYN): per-XCD tile counters (one 256-byte line each) and the producers' finish
// counter; zero between launches (the launch's last producer resets them)
#ifndef LG_PC_DYN
#define LG_PC_DYN 0
#endif
__device__ uint32_t g_pc_dyn[8 * 64];
__device__ uint32_t g_pc_dyn_fin;
// wait until *p >= v (bounded: ~2^20 polls)
__device__ __forceinline__ void pc_wait(const uint32_t* p, uint32_t v) {
    for (int it = 0; it < (1 << 20); ++it) {
        if (pc_load_acq(p) >= v) return;
        __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_fetch_or(&g_pc_spin_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the atomic must not shift the producers' vmcnt counts
}
// wait until *p >= v (true) or the producer has finished with *fin < v tiles (false); bounded
__device__ __forceinline__ bool pc_wait_or_fin(const uint32_t* p, const uint32_t* fin, uint32_t v) {
    for (int it = 0; it < (1 << 20); ++it) {
        if (pc_load_acq(p) >= v) return true;
        if (pc_load_acq(fin) < v) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_fetch_or(&g_pc_spin_err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return false;
}

// X0: layer 0 reading the compressed node init (lg_node_init_bits_fwd): x = the sensor rows
// [S][B][D], bits = [x0 > 0] of every row, a non-sensor element = bit ? relu(bias) * scale : 0
struct PcX0 {
    const uint16_t* bits;
    const float* bias;
    float scale;
    uint32_t S;
};

template <int D, bool DROP, bool RELU, bool BF, bool F16, int kPcProd, int NC, bool X0 = false>
__global__ void __launch_bounds__(64 * kPcProd * (1 + NC), kPcProd * (1 + NC) / 4)
k_gcn_fwd_pc(const int32_t* __restrict__ tab, const int2* __restrict__ pairs, const float* __restrict__ x,
             const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ y, uint32_t N,
             uint32_t B, uint32_t ngroups, lg_fastdiv fdN, float p_drop, float dscale, uint64_t seed,
             uint32_t salt, uint16_t* __restrict__ ymask, PcX0 x0) {
    using G = NmGeo<D>;
    using LY = PcLds<D, kPcProd, NC>;
    constexpr int NPF = X0 ? LG_PC_NPF_X0 : LG_PC_NPF;
    static_assert(NPF >= 1 && NPF <= kLgNmInline, "prefetch depth");
    constexpr int KS = D / 32;
    constexpr int NP = BF ? 1 : 3;
    constexpr int R = kPcRing;
    constexpr int NT = 64 * kPcProd * (1 + NC);
    static_assert(!(BF && F16), "one transform");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* lds = reinterpret_cast<float*>(smem);
    float* wst = lds + LY::WOFF;
    uint32_t* wmx = reinterpret_cast<uint32_t*>(lds + LY::XOFF);
    uint32_t* ready = reinterpret_cast<uint32_t*>(lds + LY::FOFF);
    uint32_t* done = ready + 16;
    uint32_t* fin = done + kPcProd * NC;  // tiles a producer handed over in all (~0u while it runs)
    uint32_t* ctr = fin + kPcProd;        // the workgroup's next tile (LDS atomic)
    uint32_t* meta = reinterpret_cast<uint32_t*>(lds + LY::MOFF);

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool producer = wave < kPcProd;
#ifdef LG_NM3_STAMPS
    // pc timeline (lab builds): 0 realtime, 1 clock at start, 2 after the W staging barrier,
    // 3 + t: tile t (< 16) handed over (producer) / stored (consumer), 21 clock, 22 realtime at end
    constexpr int WAVES = kPcProd * (1 + NC);
    {
        const int lane = threadIdx.x & 63;
        LG_NM3_STAMP(0, __builtin_amdgcn_s_memrealtime());
        LG_NM3_STAMP(1, __builtin_amdgcn_s_memtime());
    }
#endif
#ifdef LG_PC_PROBE
    const uint64_t probe_rt0 = __builtin_amdgcn_s_memrealtime(), probe_c0 = __builtin_amdgcn_s_memtime();
    auto probe_end = [&](uint64_t c1, uint64_t tiles) {
        const uint64_t c2 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0) {
            uint64_t* o = g_nm3_stamps + (static_cast<size_t>(blockIdx.x) * (kPcProd * (1 + NC)) + wave) * kNm3Stamps;
            o[0] = probe_rt0;
            o[1] = probe_c0;
            o[2] = c1;
            o[3] = tiles;
            o[21] = c2;
            o[22] = rt1;
            o[23] = (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11))) << 32) |
                    static_cast<uint64_t>(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));
        }
    };
#endif
    const int prod = producer ? wave : (wave - kPcProd) % kPcProd;  // the producer this wave is or serves
    const int cons = producer ? 0 : (wave - kPcProd) / kPcProd;     // consumer index 0 .. NC-1
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const int rl = lane / G::LPR, fg = lane % G::LPR;
    float* ring = lds + LY::ROFF + prod * R * LY::TILE;
    const uint64_t bytes = static_cast<uint64_t>(N) * B * (4u * D);
    // Tiles are dealt to WORKGROUPS statically (XCD-aware, nm_sched at one "wave" per workgroup:
    // workgroup-strided tiles of its XCD's chunk) and to the workgroup's producers dynamically
    // through an LDS counter: a producer that draws cheap tiles takes more of them, so the
    // workgroup's tiles finish together (with 4 producers per workgroup the static per-producer
    // split left 1/3 of them a whole tile behind the rest: 10 vs 11 tiles at B = 256).
    const NmSched sc = nm_sched(static_cast<int64_t>(ngroups) * N, 0, 1);
    // tile indices as 32-bit scalars (ntiles < 2^26, lg_gcn_fwd_nm): a 64-bit compare needs a VGPR
    // pair, which the compiler took from a prefetch buffer's registers — and then drained every load
    // in flight at each step's issue (s_waitcnt vmcnt(0)) before it could reuse them
    const int32_t tend = static_cast<int32_t>(sc.end), tfirst = static_cast<int32_t>(sc.first),
                  tstride = static_cast<int32_t>(sc.stride);
    const float fold = DROP ? dscale : 1.0f;  // relu(s z) = s relu(z), s > 0

    auto tile_coords = [&](int32_t tile, uint32_t& n, uint32_t& b0, uint32_t& nb) {
        const bool valid = tile < tend;
        const uint32_t t32 = static_cast<uint32_t>(valid ? tile : 0);
        const uint32_t grp = lg_div(t32, fdN);
        n = t32 - grp * N;
        b0 = grp * 16;
        nb = valid ? min(16u, B - b0) : 0u;
    };

    // W (fp32, x fold) and bias to LDS by the whole workgroup (F16: and the max |W|), and the
    // records of the workgroup's first kPcRecs tiles (every load in flight before the first store)
    int32_t* recs = reinterpret_cast<int32_t*>(lds + LY::COFF);
    // the split W staging pays on layer 0 (X0: -1 us in the step) and costs the dense layers ~1 us
    // (r05w, same box, in-graph: 22.1-22.5 against 21.0-21.1 us: their producers then read every
    // record from L2), so only X0 takes it -- unless the producers stage the records themselves
    // (kPrecs: after the counter barrier, synchronised among the producer waves alone)
    constexpr bool kWs = kPcWsplit && (X0 || LG_PC_WS_DENSE);
    constexpr bool kPrecs = kWs && LG_PC_PREC && kPcRecs > 0;
    // LG_PC_EARLY (dense layers): the producers' first two tiles (draws p and kPcProd + p, the
    // counter starting past them) are issued before the prologue barrier, from records read
    // through the scalar cache, while the consumer waves alone stage W, the bias and the records:
    // the kernel's first gathers overlap the W staging instead of following it
    constexpr bool kEarly = LG_PC_EARLY && !kWs && !LG_PC_STATIC && !LG_PC_DYN;
    const int nrec = ((kWs && !kPrecs) || LG_PC_STATIC || LG_PC_DYN) ? 0 : min(kPcRecs, tend > tfirst ? (tend - tfirst + tstride - 1) / tstride : 0);
    uint32_t* wrdy = ctr + 1;  // kWs: consumer waves done staging W
    uint32_t* prdy = ctr + 2;  // kPrecs: producer waves done staging the records
    if constexpr (kWs) {
        if (threadIdx.x < 16 + kPcProd * NC) ready[threadIdx.x] = 0u;  // ready[] and done[]
        if (threadIdx.x < kPcProd) fin[threadIdx.x] = ~0u;
        if (threadIdx.x == 0) {
            *ctr = 0u;
            *wrdy = 0u;
            *prdy = 0u;
        }
    } else {
        // the staging threads: all of the workgroup, or (kEarly) its consumer waves
        constexpr int SNT = kEarly ? NT - 64 * kPcProd : NT;
        const int st = static_cast<int>(threadIdx.x) - (kEarly ? 64 * kPcProd : 0);
        if (!kEarly || !producer) {
            constexpr int W4 = D * D / 4, WPER = (W4 + SNT - 1) / SNT, RPER = kPcRecs ? (4 * kPcRecs + SNT - 1) / SNT : 1;
            f32x4 wv[WPER];
#pragma unroll
            for (int u = 0; u < WPER; ++u) wv[u] = ld4(W + 4 * min<int>(u * SNT + st, W4 - 1));
            lg_u32x4 rv[RPER];
#pragma unroll
            for (int u = 0; u < RPER; ++u) {  // quarter (i & 3) of record i >> 2
                const int i = u * SNT + st;
                uint32_t n, b0, nb;
                tile_coords(i < 4 * nrec ? tfirst + (i >> 2) * tstride : tend, n, b0, nb);
                rv[u] = reinterpret_cast<const lg_u32x4*>(tab)[4 * (static_cast<size_t>(N) + n) + (i & 3)];
            }
            const float bb = (bias && st < D) ? bias[st] : 0.f;
            uint32_t wm = 0;
#pragma unroll
            for (int u = 0; u < WPER; ++u) {
                const int i = u * SNT + st;
                f32x4 w = wv[u] * fold;
                asm volatile("" : "+v"(w));  // rounded before any split (no contraction)
                if (i < W4) {
                    st4(wst + (i / (D / 4)) * LY::WS + 4 * (i % (D / 4)), w);
#pragma unroll
                    for (int c = 0; c < 4; ++c) wm = max(wm, __float_as_uint(fabsf(w[c])));
                }
            }
#pragma unroll
            for (int u = 0; u < RPER; ++u) {
                const int i = u * SNT + st;
                if (i < 4 * nrec) reinterpret_cast<lg_u32x4*>(recs)[i] = rv[u];
            }
            if (st < D) wst[D * LY::WS + st] = bb * fold;
            if constexpr (F16) {
                wm = lg_wave_max_bits(wm);
                if (lane == 0) wmx[wave] = wm;
            }
        }
        if (threadIdx.x < 16 + kPcProd * NC) ready[threadIdx.x] = 0u;  // ready[] and done[]
        if (threadIdx.x < kPcProd) fin[threadIdx.x] = ~0u;
        if (threadIdx.x == 0) *ctr = kEarly ? 2u * kPcProd : 0u;
    }
    if (!kEarly || !producer) __syncthreads();  // kEarly: the producers arrive after their first issues
    if (kPrecs && producer) {  // the producers' record staging (the workgroup's first nrec tiles)
        constexpr int PT = 64 * kPcProd, RP = (4 * kPcRecs + PT - 1) / PT;
        lg_u32x4 rv[RP];
#pragma unroll
        for (int u = 0; u < RP; ++u) {  // quarter (i & 3) of record i >> 2
            const int i = u * PT + static_cast<int>(threadIdx.x);
            if (i < 4 * nrec) {
                uint32_t n, b0, nb;
                tile_coords(tfirst + (i >> 2) * tstride, n, b0, nb);
                rv[u] = reinterpret_cast<const lg_u32x4*>(tab)[4 * (static_cast<size_t>(N) + n) + (i & 3)];
            }
        }
#pragma unroll
        for (int u = 0; u < RP; ++u) {
            const int i = u * PT + static_cast<int>(threadIdx.x);
            if (i < 4 * nrec) reinterpret_cast<lg_u32x4*>(recs)[i] = rv[u];
        }
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(prdy, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        pc_wait(prdy, static_cast<uint32_t>(kPcProd));
    }
    if (kWs && !producer) {  // the consumers' W staging (all loads in flight before the first store)
        constexpr int CT = 64 * kPcProd * NC, W4 = D * D / 4, WPER = (W4 + CT - 1) / CT;
        const int ct = static_cast<int>(threadIdx.x) - 64 * kPcProd;
        f32x4 wv[WPER];
#pragma unroll
        for (int u = 0; u < WPER; ++u) wv[u] = ld4(W + 4 * min<int>(u * CT + ct, W4 - 1));
        const float bb = (bias && ct < D) ? bias[ct] : 0.f;
        uint32_t wm = 0;
#pragma unroll
        for (int u = 0; u < WPER; ++u) {
            const int i = u * CT + ct;
            f32x4 w = wv[u] * fold;
            asm volatile("" : "+v"(w));  // rounded before any split (no contraction)
            if (i < W4) {
                st4(wst + (i / (D / 4)) * LY::WS + 4 * (i % (D / 4)), w);
#pragma unroll
                for (int c = 0; c < 4; ++c) wm = max(wm, __float_as_uint(fabsf(w[c])));
            }
        }
        if (ct < D) wst[D * LY::WS + ct] = bb * fold;
        if constexpr (F16) {
            wm = lg_wave_max_bits(wm);
            if (lane == 0) wmx[wave] = wm;
        }
        if (lane == 0) __hip_atomic_fetch_add(wrdy, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        pc_wait(wrdy, static_cast<uint32_t>(kPcProd * NC));
    }
#ifdef LG_PC_PROBE
    const uint64_t probe_c1 = __builtin_amdgcn_s_memtime();
#endif
#ifdef LG_NM3_STAMPS
    LG_NM3_STAMP(2, __builtin_amdgcn_s_memtime());
    auto pc_stamp_end = [&]() {
        LG_NM3_STAMP(21, __builtin_amdgcn_s_memtime());
        LG_NM3_STAMP(22, __builtin_amdgcn_s_memrealtime());
        LG_NM3_STAMP(23, (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11))) << 32) |
                             static_cast<uint64_t>(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11))));
    };
#endif

    if (producer) {
        // ---------------- producer: gather + accumulate, two tiles in flight
        const uint32_t pkey = LG_PC_PSEED && DROP ? lg_dropout_key_dev(seed, salt) : 0u;
#if LG_PC_PRIO
        // the producer's instruction stream is the pipeline's critical path; its two consumers on
        // the same SIMD have ring slack, so the producer goes first when both are ready to issue
        __builtin_amdgcn_s_setprio(LG_PC_PRIO);
#endif
        // X0 (layer 0 on the compressed node init): a neighbour whose record col carries
        // kLgSensorCol is a sensor row of x (= xs0 [S][B][D]) at its slot; any other
        // neighbour's block is its [x0 > 0] mask word (one uint16 per lane), x0 = bit ? v0 : 0
        const __amdgpu_buffer_rsrc_t xrs = nm_rsrc(x, X0 ? static_cast<uint64_t>(x0.S) * B * (4u * D) : bytes),
                                     xrs0 = nm_rsrc(x, 0);
        const __amdgpu_buffer_rsrc_t brs = nm_mask_rsrc(x0.bits, N, ngroups);
        f32x4 v0 = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (X0) {
            const f32x4 bv = ld4(x0.bias + 4 * fg);
#pragma unroll
            for (int i = 0; i < 4; ++i) v0[i] = fmaxf(bv[i], 0.f) * x0.scale;
        }
        uint32_t loff[G::K];
#pragma unroll
        for (int k = 0; k < G::K; ++k) loff[k] = (G::RPI * k + rl) * (4u * D) + 16u * fg;
        f32x4 pf[2][NPF][G::K];
        uint32_t pb[2][X0 ? NPF : 1];  // X0: the neighbours' mask words
        uint32_t lo[2][G::K];
        NmRec rec[2];
        uint32_t tn[2], tb0[2], tnb[2];
        // one neighbour's block: its rows into blk or, X0, its mask word into bw (an absent
        // neighbour, have == false, and X0's sensor neighbours read out of range: zero bits).
        // X0's sensor rows are added by the consumer (ring-slot metadata), so the producer issues
        // one 2-byte load per neighbour instead of the rows.
        auto load_nb = [&](int c, bool have, uint32_t b0, const uint32_t (&lk)[G::K], f32x4 (&blk)[G::K], uint32_t& bw) {
#ifdef LG_PC_LAB_NOLOAD  // lab: no gather loads (the neighbour blocks read as lane-dependent constants)
            bw = lane;
#pragma unroll
            for (int k = 0; k < G::K; ++k) blk[k] = f32x4{1.f * k, 1.f * lane, 0.5f, 0.25f};
            return;
#endif
            if constexpr (X0) {
                const bool sens = (c & kLgSensorCol) != 0;
                bw = pc_load_u16(brs, have && !sens ? nm_mask_off(static_cast<uint32_t>(c), b0 >> 4, ngroups, lane)
                                                    : kNm3BlkOob + 2u * lane);
                return;
            }
            const bool rows = have;
            const uint32_t base = rows ? (static_cast<uint32_t>(c) * B + b0) * (4u * D) : 0u;
            const __amdgpu_buffer_rsrc_t rs = rows ? xrs : xrs0;
#pragma unroll
            for (int k = 0; k < G::K; ++k) blk[k] = pc_load_b128(rs, lk[k], base);
        };
        // the rest-of-row blocks (loaded and consumed within one tile): the compiler's loads
        auto load_rest = [&](int c, bool have, uint32_t b0, const uint32_t (&lk)[G::K], f32x4 (&blk)[G::K], uint32_t& bw) {
            if constexpr (X0) {
                const bool sens = (c & kLgSensorCol) != 0;
                bw = __builtin_amdgcn_raw_buffer_load_b16(
                    brs, have && !sens ? nm_mask_off(static_cast<uint32_t>(c), b0 >> 4, ngroups, lane) : kNm3BlkOob + 2u * lane,
                    0, 0);
                return;
            }
            const uint32_t base = have ? (static_cast<uint32_t>(c) * B + b0) * (4u * D) : 0u;
            const __amdgpu_buffer_rsrc_t rs = have ? xrs : xrs0;
#pragma unroll
            for (int k = 0; k < G::K; ++k)
                blk[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lk[k], base, 0));
        };
        constexpr int LPT = X0 ? NPF : NPF * G::K;  // prefetch loads per tile
        // slot k of a loaded neighbour block as values.  X0: from the mask word (zero for a
        // sensor neighbour), branch-free (a branch on the neighbour kind here made the compiler
        // read the rest-of-row mask words before their loads had landed: wrong bits for slots
        // k >= 1 of degree-5 nodes, r04f)
        auto nbv = [&](int c, const f32x4 (&blk)[G::K], uint32_t bw, int k) -> f32x4 {
            (void)c;
            if constexpr (X0) {
                const uint32_t w = bw >> (4 * k);
                f32x4 r;
#pragma unroll
                for (int i = 0; i < 4; ++i) r[i] = (w >> i) & 1u ? v0[i] : 0.f;
                return r;
            }
            return blk[k];
        };
        // the workgroup's next tile (an LDS atomic; past tend once its tiles are all dealt) and
        // its record (staged in LDS for the first kPcRecs draws)
        uint32_t gcount = 0;  // LG_PC_STATIC: this producer's draws so far
        auto grab = [&](NmRec& r) -> int32_t {
#if LG_PC_DYN
            // dynamic dealing over the XCD's tile range: a global counter per XCD, one atomic per
            // draw, requested a whole step before the tile's loads issue
            uint32_t di = 0;
            if (lane == 0)
                di = __hip_atomic_fetch_add(&g_pc_dyn[64 * (blockIdx.x % 8)], 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
            di = __builtin_amdgcn_readfirstlane(di);
            const int32_t dchunk = static_cast<int32_t>((static_cast<int64_t>(ngroups) * N + 7) / 8);
            const int32_t tile = gridDim.x >= 8 ? static_cast<int32_t>(blockIdx.x % 8) * dchunk + static_cast<int32_t>(di)
                                                : tend;
            {
                uint32_t n, b0, nb;
                tile_coords(tile, n, b0, nb);
                r = nm_rec(tab, N + n);
            }
            return tile;
#elif LG_PC_STATIC
            // static dealing: draw i of producer p is the workgroup's tile p + 4 i; its record by
            // scalar loads, requested a whole step before the tile's loads issue
            const int32_t tile = tfirst + static_cast<int32_t>(gcount * kPcProd + prod) * tstride;
            ++gcount;
            {
                uint32_t n, b0, nb;
                tile_coords(tile, n, b0, nb);
                r = nm_rec(tab, N + n);
            }
            return tile;
#else
            uint32_t i = 0;
            if (lane == 0) i = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            i = __builtin_amdgcn_readfirstlane(i);
            const int32_t tile = tfirst + static_cast<int32_t>(i) * tstride;
            if (static_cast<int>(i) < nrec) {
                const int4* rp = reinterpret_cast<const int4*>(recs) + 4 * i;
                const int4 a = rp[0], b = rp[1], c = rp[2], d = rp[3];
                auto u = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
                r.e0 = u(a.x);
                r.e1 = u(a.y);
                r.p[0] = int2{u(a.z), u(a.w)};
                r.p[1] = int2{u(b.x), u(b.y)};
                r.p[2] = int2{u(b.z), u(b.w)};
                r.p[3] = int2{u(c.x), u(c.y)};
                r.p[4] = int2{u(c.z), u(c.w)};
                r.p[5] = int2{u(d.x), u(d.y)};
                r.self = u(d.z);
                r.node = u(d.w);
            } else {
                uint32_t n, b0, nb;
                tile_coords(tile, n, b0, nb);
                r = nm_rec(tab, N + n);
            }
            return tile;
#endif
        };
        int32_t tl[2];  // the tile whose blocks are in flight in buffer b
        // r: the tile's node-table record (schedule section: slot -> record with its node id),
        // requested by the caller a phase earlier
        auto issue = [&](auto bc, const NmRec& r, int32_t tile) {
            constexpr int b = decltype(bc)::value;
            uint32_t n, b0, nb;
            tile_coords(tile, n, b0, nb);
            tl[b] = tile;
            rec[b] = r;
            n = static_cast<uint32_t>(r.node);
            tn[b] = n;
            tb0[b] = b0;
            tnb[b] = nb;
#pragma unroll
            for (int k = 0; k < G::K; ++k) lo[b][k] = (G::RPI * k + rl) < static_cast<int>(nb) ? loff[k] : kNm3RowOob;
#pragma unroll
            for (int i = 0; i < NPF; ++i) load_nb(r.p[i].x, r.e0 + i < r.e1, b0, lo[b], pf[b][i], pb[b][X0 ? i : 0]);
        };
        // tile t of this producer from buffer b: accumulate, hand over, refill b with tile t + 2
        auto step = [&](auto bc, int64_t t) -> bool {
            constexpr int b = decltype(bc)::value;
            const int32_t tile = tl[b];
            if (tile >= tend) return false;
            // the producer's tile t + 2 is drawn (its record from LDS, or in flight while this tile
            // is accumulated)
            NmRec nxt;
            const int32_t tnext = grab(nxt);
            asm volatile("" ::: "memory");  // keep the request here (the compiler sinks it to its use)
            const NmRec& cur = rec[b];
            const int e0 = cur.e0, e1 = cur.e1;
            const uint32_t b0 = tb0[b];
            // this buffer's loads are the older half of those in flight (the other buffer's tile
            // was issued after them)
            pc_vm_wait<LPT>();
#pragma unroll
            for (int i = 0; i < NPF; ++i) {
                if constexpr (X0) pc_pin(pb[b][i]);
                else
#pragma unroll
                    for (int k = 0; k < G::K; ++k) pc_pin(pf[b][i][k]);
            }
            f32x4 acc[G::K];
            {
                const float w = e0 < e1 ? __int_as_float(cur.p[0].y) : 0.f;
                const int c = e0 < e1 ? cur.p[0].x : kLgSensorCol;  // absent: the zero rows, weight 0
#pragma unroll
                for (int k = 0; k < G::K; ++k) acc[k] = nbv(c, pf[b][0], pb[b][0], k) * w;
            }
#pragma unroll
            for (int i = 1; i < NPF; ++i) {
                if (e0 + i < e1) {
                    const float w = __int_as_float(cur.p[i].y);
#pragma unroll
                    for (int k = 0; k < G::K; ++k) pk_fma4(acc[k], w, nbv(cur.p[i].x, pf[b][i], pb[b][X0 ? i : 0], k));
                }
            }
            if (e0 + NPF < e1) {  // the rest of the row (degree > NPF): all inline blocks in flight at once
                if constexpr (NPF < kLgNmInline) {
                    constexpr int NI = kLgNmInline - NPF;
                    f32x4 va[NI][G::K];
                    uint32_t vb[NI];
#pragma unroll
                    for (int i = 0; i < NI; ++i) load_rest(cur.p[NPF + i].x, e0 + NPF + i < e1, b0, lo[b], va[i], vb[i]);
#pragma unroll
                    for (int i = 0; i < NI; ++i) {  // an absent entry: zero blocks at weight 0 (acc unchanged)
                        const float wa = e0 + NPF + i < e1 ? __int_as_float(cur.p[NPF + i].y) : 0.f;
#pragma unroll
                        for (int k = 0; k < G::K; ++k) pk_fma4(acc[k], wa, nbv(cur.p[NPF + i].x, va[i], vb[i], k));
                    }
                }
                for (int e = e0 + kLgNmInline; e < e1; ++e) {
                    const int2 pa = pairs[e];
                    f32x4 vr[G::K];
                    uint32_t vw;
                    load_rest(pa.x, true, b0, lo[b], vr, vw);
                    const float wa = __int_as_float(pa.y);
#pragma unroll
                    for (int k = 0; k < G::K; ++k) pk_fma4(acc[k], wa, nbv(pa.x, vr, vw, k));
                }
            }
            // X0: the row's sensor entries (the consumer adds their rows): up to kPcSens in the
            // slot metadata, more (a node with over kPcSens sensor neighbours) flagged for a scan
            uint32_t nsx = 0, ss0 = 0, ss1 = 0, ss2 = 0, sw0 = 0, sw1 = 0, sw2 = 0;
            if constexpr (X0) {
                auto addsens = [&](int2 pe) {
                    if (!(pe.x & kLgSensorCol)) return;
                    const uint32_t sv = static_cast<uint32_t>(pe.x & ~kLgSensorCol), wv = static_cast<uint32_t>(pe.y);
                    if (nsx == 0) { ss0 = sv; sw0 = wv; }
                    if (nsx == 1) { ss1 = sv; sw1 = wv; }
                    if (nsx == 2) { ss2 = sv; sw2 = wv; }
                    ++nsx;
                };
#pragma unroll
                for (int i = 0; i < kLgNmInline; ++i)
                    if (e0 + i < e1) addsens(cur.p[i]);
                for (int e = e0 + kLgNmInline; e < e1; ++e) addsens(pairs[e]);
            }
            const int sl = static_cast<int>(t % R);
            const uint32_t mn = tn[b], mnb = tnb[b];
            // buffer b is free again: tile t + 2 goes in flight before the hand-off waits
            issue(bc, nxt, tnext);
            // slot sl last held tile t - R, consumed by consumer (t - R) % NC as its ((t - R) / NC)-th
            if (t >= R) pc_wait(&done[prod * NC + static_cast<int>((t - R) % NC)], static_cast<uint32_t>((t - R) / NC + 1));
            float* slot = ring + sl * LY::TILE;
#pragma unroll
            for (int k = 0; k < G::K; ++k) st4(slot + LY::tix(G::RPI * k + rl, fg), acc[k]);
            uint32_t pmx = 0;
            if constexpr (LG_PC_PMAX && F16 && !X0) {  // the tile's largest |value| (the consumer's f16 scale)
                float mf = 0.f;
#pragma unroll
                for (int k = 0; k < G::K; ++k)
#pragma unroll
                    for (int c = 0; c < 4; ++c) mf = fmaxf(mf, fabsf(acc[k][c]));
                pmx = lg_wave_max_bits(__float_as_uint(mf));
            }
            if constexpr (LG_PC_PSEED && DROP) {  // the consumer lane (j, q)'s row-stream seed
                uint32_t* sd = reinterpret_cast<uint32_t*>(lds + LY::SOFF) + 64 * (prod * R + sl);
                sd[lane] = lg_row_stream_seed(pkey, static_cast<uint64_t>(b0 + j) * N + mn, static_cast<uint32_t>(q));
            }
            if (lane == 0) {
                uint32_t* m = meta + kPcMeta * (prod * R + sl);
                m[0] = mn;
                m[1] = b0;
                m[2] = mnb;
                if constexpr (LG_PC_PMAX && F16 && !X0) m[10] = pmx;
                if constexpr (X0) {
                    m[3] = nsx;
                    m[4] = ss0;
                    m[5] = sw0;
                    m[6] = ss1;
                    m[7] = sw1;
                    m[8] = ss2;
                    m[9] = sw2;
                }
            }
            pc_store_rel(&ready[prod], static_cast<uint32_t>(t + 1));
#ifdef LG_NM3_STAMPS
            if (t < 16) LG_NM3_STAMP(3 + t, __builtin_amdgcn_s_memtime());
#endif
            return true;
        };
        {
            NmRec r0, r1;
            int32_t f0, f1;
            if constexpr (kEarly) {  // draws prod and kPcProd + prod, records through the scalar cache
                auto early = [&](int i, NmRec& r) {
                    const int32_t tile = tfirst + i * tstride;
                    uint32_t n, b0, nb;
                    tile_coords(tile, n, b0, nb);
                    r = nm_rec(tab, N + n);
                    return tile;
                };
                f0 = early(prod, r0);
                f1 = early(kPcProd + prod, r1);
            } else {
                f0 = grab(r0);
                f1 = grab(r1);
            }
            issue(std::integral_constant<int, 0>{}, r0, f0);
            issue(std::integral_constant<int, 1>{}, r1, f1);
        }
        if constexpr (kEarly) __syncthreads();  // the prologue barrier (W, bias, records, counter)
        int64_t t = 0;
        for (;; t += 2) {
            if (!step(std::integral_constant<int, 0>{}, t)) break;
            if (!step(std::integral_constant<int, 1>{}, t + 1)) {
                ++t;
                break;
            }
        }
        // tiles are drawn in increasing order, so the first one past tend ends the producer
        pc_vm_wait<0>();  // the last (empty) prefetches
        if (lane == 0) pc_store_rel(&fin[prod], static_cast<uint32_t>(t));
#if LG_PC_DYN
        if (lane == 0) {  // the launch's last producer: the counters back to 0 for the next launch
            const uint32_t f = __hip_atomic_fetch_add(&g_pc_dyn_fin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (f + 1 == gridDim.x * kPcProd) {
                for (int x = 0; x < 8; ++x) __hip_atomic_store(&g_pc_dyn[64 * x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&g_pc_dyn_fin, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#endif
#ifdef LG_NM3_STAMPS
        pc_stamp_end();
#endif
#ifdef LG_PC_PROBE
        probe_end(probe_c1, static_cast<uint64_t>(t));
#endif
        return;
    }

    // ---------------- consumer: transform + epilogue
#if LG_PC_CPRIO
    __builtin_amdgcn_s_setprio(LG_PC_CPRIO);
#endif
    const __amdgpu_buffer_rsrc_t yrs = nm_rsrc(y, bytes);
    const __amdgpu_buffer_rsrc_t srs = nm_rsrc(x, X0 ? static_cast<uint64_t>(x0.S) * B * (4u * D) : 0);  // X0: xs0
    const __amdgpu_buffer_rsrc_t mrs = nm_mask_rsrc(ymask, N, ngroups);
    uint32_t loff[G::K];
#pragma unroll
    for (int k = 0; k < G::K; ++k) loff[k] = (G::RPI * k + rl) * (4u * D) + 16u * fg;
    int sw = 0;  // F16: W's scale exponent
    if constexpr (F16) {
        uint32_t m = 0;
        for (int w = (kWs || kEarly) ? kPcProd : 0; w < kPcProd * (1 + NC); ++w) m = max(m, wmx[w]);
        sw = lg_f16_scale_exp(__builtin_amdgcn_readfirstlane(m));
    }
    lg_bf16x8 wf[NP][G::CH][KS];
    lg_f16x8 wh[2][G::CH][KS];
#pragma unroll
    for (int mt = 0; mt < G::CH; ++mt) {
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const float* wp = wst + (16 * mt + j) * LY::WS + 32 * s2 + 8 * q;
            const f32x4 wa = ld4(wp), wb = ld4(wp + 4);
            if constexpr (F16) {
                const float sc2 = lg_pow2f(sw);
                split2_f16_x8(wa * sc2, wb * sc2, wh[0][mt][s2], wh[F16 ? 1 : 0][mt][s2]);
                continue;
            }
            lg_bf16x8 f0, f1, f2;
            split3_x8(wa, wb, f0, f1, f2);
            wf[0][mt][s2] = f0;
            if constexpr (!BF) {
                wf[NP > 1 ? 1 : 0][mt][s2] = f1;
                wf[NP > 2 ? 2 : 0][mt][s2] = f2;
            }
        }
    }
    const uint32_t key = lg_dropout_key_dev(seed, salt);
    const uint32_t thr = lg_keep_threshold16(p_drop);
    int64_t u = 0;
    for (;; ++u) {
        const int64_t t = u * NC + cons;  // this consumer's u-th tile of its producer
        // wait for tile t, or for the producer's end (it handed over fin[prod] tiles in all)
        if (!pc_wait_or_fin(&ready[prod], &fin[prod], static_cast<uint32_t>(t + 1))) break;
        const int sl = static_cast<int>(t % R);
        float* slot = ring + sl * LY::TILE;
        const uint32_t* m = meta + kPcMeta * (prod * R + sl);
        const uint32_t n = __builtin_amdgcn_readfirstlane(m[0]), b0 = __builtin_amdgcn_readfirstlane(m[1]),
                       nb = __builtin_amdgcn_readfirstlane(m[2]);
#ifdef LG_PC_LAB_NOCONS  // lab: consumers hand the slot straight back
        pc_store_rel(&done[prod * NC + cons], static_cast<uint32_t>(u + 1));
        continue;
#endif
        f32x4 bq[KS][2];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            bq[s2][0] = ld4(slot + LY::tix(j, 8 * s2 + 2 * q));
            bq[s2][1] = ld4(slot + LY::tix(j, 8 * s2 + 2 * q + 1));
        }
        if constexpr (X0) {  // the tile's sensor neighbours: w x (their xs0 rows), in entry order
            const uint32_t ns = __builtin_amdgcn_readfirstlane(m[3]);
            auto addrow = [&](uint32_t sv, float wv) {
#pragma unroll
                for (int s2 = 0; s2 < KS; ++s2)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const uint32_t off = static_cast<uint32_t>(j) < nb
                                                 ? ((sv * B + b0 + j) * D + 4 * (8 * s2 + 2 * q + h)) * 4u
                                                 : kNm3RowOob;
                        pk_fma4(bq[s2][h], wv,
                                __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(srs, off, 0, 0)));
                    }
            };
            if (ns > static_cast<uint32_t>(kPcSens)) {  // rare: scan the node's row (node-order section)
                const NmRec r = nm_rec(tab, n);
                for (int i = 0; i < kLgNmInline; ++i)
                    if (r.e0 + i < r.e1 && (r.p[i].x & kLgSensorCol))
                        addrow(static_cast<uint32_t>(r.p[i].x & ~kLgSensorCol), __int_as_float(r.p[i].y));
                for (int e = r.e0 + kLgNmInline; e < r.e1; ++e) {
                    const int2 pe = pairs[e];
                    if (pe.x & kLgSensorCol) addrow(static_cast<uint32_t>(pe.x & ~kLgSensorCol), __int_as_float(pe.y));
                }
            } else {
                for (uint32_t i = 0; i < ns; ++i)
                    addrow(__builtin_amdgcn_readfirstlane(m[4 + 2 * i]), __uint_as_float(__builtin_amdgcn_readfirstlane(m[5 + 2 * i])));
            }
        }
        uint32_t st = 0;
        if constexpr (DROP) {
            if constexpr (LG_PC_PSEED) st = reinterpret_cast<const uint32_t*>(lds + LY::SOFF)[64 * (prod * R + sl) + lane];
            else st = lg_row_stream_seed(key, static_cast<uint64_t>(b0 + j) * N + n, q);
        }
        f32x4 o[G::CH];
#ifdef LG_PC_LAB_NOMFMA  // lab: no transform (the tile's values stand in for the product)
#pragma unroll
        for (int mt = 0; mt < G::CH; ++mt) o[mt] = bq[mt % KS][mt / KS % 2];
        if constexpr (false) {
#else
        if constexpr (F16) {
#endif
            // the tile's scale from its largest |value| (the B-operand values are the whole tile;
            // fmaxf on |.| source modifiers: three values an instruction)
            int sa;
            if constexpr (LG_PC_PMAX && !X0) {
                sa = lg_f16_scale_exp(__builtin_amdgcn_readfirstlane(m[10]));
            } else {
                float mxf = 0.f;
#pragma unroll
                for (int s2 = 0; s2 < KS; ++s2)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int c = 0; c < 4; ++c) mxf = fmaxf(mxf, fabsf(bq[s2][h][c]));
                sa = lg_f16_scale_exp(lg_wave_max_bits(__float_as_uint(mxf)));
            }
            const float sc2 = lg_pow2f(sa);
#pragma unroll
            for (int mt = 0; mt < G::CH; ++mt) o[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                lg_f16x8 b0h, b1h;
                split2_f16_x8(bq[s2][0] * sc2, bq[s2][1] * sc2, b0h, b1h);
#pragma unroll
                for (int mt = 0; mt < G::CH; ++mt) {  // smallest terms first
                    o[mt] = mfma_h(wh[F16 ? 1 : 0][mt][s2], b0h, o[mt]);
                    o[mt] = mfma_h(wh[0][mt][s2], b1h, o[mt]);
                    o[mt] = mfma_h(wh[0][mt][s2], b0h, o[mt]);
                }
            }
            const float us = lg_pow2f(-(sa + sw));  // unscale (exact) and the bias in one rounding
#pragma unroll
            for (int mt = 0; mt < G::CH; ++mt) {
                const f32x4 bv = ld4(wst + D * LY::WS + 16 * mt + 4 * q);  // bias * fold
#pragma unroll
                for (int c = 0; c < 4; ++c) o[mt][c] = fmaf(o[mt][c], us, bv[c]);
            }
        } else {
#pragma unroll
            for (int mt = 0; mt < G::CH; ++mt) o[mt] = ld4(wst + D * LY::WS + 16 * mt + 4 * q);  // bias * fold
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                lg_bf16x8 b0f, b1f, b2f;
                split3_x8(bq[s2][0], bq[s2][1], b0f, b1f, b2f);
#pragma unroll
                for (int mt = 0; mt < G::CH; ++mt) {
                    if constexpr (BF) {
                        o[mt] = mfma_bf(wf[0][mt][s2], b0f, o[mt]);
                        continue;
                    }
                    o[mt] = mfma_bf(wf[NP > 2 ? 2 : 0][mt][s2], b0f, o[mt]);
                    o[mt] = mfma_bf(wf[NP > 1 ? 1 : 0][mt][s2], b1f, o[mt]);
                    o[mt] = mfma_bf(wf[0][mt][s2], b2f, o[mt]);
                    o[mt] = mfma_bf(wf[NP > 1 ? 1 : 0][mt][s2], b0f, o[mt]);
                    o[mt] = mfma_bf(wf[0][mt][s2], b1f, o[mt]);
                    o[mt] = mfma_bf(wf[0][mt][s2], b0f, o[mt]);
                }
            }
        }
#ifndef LG_PC_LAB_NOEPI  // lab: no ReLU / dropout
#pragma unroll
        for (int mt = 0; mt < G::CH; ++mt) {
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                float v = o[mt][reg];
                if constexpr (RELU) v = __int_as_float(max(__float_as_int(v), 0));
                if constexpr (DROP) {
                    if ((reg & 1) == 0) st = lg_xorshift32(st);
                    const uint32_t u16 = (reg & 1) ? (st >> 16) : (st & 0xFFFFu);
                    v = u16 >= thr ? v : 0.0f;
                }
                o[mt][reg] = v;
            }
        }
#endif
        // y back through the slot (the B-operand reads above are older LDS operations of
        // this wave, so they complete first)
#pragma unroll
        for (int mt = 0; mt < G::CH; ++mt) st4(slot + LY::tix(j, 4 * mt + q), o[mt]);
        const uint32_t ob = (n * B + b0) * (4u * D);
        f32x4 vk[G::K];
#pragma unroll
        for (int k = 0; k < G::K; ++k) {
            const uint32_t lk = (G::RPI * k + rl) < static_cast<int>(nb) ? loff[k] : kNm3RowOob;
            vk[k] = ld4(slot + LY::tix(G::RPI * k + rl, fg));
#if !defined(LG_PC_LAB_NOSTORE) && !defined(LG_PC_LAB_NOYSTORE)  // lab: no y stores (NOSTORE: nor mask words)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, vk[k]),
                                                   yrs, lk, ob, kLgActAux);
#endif
        }
#if defined(LG_PC_LAB_NOSTORE) || defined(LG_PC_LAB_NOMASK)
        if (false) {
#else
        if (ymask) {
#endif
            uint32_t bits = 0;
#pragma unroll
            for (int k = G::K - 1; k >= 0; --k)
#pragma unroll
                for (int i = 3; i >= 0; --i) {
                    const uint32_t uu = RELU ? __float_as_uint(vk[k][i])
                                             : static_cast<uint32_t>(max(__float_as_int(vk[k][i]), 0));
                    bits = __builtin_amdgcn_alignbit(bits, uu + 0x7FFFFFFFu, 31);
                }
            __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(bits), mrs, nm_mask_off(n, b0 >> 4, ngroups, lane),
                                                  0, kLgActAux);
        }
        lg_store_guard(vk);
        pc_store_rel(&done[prod * NC + cons], static_cast<uint32_t>(u + 1));  // the slot's reads are done (release)
#ifdef LG_NM3_STAMPS
        if (u < 16) LG_NM3_STAMP(3 + u, __builtin_amdgcn_s_memtime());
#endif
    }
#ifdef LG_NM3_STAMPS
    pc_stamp_end();
#endif
#ifdef LG_PC_PROBE
    probe_end(probe_c1, static_cast<uint64_t>(u));
#endif
}

// ------------------------------------------------------------------ backward, node-table pipeline
// lg_gcn_bwd_nm on k_gcn_fwd_nm3's pipeline: the tile's CSR record (transposed CSR) is one
// scalar load issued a tile ahead; the tile's NPF first neighbour dz blocks (MASK_IN: and
// their y blocks for the [y > 0] mask) and its own x block are in flight under the previous
// tile's MFMA work; the row's self entry (the node table's `self`) supplies the tile's own
// dz rows for db, so the own dy / y blocks are not read twice.  Both GEMMs run on bf16
// MFMA with 3-way split operands (split_bf16.h, fp32-level accuracy):
//   dx^T = W^T t^T   (16x16x32, W^T split once per workgroup in LDS)
//   dW  += t^T x     (16x16x16, K = the tile's 16 rows; t and x columns split per tile)
// The round-1 kernel (k_gcn_bwd_nm) walked rowptr -> pair -> block as dependent round trips
// and ran dW and dx on f32 MFMA (4096 cycles per tile against 1536 here).
#ifndef LG_NB3_WFRAG
#define LG_NB3_WFRAG 1  // lab: 0 = the round-5 row-major W^T planes (stride LG_NB3_SBPAD + D halves)
#endif
#ifndef LG_NB3_SBPAD
#define LG_NB3_SBPAD 8
#endif
template <int D, bool MASK_IN>
struct Nb3Lds {
    // W^T planes.  The dx product reads a plane as MFMA A fragments, ds_read_b128, lane (j, q)
    // at row 16 mt + j, halves 32 s2 + 8 q.  Row-major with a padded row stride, the guide's LDS
    // banking (tools/lab/lds_banks.py: lane groups {0-3, 12-15, 20-27}, ...) hits banks twice at
    // D + 8 = 72 halves on all 24 plane reads of a tile, and a conflict-free stride (80) cost
    // VGPRs (r06f).  LG_NB3_WFRAG: the planes are stored in fragment order instead, fragment
    // (mt, s2) a 1 KB block with lane l's 16 bytes at 16 l: every read is 64 consecutive 16-byte
    // pieces (conflict-free), addressed by one per-lane base plus immediates, and a plane is
    // D x D halves (no padding).  The prologue's element writes scatter (once per workgroup).
    static constexpr int SB = LG_NB3_WFRAG ? D : (D == 64 ? D + LG_NB3_SBPAD : D + 8);
    static constexpr int WF = (3 * D * SB) / 2;          // W^T split parts (bf16), in floats
    static constexpr int TL = 2 * NmGeo<D>::TILE;         // per wave: t tile + x tile
    static constexpr int L = D * D + 2 * D;               // slab row: dW, db, d(node bias)
    static constexpr int MX = WF + kNmBwdWaves3 * TL > L ? WF + kNmBwdWaves3 * TL : L;
    static constexpr size_t BYTES = 4 * static_cast<size_t>(MX);
};

#ifndef LG_NB3_SPLIT
#define LG_NB3_SPLIT 0  // lab: 1 = the tail round of k_gcn_bwd_nm3 in pieces (r06x: 50.3 vs 48.0 us, slower)
#endif
#ifndef LG_NB3_NPF
#define LG_NB3_NPF 3  // neighbour blocks in flight in the backward (4: 44.6 / 40.2 against 43.2 / 38.7 us, r06zl)
#endif
// MB (with MASK_IN): the layer's output mask comes as the forward's ymask bits instead of a
// gather of y, so the prefetch keeps the unmasked depth.
// X0 (layer 0 on the compressed node init, lg_gcn_bwd_nm_x0): the tile's own x block is a
// sensor row block of x = xs0 [S][B][D] (pos_slot of the schedule position >= 0) or, for any
// other node, its [x0 > 0] mask word: x0 = bit ? relu(bias) * scale : 0.
struct NbX0 {
    const uint16_t* bits;
    const float* bias;
    float scale;
    uint32_t S;
    const int32_t* pos_slot;
};
// F16 (the fp32 tier's default, ABI 22): both GEMMs on the 2-way f16 split (split_bf16.h
// f16x2: 3 f16 MFMAs per product instead of 6 bf16 ones, half the split VALU and W^T planes)
// with power-of-two scales: W^T per workgroup (2^sW), a tile's t and x blocks per tile (the
// wave's own tile: a wave max each, 2^st, 2^sx).  dx^T is unscaled by 2^-(sW + st); dW
// accumulates in units of 2^T, T = st + sx of the latest tile, the accumulators rescaled
// (exactly) when T changes and unscaled once at the end.
template <int D, bool MASK_IN, bool NB, bool BF = false, bool MB = false, bool X0 = false, bool F16 = false>
__global__ void __launch_bounds__(64 * kNmBwdWaves3, 2)
k_gcn_bwd_nm3(const int32_t* __restrict__ tab, const int2* __restrict__ pairs, const float* __restrict__ dy,
              const float* __restrict__ yv, const float* __restrict__ x, const float* __restrict__ W,
              const int32_t* __restrict__ node_slot, float* __restrict__ dxo, float* __restrict__ slab, uint32_t N,
              uint32_t B, uint32_t ngroups, lg_fastdiv fdN, int mask_out, float scale_in, float scale_out,
              const uint16_t* __restrict__ ymask, NbX0 x0) {
    static_assert(!MB || MASK_IN, "mask bits replace the y gather of MASK_IN");
    constexpr bool MY = MASK_IN && !MB;  // mask from gathered y rows
    using G = NmGeo<D>;
    using LY = Nb3Lds<D, MASK_IN>;
    constexpr int SB = LY::SB;
    constexpr int NPF = MY ? 2 : LG_NB3_NPF;
    constexpr int L = LY::L;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint16_t* wsl = reinterpret_cast<uint16_t*>(smem);  // 3 x W^T [in][out] bf16, stride SB
    float* tiles = reinterpret_cast<float*>(smem) + LY::WF;

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
#ifdef LG_NM3_STAMPS
    constexpr int WAVES = kNmBwdWaves3;
    LG_NM3_STAMP(0, __builtin_amdgcn_s_memrealtime());
    LG_NM3_STAMP(1, __builtin_amdgcn_s_memtime());
    int tcount = 0;
#endif
    const int rl = lane / G::LPR, fg = lane % G::LPR;
    float* tl = tiles + wave * LY::TL;  // t tile [row][feature], later dx
    float* xl = tl + G::TILE;           // x tile [row][feature]
    // LDS addresses: tile row r, 16-byte chunk c4 (rows padded to G::S floats); W^T plane element
    // (row i, column o) at wix(i, o) halves
    auto tix = [&](int r, int c4) { return r * G::S + 4 * c4; };
    auto tel = [&](int r, int c) { return r * G::S + c; };
    auto wix = [&](int i, int o) {
        if constexpr (LG_NB3_WFRAG)  // fragment (i / 16, o / 32), lane (i % 16) + 16 ((o % 32) / 8), half o % 8
            return (((i >> 4) * (D / 32) + (o >> 5)) * 64 + (i & 15) + 16 * ((o & 31) >> 3)) * 8 + (o & 7);
        else
            return i * SB + o;
    };
    // the A fragment (mt, s2) of lane (j, q): W^T rows 16 mt + j, columns 32 s2 + 8 q .. + 7
    auto wrd = [&](int mt, int s2) {
        if constexpr (LG_NB3_WFRAG)
            return (mt * (D / 32) + s2) * 512 + 8 * lane;
        else
            return wix(16 * mt + j, 32 * s2 + 8 * q);
    };
    constexpr int WP = D * SB;  // halves per W^T plane
    const uint64_t bytes = static_cast<uint64_t>(N) * B * (4u * D);
    const __amdgpu_buffer_rsrc_t dys = nm_rsrc(dy, bytes), ms = nm_rsrc(MY ? yv : dy, bytes),
                                 xs = nm_rsrc(x, X0 ? static_cast<uint64_t>(x0.S) * B * (4u * D) : bytes),
                                 dxs = nm_rsrc(dxo, bytes);
    const __amdgpu_buffer_rsrc_t mbs = nm_mask_rsrc(ymask, N, ngroups);
    const __amdgpu_buffer_rsrc_t x0bs = nm_mask_rsrc(x0.bits, N, ngroups);
    f32x4 v0 = f32x4{0.f, 0.f, 0.f, 0.f};  // X0: a kept non-sensor element of the lane's slots
    if constexpr (X0) {
        const f32x4 bv = ld4(x0.bias + 4 * fg);
#pragma unroll
        for (int i = 0; i < 4; ++i) v0[i] = fmaxf(bv[i], 0.f) * x0.scale;
    }
    uint32_t loff[G::K];
#pragma unroll
    for (int k = 0; k < G::K; ++k) loff[k] = (G::RPI * k + rl) * (4u * D) + 16u * fg;
    const NmSched sc = nm_sched(static_cast<int64_t>(ngroups) * N, wave, kNmBwdWaves3);
    // 32-bit scalar tile indices (ntiles < 2^26; see k_gcn_fwd_pc): no 64-bit compares in VGPR pairs
    const int32_t tfirst = static_cast<int32_t>(sc.first), tstride = static_cast<int32_t>(sc.stride);
    // LG_NB3_SPLIT: the tail round in pieces.  The waves of an XCD's chunk (nm_sched) walk
    // F = C / stride full rounds of its C tiles; the R = C - F stride tiles left would run as a
    // last round on R of the stride waves (L-TOWN-A, B = 256: 1,322 tiles over 256 waves, a 6th
    // round for 42 of them).  Those R tiles are cut into q pieces of 16 / q rows each (q the
    // largest power of two <= K with q R <= stride), so the last round is q R shorter tiles on
    // as many waves.  A piece is the tile with the other rows' loads out of range (their t, x and
    // dx rows are zeros, their stores dropped): the same record, mask words and arithmetic.
    // Virtual index v: [cs, cs + F stride) full tiles, then q R pieces.
    int32_t vcs = 0, vfull = 0, vend = static_cast<int32_t>(sc.end);
    int qsh = 0;
    {
        const int64_t G = gridDim.x;
        const int64_t ntiles = static_cast<int64_t>(ngroups) * N;
        int64_t c0 = 0, c1 = ntiles;
        if (G >= 8) {
            const int64_t chunk = (ntiles + 7) / 8, x = blockIdx.x % 8;
            c0 = std::min<int64_t>(ntiles, x * chunk);
            c1 = std::min<int64_t>(ntiles, c0 + chunk);
        }
        const int64_t C = c1 - c0, W = sc.stride, F = C / W, R = C - F * W;
        vcs = static_cast<int32_t>(c0);
        vfull = static_cast<int32_t>(c0 + F * W);
        if (LG_NB3_SPLIT && R > 0)
            while (qsh < 2 && (int64_t{2} << qsh) <= G::K && (R << (qsh + 1)) <= W) ++qsh;
        vend = static_cast<int32_t>(c0 + F * W + (R << qsh));
    }
    const int32_t tend = vend;

    // virtual index -> (node, window base b0, rows [rlo, nb) of the 16-row block)
    auto tile_coords = [&](int32_t v, uint32_t& n, uint32_t& b0, uint32_t& nb, uint32_t& rlo) {
        const bool valid = v < vend;
        int32_t tile = valid ? v : vcs;
        rlo = 0;
        uint32_t rhi = 16;
        if (qsh && tile >= vfull) {
            const int32_t h = tile - vfull;
            tile = vfull + (h >> qsh);
            const uint32_t rows = 16u >> qsh;
            rlo = static_cast<uint32_t>(h & ((1 << qsh) - 1)) * rows;
            rhi = rlo + rows;
        }
        const uint32_t t32 = static_cast<uint32_t>(tile);
        const uint32_t grp = lg_div(t32, fdN);
        n = t32 - grp * N;
        b0 = grp * 16;
        nb = valid ? min(rhi, B - b0) : 0u;
    };
    auto ld = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off) {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    };
    // dz of one loaded block: MASK_IN applies this layer's relu/dropout backward
    auto dzf = [&](const f32x4& g, const f32x4& m) {
        if constexpr (!MASK_IN) return g;
        f32x4 r;
#pragma unroll
        for (int c = 0; c < 4; ++c) r[c] = m[c] > 0.f ? g[c] * scale_in : 0.f;
        return r;
    };
    // the same from mask bits (slot k of the lane)
    auto dzb = [&](const f32x4& g, uint32_t bits, int k) {
        f32x4 r;
#pragma unroll
        for (int c = 0; c < 4; ++c) r[c] = (bits >> (4 * k + c)) & 1u ? g[c] * scale_in : 0.f;
        return r;
    };
    // mask bits of the 16-row block of node m in window group grp (0 for an absent block)
    auto ldb = [&](uint32_t m, uint32_t grp, bool have) -> uint32_t {
        return __builtin_amdgcn_raw_buffer_load_b16(mbs, have ? nm_mask_off(m, grp, ngroups, lane) : kNm3BlkOob + 2u * lane,
                                                    0, 0);
    };

    // tile in flight: record, coordinates, lane offsets, first NPF neighbour blocks, own x block
    f32x4 pf[NPF][G::K], pm[MY ? NPF : 1][G::K], px[G::K];
    uint32_t pxb = 0;  // X0: the tile's own mask word
    uint32_t pmb[MB ? NPF : 1];
    uint32_t lo[G::K];
    NmRec cur;
    uint32_t cn, cb0;
    int cslot = -1;  // X0: the tile's sensor slot (-1: its x block is a mask word in px[0][0])
    auto issue = [&](const NmRec& r, uint32_t n, uint32_t b0, uint32_t nb, uint32_t rlo, int pslot) {
        n = static_cast<uint32_t>(r.node);  // tiles run in the table's schedule order (slot -> node)
        cur = r;
        cn = n;
        cb0 = b0;
        cslot = pslot;
#pragma unroll
        for (int k = 0; k < G::K; ++k) {
            const int row = G::RPI * k + rl;
            lo[k] = row < static_cast<int>(nb) && row >= static_cast<int>(rlo) ? loff[k] : kNm3RowOob;
        }
        // X0: both the sensor-row and the mask-word loads are always issued, the one that does
        // not apply out of range (a load under a branch is waited for where the branch merges)
        if constexpr (X0)
            pxb = __builtin_amdgcn_raw_buffer_load_b16(
                x0bs, nb && pslot < 0 ? nm_mask_off(n, b0 >> 4, ngroups, lane) : kNm3BlkOob + 2u * lane, 0, 0);
        const bool rows = nb > rlo && (!X0 || pslot >= 0);
        const uint32_t ob = rows ? ((X0 ? static_cast<uint32_t>(pslot) : n) * B + b0) * (4u * D) : kNm3BlkOob;
#pragma unroll
        for (int k = 0; k < G::K; ++k) px[k] = ld(xs, lo[k] + ob);
#pragma unroll
        for (int i = 0; i < NPF; ++i) {
            const bool have = r.e0 + i < r.e1;
            const uint32_t base = have ? (static_cast<uint32_t>(r.p[i].x) * B + b0) * (4u * D) : kNm3BlkOob;
#pragma unroll
            for (int k = 0; k < G::K; ++k) {
                pf[i][k] = ld(dys, lo[k] + base);
                if constexpr (MY) pm[i][k] = ld(ms, lo[k] + base);
            }
            if constexpr (MB) pmb[i] = ldb(static_cast<uint32_t>(r.p[i].x), b0 >> 4, have);
        }
    };
    // X0: the sensor slot of schedule position i (wave-uniform scalar load, no dependence on
    // the record)
    auto pslot_of = [&](uint32_t i) -> int { return X0 ? __builtin_amdgcn_readfirstlane(x0.pos_slot[i]) : -1; };
    // W^T split to LDS: element (o, i) of W lands at row i, column o of each part
    static_assert(!(F16 && BF), "one transform");
    int sW = 0;  // F16: W's scale exponent (every wave reads all of W for its max: no barrier)
    if constexpr (F16) {
        uint32_t m = 0;
        for (int u = lane; u < D * D / 4; u += 64) {
            const f32x4 v = ld4(W + 4 * u);
#pragma unroll
            for (int c = 0; c < 4; ++c) m = max(m, __float_as_uint(fabsf(v[c])));
        }
        sW = lg_f16_scale_exp_c(lg_wave_max_bits(m));
    }
    if constexpr (LG_NB3_WFRAG) {
        // fragment (mt, s2), lane l: W^T rows 16 mt + (l & 15), columns 32 s2 + 8 (l >> 4) .. + 7,
        // i.e. W[o][i] for 8 consecutive o: column reads of W (16 lanes = 64 contiguous bytes) and
        // one 16-byte LDS store per plane (64 consecutive pieces).  The per-element form (4 float4
        // reads, 48 2-byte LDS stores a thread) left the waves 9.3 us from start to this barrier (r06y).
        constexpr int CH = D / 16, KS = D / 32, NF = CH * KS * 64, NT3 = 64 * kNmBwdWaves3;
        constexpr int IT = (NF + NT3 - 1) / NT3;
        f32x4 wu[IT], wv[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int f = min(it * NT3 + static_cast<int>(threadIdx.x), NF - 1), l = f & 63, ms = f >> 6;
            const int i = 16 * (ms / KS) + (l & 15), k0 = 32 * (ms % KS) + 8 * (l >> 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                wu[it][e] = W[(k0 + e) * D + i];
                wv[it][e] = W[(k0 + 4 + e) * D + i];
            }
        }
        {  // the first tile's loads after W's (vmcnt counts in order: the stores below wait for W alone)
            uint32_t n0, b00, nb00, rl00;
            tile_coords(tfirst, n0, b00, nb00, rl00);
            issue(nm_rec(tab, N + n0), n0, b00, nb00, rl00, pslot_of(n0));  // schedule section
        }
        const float wsc = lg_pow2f(sW);
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int f = it * NT3 + static_cast<int>(threadIdx.x);
            if (f >= NF) continue;
            uint16_t* dst = wsl + 8 * f;
            if constexpr (F16) {
                lg_f16x8 h0, h1;
                split2_f16_x8(wu[it] * wsc, wv[it] * wsc, h0, h1);
                *reinterpret_cast<lg_f16x8*>(dst) = h0;
                *reinterpret_cast<lg_f16x8*>(dst + WP) = h1;
            } else {
                lg_bf16x8 h0, h1, h2;
                split3_x8(wu[it], wv[it], h0, h1, h2);
                *reinterpret_cast<lg_bf16x8*>(dst) = h0;
                if constexpr (!BF) {
                    *reinterpret_cast<lg_bf16x8*>(dst + WP) = h1;
                    *reinterpret_cast<lg_bf16x8*>(dst + 2 * WP) = h2;
                }
            }
        }
    } else {
    {
            constexpr int W4 = D * D / 4, WPER = (W4 + 64 * kNmBwdWaves3 - 1) / (64 * kNmBwdWaves3);
            f32x4 wv[WPER];
    #pragma unroll
            for (int u = 0; u < WPER; ++u) wv[u] = ld4(W + 4 * min<int>(u * 64 * kNmBwdWaves3 + threadIdx.x, W4 - 1));
            // the first tile's loads AFTER W's: vmcnt counts in order, so the staging below waits for
            // W alone (issued first, the staging waited for the tile's 20 gathered blocks as well:
            // 9.3 us from start to the barrier, r06y)
            {
                uint32_t n0, b00, nb00, rl00;
                tile_coords(tfirst, n0, b00, nb00, rl00);
                issue(nm_rec(tab, N + n0), n0, b00, nb00, rl00, pslot_of(n0));  // schedule section
            }
            const float wsc = lg_pow2f(sW);
    #pragma unroll
            for (int u = 0; u < WPER; ++u) {
                const int i4 = u * 64 * kNmBwdWaves3 + threadIdx.x;
                if (i4 >= W4) continue;
                const int o = i4 / (D / 4), c4 = 4 * (i4 % (D / 4));
    #pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int e = wix(c4 + c, o);
                    const float w = wv[u][c];
                    if constexpr (F16) {
                        const _Float16 h0 = static_cast<_Float16>(w * wsc);
                        const _Float16 h1 = static_cast<_Float16>(w * wsc - static_cast<float>(h0));
                        wsl[e] = __builtin_bit_cast(uint16_t, h0);
                        wsl[WP + e] = __builtin_bit_cast(uint16_t, h1);
                        continue;
                    }
                    const uint16_t h0 = __builtin_bit_cast(uint16_t, static_cast<__bf16>(w));
                    const float r1 = w - __uint_as_float(static_cast<uint32_t>(h0) << 16);
                    const uint16_t h1 = __builtin_bit_cast(uint16_t, static_cast<__bf16>(r1));
                    const float r2 = r1 - __uint_as_float(static_cast<uint32_t>(h1) << 16);
                    const uint16_t h2 = __builtin_bit_cast(uint16_t, static_cast<__bf16>(r2));
                    wsl[e] = h0;
                    wsl[WP + e] = h1;
                    wsl[2 * WP + e] = h2;
                }
            }
        }
    }
    __syncthreads();
    LG_NM3_STAMP(2, __builtin_amdgcn_s_memtime());

    f32x4 dw[G::CH][G::CH];  // dW tile (mo, ni): rows o = 16mo + 4q + reg, cols i = 16ni + j
#pragma unroll
    for (int a = 0; a < G::CH; ++a)
#pragma unroll
        for (int b = 0; b < G::CH; ++b) dw[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dbacc = f32x4{0.f, 0.f, 0.f, 0.f};  // channels 4fg..4fg+3, summed over this lane's rows
    int tc = 0;  // F16: dw holds dW x 2^tc
    f32x4 nbacc[NB ? G::CH : 1];              // NB: channels 16mt + 4q + reg over this lane's rows j
#pragma unroll
    for (int mt = 0; mt < (NB ? G::CH : 1); ++mt) nbacc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int32_t tile = tfirst; tile < tend; tile += tstride) {
        const uint32_t n = cn, b0 = cb0;
        const int e0 = cur.e0, e1 = cur.e1, self = cur.self;
        uint32_t tlo[G::K];
#pragma unroll
        for (int k = 0; k < G::K; ++k) tlo[k] = lo[k];
        uint32_t nn, nb0, nnb, nrlo;
        tile_coords(tile + tstride, nn, nb0, nnb, nrlo);
        const NmRec nxt = nm_rec(tab, N + nn);
        const int nslot = pslot_of(nn);
        asm volatile("" ::: "memory");  // keep the record request here (the compiler sinks it otherwise)
        f32x4 acc[G::K], xv[G::K];
        const uint32_t xw = pxb;
#pragma unroll
        for (int k = 0; k < G::K; ++k) {
            acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (X0 && cslot < 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i) xv[k][i] = (xw >> (4 * k + i)) & 1u ? v0[i] : 0.f;
            } else {
                xv[k] = px[k];
            }
        }
#pragma unroll
        for (int i = 0; i < NPF; ++i) {
            if (e0 + i < e1) {
                const float w = __int_as_float(cur.p[i].y);
#pragma unroll
                for (int k = 0; k < G::K; ++k) {
                    const f32x4 z = MB ? dzb(pf[i][k], pmb[MB ? i : 0], k)
                                       : dzf(pf[i][k], MY ? pm[i < (MY ? NPF : 1) ? i : 0][k] : pf[i][k]);
                    pk_fma4(acc[k], w, z);
                    if (i == self) dbacc += z;
                }
            }
        }
        if (e0 + NPF < e1) {  // the rest of the row: inline pairs, then the pair array
            int2 ip[kLgNmInline - NPF];
#pragma unroll
            for (int i = 0; i < kLgNmInline - NPF; ++i) ip[i] = cur.p[NPF + i];
#pragma unroll
            for (int i = 0; i < kLgNmInline - NPF; ++i) {
                if (e0 + NPF + i < e1) {
                    const uint32_t ba = (static_cast<uint32_t>(ip[i].x) * B + b0) * (4u * D);
                    f32x4 va[G::K], vm[G::K];
#pragma unroll
                    for (int k = 0; k < G::K; ++k) {
                        va[k] = ld(dys, tlo[k] + ba);
                        vm[k] = MY ? ld(ms, tlo[k] + ba) : va[k];
                    }
                    const uint32_t bm = MB ? ldb(static_cast<uint32_t>(ip[i].x), b0 >> 4, true) : 0u;
                    const float wa = __int_as_float(ip[i].y);
#pragma unroll
                    for (int k = 0; k < G::K; ++k) {
                        const f32x4 z = MB ? dzb(va[k], bm, k) : dzf(va[k], vm[k]);
                        pk_fma4(acc[k], wa, z);
                        if (NPF + i == self) dbacc += z;
                    }
                }
            }
            for (int e = e0 + kLgNmInline; e < e1; ++e) {
                const int2 pa = pairs[e];
                const uint32_t ba = (static_cast<uint32_t>(pa.x) * B + b0) * (4u * D);
                f32x4 va[G::K], vm[G::K];
#pragma unroll
                for (int k = 0; k < G::K; ++k) {
                    va[k] = ld(dys, tlo[k] + ba);
                    vm[k] = MY ? ld(ms, tlo[k] + ba) : va[k];
                }
                const uint32_t bm = MB ? ldb(static_cast<uint32_t>(pa.x), b0 >> 4, true) : 0u;
                const float wa = __int_as_float(pa.y);
#pragma unroll
                for (int k = 0; k < G::K; ++k) pk_fma4(acc[k], wa, MB ? dzb(va[k], bm, k) : dzf(va[k], vm[k]));
            }
        }
        if (self < 0) {  // no self entry among the inline pairs: the own dz rows explicitly
            const uint32_t ob = (n * B + b0) * (4u * D);
            const uint32_t bo = MB ? ldb(n, b0 >> 4, true) : 0u;
#pragma unroll
            for (int k = 0; k < G::K; ++k)
                dbacc += MB ? dzb(ld(dys, tlo[k] + ob), bo, k) : dzf(ld(dys, tlo[k] + ob), MY ? ld(ms, tlo[k] + ob) : f32x4{});
        }
        issue(nxt, nn, nb0, nnb, nrlo, nslot);
        __builtin_amdgcn_sched_barrier(0);

        int st = 0, sx = 0;  // F16: the tile's t and x scale exponents
        if constexpr (F16) {
            uint32_t mt4 = 0, mx4 = 0;
#pragma unroll
            for (int k = 0; k < G::K; ++k)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    mt4 = max(mt4, __float_as_uint(fabsf(acc[k][c])));
                    mx4 = max(mx4, __float_as_uint(fabsf(xv[k][c])));
                }
            st = lg_f16_scale_exp_c(lg_wave_max_bits(mt4));
            sx = lg_f16_scale_exp_c(lg_wave_max_bits(mx4));
            const int d = st + sx - tc;
            if (d != 0) {  // two exact power-of-two factors (|d| <= 252)
                const float r1 = lg_pow2f(d / 2), r2 = lg_pow2f(d - d / 2);
#pragma unroll
                for (int a = 0; a < G::CH; ++a)
#pragma unroll
                    for (int b = 0; b < G::CH; ++b) dw[a][b] = (dw[a][b] * r1) * r2;
                tc = st + sx;
            }
        }
        wave_sync_nm();
#pragma unroll
        for (int k = 0; k < G::K; ++k) {
            st4(tl + tix(G::RPI * k + rl, fg), acc[k]);
            st4(xl + tix(G::RPI * k + rl, fg), xv[k]);
        }
        wave_sync_nm();
        // dW += t^T x over the tile's 16 rows: A[o][r] = t[r][o], B[r][i] = x[r][i], K = rows 4q..4q+3
        if constexpr (F16) {
            const float tsc = lg_pow2f(st), xsc = lg_pow2f(sx);
            lg_f16x4 xb[G::CH][2];
#pragma unroll
            for (int ni = 0; ni < G::CH; ++ni) {
                f32x4 v;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) v[kk] = xl[tel(4 * q + kk, 16 * ni + j)] * xsc;
                split2_f16_x4(v, xb[ni][0], xb[ni][1]);
            }
#pragma unroll
            for (int mo = 0; mo < G::CH; ++mo) {
                f32x4 v;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) v[kk] = tl[tel(4 * q + kk, 16 * mo + j)] * tsc;
                lg_f16x4 a0, a1;
                split2_f16_x4(v, a0, a1);
#pragma unroll
                for (int ni = 0; ni < G::CH; ++ni) {
                    f32x4 c = dw[mo][ni];
                    c = __builtin_amdgcn_mfma_f32_16x16x16f16(a1, xb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x16f16(a0, xb[ni][1], c, 0, 0, 0);
                    dw[mo][ni] = __builtin_amdgcn_mfma_f32_16x16x16f16(a0, xb[ni][0], c, 0, 0, 0);
                }
            }
        } else {
            lg_i16x4 xb[G::CH][3];
#pragma unroll
            for (int ni = 0; ni < G::CH; ++ni) {
                f32x4 v;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) v[kk] = xl[tel(4 * q + kk, 16 * ni + j)];
                lg_u32x2 f0, f1, f2;
                split3_x4(v, f0, f1, f2);
                xb[ni][0] = __builtin_bit_cast(lg_i16x4, f0);
                xb[ni][1] = __builtin_bit_cast(lg_i16x4, f1);
                xb[ni][2] = __builtin_bit_cast(lg_i16x4, f2);
            }
#pragma unroll
            for (int mo = 0; mo < G::CH; ++mo) {
                f32x4 v;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) v[kk] = tl[tel(4 * q + kk, 16 * mo + j)];
                lg_u32x2 f0, f1, f2;
                split3_x4(v, f0, f1, f2);
                const lg_i16x4 a0 = __builtin_bit_cast(lg_i16x4, f0), a1 = __builtin_bit_cast(lg_i16x4, f1),
                                a2 = __builtin_bit_cast(lg_i16x4, f2);
#pragma unroll
                for (int ni = 0; ni < G::CH; ++ni) {
                    f32x4 c = dw[mo][ni];
                    if constexpr (BF) {
                        dw[mo][ni] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a0, xb[ni][0], c, 0, 0, 0);
                        continue;
                    }
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a2, xb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a1, xb[ni][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a0, xb[ni][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a1, xb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a0, xb[ni][1], c, 0, 0, 0);
                    dw[mo][ni] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a0, xb[ni][0], c, 0, 0, 0);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // dx^T[i][row] = sum_o W^T[i][o] t[row][o]
        f32x4 o[G::CH];
#pragma unroll
        for (int mt = 0; mt < G::CH; ++mt) o[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (F16) {  // on the f16x2 split, unscaled by 2^-(sW + st)
            const float tsc = lg_pow2f(st);
#pragma unroll
            for (int s2 = 0; s2 < D / 32; ++s2) {
                lg_f16x8 bh[2];
                split2_f16_x8(ld4(tl + tix(j, 8 * s2 + 2 * q)) * tsc, ld4(tl + tix(j, 8 * s2 + 2 * q + 1)) * tsc,
                              bh[0], bh[1]);
#pragma unroll
                for (int mt = 0; mt < G::CH; ++mt) {
                    const int ew = wrd(mt, s2);
                    const lg_f16x8 ah[2] = {*reinterpret_cast<const lg_f16x8*>(wsl + ew),
                                            *reinterpret_cast<const lg_f16x8*>(wsl + WP + ew)};
                    o[mt] = mfma_f16x2(ah, bh, o[mt]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            const float us = lg_pow2f(-(sW + st));
#pragma unroll
            for (int mt = 0; mt < G::CH; ++mt) o[mt] *= us;
        } else {
#pragma unroll
        for (int s2 = 0; s2 < D / 32; ++s2) {
            lg_bf16x8 b0f, b1f, b2f;
            split3_x8(ld4(tl + tix(j, 8 * s2 + 2 * q)), ld4(tl + tix(j, 8 * s2 + 2 * q + 1)), b0f, b1f, b2f);
#pragma unroll
            for (int mt = 0; mt < G::CH; ++mt) {
                const int ew = wrd(mt, s2);
                const lg_bf16x8 a0 = *reinterpret_cast<const lg_bf16x8*>(wsl + ew);
                if constexpr (BF) {
                    o[mt] = mfma_bf(a0, b0f, o[mt]);
                    continue;
                }
                const lg_bf16x8 a1 = *reinterpret_cast<const lg_bf16x8*>(wsl + WP + ew);
                const lg_bf16x8 a2 = *reinterpret_cast<const lg_bf16x8*>(wsl + 2 * WP + ew);
                o[mt] = mfma_bf(a2, b0f, o[mt]);
                o[mt] = mfma_bf(a1, b1f, o[mt]);
                o[mt] = mfma_bf(a0, b2f, o[mt]);
                o[mt] = mfma_bf(a1, b0f, o[mt]);
                o[mt] = mfma_bf(a0, b1f, o[mt]);
                o[mt] = mfma_bf(a0, b0f, o[mt]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        }
        if (mask_out & 1) {
#pragma unroll
            for (int mt = 0; mt < G::CH; ++mt) {
                const f32x4 xm = ld4(xl + tix(j, 4 * mt + q));
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) o[mt][reg] = xm[reg] > 0.f ? o[mt][reg] * scale_out : 0.f;
            }
        }
        if constexpr (NB) {  // node-bias rows: the tile's node has no sensor (uniform test)
            if (node_slot[n] < 0) {
#pragma unroll
                for (int mt = 0; mt < G::CH; ++mt) nbacc[mt] += o[mt];
                // LG_F_DX_SENSOR_ROWS: the node init's backward reads only the sensor rows of dx
                if (mask_out & 2) continue;
            }
        }
        wave_sync_nm();
#pragma unroll
        for (int mt = 0; mt < G::CH; ++mt) st4(tl + tix(j, 4 * mt + q), o[mt]);
        wave_sync_nm();
        const uint32_t ob = (n * B + b0) * (4u * D);
        f32x4 vk[G::K];
#pragma unroll
        for (int k = 0; k < G::K; ++k) vk[k] = ld4(tl + tix(G::RPI * k + rl, fg));
#pragma unroll
        for (int k = 0; k < G::K; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, vk[k]),
                                                   dxs, tlo[k] + ob, 0, kLgActAux);
        lg_store_guard(vk);
#ifdef LG_NM3_STAMPS
        if (tcount < 16) LG_NM3_STAMP(3 + tcount, __builtin_amdgcn_s_memtime());
        ++tcount;
#endif
    }
#ifdef LG_NM3_STAMPS
    LG_NM3_STAMP(21, __builtin_amdgcn_s_memtime());
    LG_NM3_STAMP(22, __builtin_amdgcn_s_memrealtime());
    LG_NM3_STAMP(23, (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11))) << 32) |
                         static_cast<uint64_t>(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11))));
#endif
    if constexpr (F16) {  // dw back to units of 1 (two exact factors)
        const float r1 = lg_pow2f(-(tc / 2)), r2 = lg_pow2f(-(tc - tc / 2));
#pragma unroll
        for (int a = 0; a < G::CH; ++a)
#pragma unroll
            for (int b = 0; b < G::CH; ++b) dw[a][b] = (dw[a][b] * r1) * r2;
    }
    if constexpr (NB) {  // fold the 16 row lanes j of each (q, reg)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1)
#pragma unroll
            for (int mt = 0; mt < G::CH; ++mt)
#pragma unroll
                for (int i = 0; i < 4; ++i) nbacc[mt][i] += __shfl_xor(nbacc[mt][i], off);
    }
    // ---- per-block reduction of dW / db / node bias (fixed wave order -> deterministic)
#pragma unroll
    for (int off = G::LPR; off < 64; off <<= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) dbacc[i] += __shfl_xor(dbacc[i], off);
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // reuse the whole LDS image
    for (int i = threadIdx.x; i < L; i += blockDim.x) red[i] = 0.f;
    for (int wv2 = 0; wv2 < kNmBwdWaves3; ++wv2) {
        __syncthreads();
        if (wave == wv2) {
#pragma unroll
            for (int mo = 0; mo < G::CH; ++mo)
#pragma unroll
                for (int ni = 0; ni < G::CH; ++ni)
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg)
                        red[(16 * mo + 4 * q + reg) * D + 16 * ni + j] += dw[mo][ni][reg];
            if (lane < G::LPR)
#pragma unroll
                for (int i = 0; i < 4; ++i) red[D * D + 4 * lane + i] += dbacc[i];
            if (NB && j == 0)
#pragma unroll
                for (int mt = 0; mt < G::CH; ++mt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) red[D * D + D + 16 * mt + 4 * q + i] += nbacc[mt][i];
        }
    }
    __syncthreads();
    float* out = slab + static_cast<int64_t>(blockIdx.x) * L;
    for (int i = threadIdx.x; i < L; i += blockDim.x) out[i] = red[i];
}

// ------------------------------------------------------------------ single graph (B = 1), row tiles
// GCNConv on ONE graph (the reference module's own call shape, x [N][D]; BASELINE configs[4]:
// 100k nodes, 300k edge columns).  The node-major kernels tile one node x 16 windows and
// share the node's neighbour list across the tile; at B = 1 a tile is 16 NODES (16
// consecutive slots of the node table's schedule section, RCM order), each with its own
// neighbour list.  Lane (rl, fg) owns features 4 fg.. of tile rows 4 k + rl (D = 64: the 16
// lanes of a DPP row cover one node row).  Per tile:
//   * the 16 records are ONE coalesced vector load (lane fg of a row holds word fg of its
//     node's 64-byte record), requested a tile ahead; e0, e1, the six inline (col, w) pairs,
//     self and node are broadcast inside each 16-lane row by DPP row_newbcast (VALU, no
//     LDS, no scalar round trip per row);
//   * the inline neighbour rows of the 16 nodes in batches of 4 slots (buffer loads with the
//     per-lane row address in the VGPR offset, an absent neighbour out of range), entries
//     beyond six from the pair array afterwards;
//   * the tile goes through LDS (XOR swizzle) to the MFMA transform on the 3-way bf16 split
//     (W's parts in LDS in fragment order: one conflict-free ds_read_b128 per fragment), and
//     rows go back out whole through the same LDS tile.
// The window-major kernel (k_gcn_fwd) it replaces at B = 1 walked rowptr -> col -> row as
// three dependent global round trips per round of two neighbours (profiles/r03: 0.25 of
// HBM peak at C5).
constexpr int kRowWaves = 4;
#ifndef LG_ROWS_FWD_NB
#define LG_ROWS_FWD_NB 4  // inline neighbours per gather batch (x 4 rows per lane; 2 / 3 / 4 / 6 measured, profiles/r03/r03ad)
#endif
#ifndef LG_ROWS_BWD_NB
#define LG_ROWS_BWD_NB 4
#endif

template <int n>
__device__ __forceinline__ int row_bcast(int v) {  // lane n of each 16-lane row, to the row
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + n, 0xF, 0xF, false);
}

struct RowsLds {  // floats
    static constexpr int D = 64, CH = 4, KS = 2;
    static constexpr int WFR = 3 * CH * KS * 64 * 4;   // W (fwd) or W^T (bwd) bf16 split parts, fragment order
    static constexpr int BOFF = WFR;                    // bias [D]
    static constexpr int TOFF = BOFF + D;               // per wave: tile (fwd) / t tile + x tile (bwd)
    static constexpr int TILE = 16 * D;
    static constexpr int L = D * D + 2 * D;
    static constexpr size_t fwd_bytes() { return 4 * static_cast<size_t>(TOFF + kRowWaves * TILE); }
    static constexpr size_t bwd_bytes() {
        return 4 * static_cast<size_t>(TOFF + 2 * kRowWaves * TILE > L ? TOFF + 2 * kRowWaves * TILE : L);
    }
    static __device__ __forceinline__ int tix(int r, int c) { return r * D + 4 * (c ^ r); }
};

// The 3-way bf16 split of M (TRANS: of M^T) into fragment order: fragment (part, mt, s2),
// lane (j, q) holds A[i = 16 mt + j][k = 32 s2 + 8 q + e], A = M or M^T, M [D][D] row-major.
template <bool TRANS>
__device__ __forceinline__ void stage_frag3(uint32_t* wfr, const float* __restrict__ M, int nthreads) {
    constexpr int D = 64, CH = 4, KS = 2;
    for (int f = threadIdx.x; f < CH * KS * 64; f += nthreads) {
        const int l = f & 63, ms = f >> 6, mt = ms / KS, s2 = ms % KS;
        const int i = 16 * mt + (l & 15), k0 = 32 * s2 + 8 * (l >> 4);
        f32x4 u, v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            u[e] = TRANS ? M[(k0 + e) * D + i] : M[i * D + k0 + e];
            v[e] = TRANS ? M[(k0 + 4 + e) * D + i] : M[i * D + k0 + 4 + e];
        }
        lg_bf16x8 f0, f1, f2;
        split3_x8(u, v, f0, f1, f2);
        *reinterpret_cast<lg_bf16x8*>(wfr + 4 * ((0 * CH * KS + ms) * 64 + l)) = f0;
        *reinterpret_cast<lg_bf16x8*>(wfr + 4 * ((1 * CH * KS + ms) * 64 + l)) = f1;
        *reinterpret_cast<lg_bf16x8*>(wfr + 4 * ((2 * CH * KS + ms) * 64 + l)) = f2;
    }
}

// dst^T (16 rows x 64) = A (from the fragments) x tile^T, tile rows j: o[mt] = rows j,
// columns 16 mt + 4 q .. (the fwd transform with A = W, the bwd dx with A = W^T)
__device__ __forceinline__ void rows_transform(const uint32_t* wfr, const float* tl, int lane, f32x4 (&o)[4]) {
    using LY = RowsLds;
    constexpr int CH = 4, KS = 2;
    const int j = lane & 15, q = lane >> 4;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
        lg_bf16x8 b[3];
        split3_x8(ld4(tl + LY::tix(j, 8 * s2 + 2 * q)), ld4(tl + LY::tix(j, 8 * s2 + 2 * q + 1)), b[0], b[1], b[2]);
#pragma unroll
        for (int mt = 0; mt < CH; ++mt) {
            lg_bf16x8 a[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const lg_bf16x8*>(wfr + 4 * ((p * CH * KS + mt * KS + s2) * 64 + lane));
            o[mt] = mfma_split(a, b, o[mt]);
        }
    }
}

// One tile's records (lane fg: word fg of row 4 k + rl's record) and their decoding
struct RowsRec {
    int e0[4], e1[4], self[4], node[4];
    int col[4][kLgNmInline];
    float w[4][kLgNmInline];
};
__device__ __forceinline__ void rows_decode(const int (&rw)[4], RowsRec& r) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        r.e0[k] = row_bcast<0>(rw[k]);
        r.e1[k] = row_bcast<1>(rw[k]);
        r.col[k][0] = row_bcast<2>(rw[k]);
        r.w[k][0] = __int_as_float(row_bcast<3>(rw[k]));
        r.col[k][1] = row_bcast<4>(rw[k]);
        r.w[k][1] = __int_as_float(row_bcast<5>(rw[k]));
        r.col[k][2] = row_bcast<6>(rw[k]);
        r.w[k][2] = __int_as_float(row_bcast<7>(rw[k]));
        r.col[k][3] = row_bcast<8>(rw[k]);
        r.w[k][3] = __int_as_float(row_bcast<9>(rw[k]));
        r.col[k][4] = row_bcast<10>(rw[k]);
        r.w[k][4] = __int_as_float(row_bcast<11>(rw[k]));
        r.col[k][5] = row_bcast<12>(rw[k]);
        r.w[k][5] = __int_as_float(row_bcast<13>(rw[k]));
        r.self[k] = row_bcast<14>(rw[k]);
        r.node[k] = row_bcast<15>(rw[k]);
    }
}
// record words of tile `tile` (slots 16 tile + 4 k + rl; past N: an empty row)
__device__ __forceinline__ void rows_load_rec(const int32_t* __restrict__ tab, uint32_t N, int64_t tile, int lane,
                                              int (&rw)[4]) {
    const int rl = lane >> 4, fg = lane & 15;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t slot = 16 * tile + 4 * k + rl;
        rw[k] = slot < N ? tab[16 * (static_cast<int64_t>(N) + slot) + fg] : 0;
    }
}
// acc[k] = sum over row 4k + rl's entries (CSR order) of w * src[col] (features 4 fg..); own[k]
// = the row's own src row (from its self entry, else loaded) when OWN
template <bool OWN, int NBATCH>
__device__ __forceinline__ void rows_gather(const RowsRec& r, const int2* __restrict__ pairs, __amdgpu_buffer_rsrc_t src,
                                            int lane, f32x4 (&acc)[4], f32x4 (&own)[4]) {
    constexpr int D = 64;
    const uint32_t lo = 16u * static_cast<uint32_t>(lane & 15);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (OWN) own[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    int maxd = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) maxd = max(maxd, r.e1[k] - r.e0[k]);
    // inline entries in batches of NBATCH x 4 rows in flight; a batch no row reaches is skipped
#pragma unroll
    for (int i0 = 0; i0 < kLgNmInline; i0 += NBATCH) {
        if (__builtin_amdgcn_ballot_w64(maxd > i0) == 0) break;
        f32x4 v[4][NBATCH];
#pragma unroll
        for (int i = 0; i < NBATCH; ++i)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (i0 + i >= kLgNmInline) continue;  // past the inline six: never read
                const bool have = r.e0[k] + i0 + i < r.e1[k];
                // per-lane row: the whole address in the VGPR offset (a per-lane descriptor or soffset
                // is a waterfall loop: measured 27.5 -> 17 us at C5); an absent slot reads out of
                // range (0, no memory request)
                const uint32_t off = lo + static_cast<uint32_t>(r.col[k][i0 + i < kLgNmInline ? i0 + i : 0]) * (4u * D);
                v[k][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(src, have ? off : kNm3RowOob, 0, 0));
            }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int i = 0; i < NBATCH; ++i) {
                if (i0 + i >= kLgNmInline) continue;
                pk_fma4(acc[k], r.e0[k] + i0 + i < r.e1[k] ? r.w[k][i0 + i] : 0.f, v[k][i]);  // absent: 0 x 0
                if (OWN && i0 + i == r.self[k]) own[k] = v[k][i];
            }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        for (int e = r.e0[k] + kLgNmInline; e < r.e1[k]; ++e) {  // per-row tail (degree > 6)
            const int2 pa = pairs[e];
            const f32x4 t = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(src, lo + static_cast<uint32_t>(pa.x) * (4u * D), 0, 0));
            pk_fma4(acc[k], __int_as_float(pa.y), t);
        }
        if (OWN && (r.self[k] < 0) && r.e0[k] < r.e1[k])  // self entry past the inline six
            own[k] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(src, lo + static_cast<uint32_t>(r.node[k]) * (4u * D), 0, 0));
    }
}

template <bool BIAS>
__global__ void __launch_bounds__(64 * kRowWaves)
k_gcn_fwd_rows(const int32_t* __restrict__ tab, const int2* __restrict__ pairs, const float* __restrict__ x,
               const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ y, uint32_t N) {
    constexpr int D = 64;
    using LY = RowsLds;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* lds = reinterpret_cast<float*>(smem);
    uint32_t* wfr = reinterpret_cast<uint32_t*>(lds);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4, rl = lane >> 4, fg = lane & 15;
    float* tl = lds + LY::TOFF + wave * LY::TILE;
    const int64_t ntiles = (static_cast<int64_t>(N) + 15) / 16;
    const NmSched sc = nm_sched(ntiles, wave, kRowWaves);
    const uint64_t bytes = static_cast<uint64_t>(N) * (4u * D);
    const __amdgpu_buffer_rsrc_t xs = nm_rsrc(x, bytes), ys = nm_rsrc(y, bytes);
#ifdef LG_NM3_STAMPS
    constexpr int WAVES = kRowWaves;
    int tcount = 0;
    LG_NM3_STAMP(0, __builtin_amdgcn_s_memrealtime());
    LG_NM3_STAMP(1, __builtin_amdgcn_s_memtime());
#endif
    int rw[4];
    rows_load_rec(tab, N, sc.first < sc.end ? sc.first : 0, lane, rw);
    stage_frag3<false>(wfr, W, 64 * kRowWaves);
    if (threadIdx.x < D) lds[LY::BOFF + threadIdx.x] = BIAS ? bias[threadIdx.x] : 0.f;
    __syncthreads();
#ifdef LG_NM3_STAMPS
    LG_NM3_STAMP(2, __builtin_amdgcn_s_memtime());
#endif
    for (int64_t tile = sc.first; tile < sc.end; tile += sc.stride) {
        RowsRec r;
        rows_decode(rw, r);
        rows_load_rec(tab, N, tile + sc.stride < sc.end ? tile + sc.stride : tile, lane, rw);  // next tile's records
        f32x4 acc[4], own[4];
        rows_gather<false, LG_ROWS_FWD_NB>(r, pairs, xs, lane, acc, own);
#ifdef LG_NM3_STAMPS
        asm volatile("" ::"v"(acc[0]), "v"(acc[1]), "v"(acc[2]), "v"(acc[3]));
        if (tcount < 6) LG_NM3_STAMP(3 + 3 * tcount, __builtin_amdgcn_s_memtime());
#endif
        wave_sync_nm();
#pragma unroll
        for (int k = 0; k < 4; ++k) st4(tl + LY::tix(4 * k + rl, fg), acc[k]);
        wave_sync_nm();
        f32x4 o[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) o[mt] = ld4(lds + LY::BOFF + 16 * mt + 4 * q);
        rows_transform(wfr, tl, lane, o);
#ifdef LG_NM3_STAMPS
        asm volatile("" ::"v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]));
        if (tcount < 6) LG_NM3_STAMP(4 + 3 * tcount, __builtin_amdgcn_s_memtime());
#endif
        wave_sync_nm();
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) st4(tl + LY::tix(j, 4 * mt + q), o[mt]);
        wave_sync_nm();
        f32x4 vk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) vk[k] = ld4(tl + LY::tix(4 * k + rl, fg));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool valid = 16 * tile + 4 * k + rl < N;
            const uint32_t off = valid ? static_cast<uint32_t>(r.node[k]) * (4u * D) + 16u * fg : kNm3RowOob;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, vk[k]),
                                                   ys, off, 0, kLgActAux);
        }
        lg_store_guard(vk);
#ifdef LG_NM3_STAMPS
        if (tcount < 6) LG_NM3_STAMP(5 + 3 * tcount, __builtin_amdgcn_s_memtime());
        ++tcount;
#endif
    }
#ifdef LG_NM3_STAMPS
    LG_NM3_STAMP(21, __builtin_amdgcn_s_memtime());
    LG_NM3_STAMP(22, __builtin_amdgcn_s_memrealtime());
    LG_NM3_STAMP(23, (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11))) << 32) |
                         static_cast<uint64_t>(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11))));
#endif
}

// Backward on one graph: t = Ahat^T dy (transposed table), dx = t W, dW += t^T x, db += the
// rows' own dy; dW / db per workgroup in a fixed wave order into the slab row.
__global__ void __launch_bounds__(64 * kRowWaves, 2)
k_gcn_bwd_rows(const int32_t* __restrict__ tab, const int2* __restrict__ pairs, const float* __restrict__ dy,
               const float* __restrict__ x, const float* __restrict__ W, float* __restrict__ dxo,
               float* __restrict__ slab, uint32_t N) {
    constexpr int D = 64;
    using LY = RowsLds;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* lds = reinterpret_cast<float*>(smem);
    uint32_t* wfr = reinterpret_cast<uint32_t*>(lds);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4, rl = lane >> 4, fg = lane & 15;
    float* tl = lds + LY::TOFF + 2 * wave * LY::TILE;
    float* xl = tl + LY::TILE;
    const int64_t ntiles = (static_cast<int64_t>(N) + 15) / 16;
    const NmSched sc = nm_sched(ntiles, wave, kRowWaves);
    const uint64_t bytes = static_cast<uint64_t>(N) * (4u * D);
    const __amdgpu_buffer_rsrc_t dys = nm_rsrc(dy, bytes), xs = nm_rsrc(x, bytes),
                                 dxs = nm_rsrc(dxo, bytes);
    int rw[4];
    rows_load_rec(tab, N, sc.first < sc.end ? sc.first : 0, lane, rw);
    stage_frag3<true>(wfr, W, 64 * kRowWaves);
    __syncthreads();
    f32x4 dw[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) dw[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dbacc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int64_t tile = sc.first; tile < sc.end; tile += sc.stride) {
        RowsRec r;
        rows_decode(rw, r);
        rows_load_rec(tab, N, tile + sc.stride < sc.end ? tile + sc.stride : tile, lane, rw);
        f32x4 xv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool valid = 16 * tile + 4 * k + rl < N;
            xv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  xs, valid ? static_cast<uint32_t>(r.node[k]) * (4u * D) + 16u * fg : kNm3RowOob,
                                                  0, 0));
        }
        f32x4 acc[4], own[4];
        rows_gather<true, LG_ROWS_BWD_NB>(r, pairs, dys, lane, acc, own);
#pragma unroll
        for (int k = 0; k < 4; ++k) dbacc += own[k];
        wave_sync_nm();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            st4(tl + LY::tix(4 * k + rl, fg), acc[k]);
            st4(xl + LY::tix(4 * k + rl, fg), xv[k]);
        }
        wave_sync_nm();
        // dW += t^T x over the tile's 16 rows (K = rows 4q..4q+3), bf16 split, in place
        {
            lg_i16x4 xb[4][3];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                f32x4 v;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int rr = 4 * q + kk, c = 16 * ni + j;
                    v[kk] = xl[LY::tix(rr, c >> 2) + (c & 3)];
                }
                lg_u32x2 f0, f1, f2;
                split3_x4(v, f0, f1, f2);
                xb[ni][0] = __builtin_bit_cast(lg_i16x4, f0);
                xb[ni][1] = __builtin_bit_cast(lg_i16x4, f1);
                xb[ni][2] = __builtin_bit_cast(lg_i16x4, f2);
            }
#pragma unroll
            for (int mo = 0; mo < 4; ++mo) {
                f32x4 v;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int rr = 4 * q + kk, c = 16 * mo + j;
                    v[kk] = tl[LY::tix(rr, c >> 2) + (c & 3)];
                }
                lg_u32x2 f0, f1, f2;
                split3_x4(v, f0, f1, f2);
                const lg_i16x4 a0 = __builtin_bit_cast(lg_i16x4, f0), a1 = __builtin_bit_cast(lg_i16x4, f1),
                                a2 = __builtin_bit_cast(lg_i16x4, f2);
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) {
                    f32x4 c = dw[mo][ni];
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a2, xb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a1, xb[ni][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a0, xb[ni][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a1, xb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a0, xb[ni][1], c, 0, 0, 0);
                    dw[mo][ni] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a0, xb[ni][0], c, 0, 0, 0);
                }
            }
        }
        f32x4 o[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) o[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        rows_transform(wfr, tl, lane, o);  // dx^T = W^T t^T
        wave_sync_nm();
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) st4(tl + LY::tix(j, 4 * mt + q), o[mt]);
        wave_sync_nm();
        f32x4 vk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) vk[k] = ld4(tl + LY::tix(4 * k + rl, fg));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool valid = 16 * tile + 4 * k + rl < N;
            const uint32_t off = valid ? static_cast<uint32_t>(r.node[k]) * (4u * D) + 16u * fg : kNm3RowOob;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, vk[k]),
                                                   dxs, off, 0, kLgActAux);
        }
        lg_store_guard(vk);
    }
    // db: fold the 4 row groups (lanes fg, fg + 16, ..), then waves in a fixed order
#pragma unroll
    for (int off = 16; off < 64; off <<= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) dbacc[i] += __shfl_xor(dbacc[i], off);
    __syncthreads();
    constexpr int L = LY::L;
    float* red = lds;
    for (int i = threadIdx.x; i < L; i += blockDim.x) red[i] = 0.f;
    for (int wv2 = 0; wv2 < kRowWaves; ++wv2) {
        __syncthreads();
        if (wave == wv2) {
#pragma unroll
            for (int mo = 0; mo < 4; ++mo)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) red[(16 * mo + 4 * q + reg) * D + 16 * ni + j] += dw[mo][ni][reg];
            if (lane < 16)
#pragma unroll
                for (int i = 0; i < 4; ++i) red[D * D + 4 * lane + i] += dbacc[i];
        }
    }
    __syncthreads();
    float* out = slab + static_cast<int64_t>(blockIdx.x) * L;
    for (int i = threadIdx.x; i < L; i += blockDim.x) out[i] = red[i];
}

template <typename Kern>
int nm_grid(Kern kernel, int threads, size_t dyn, int64_t ntiles, int waves, int cap_per_cu) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        static_cast<int>(dyn));
    int per_cu = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, dyn) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const int64_t want = (ntiles + waves - 1) / waves;
    const int64_t cap = static_cast<int64_t>(std::min(per_cu, cap_per_cu)) * lg_num_cus();
    return static_cast<int>(std::max<int64_t>(1, std::min(want, cap)));
}

bool nm_fits(int64_t B, int64_t N, int64_t D) { return N * B * D * 4 <= static_cast<int64_t>(kNm3MaxBytes); }

template <int D, bool DR, bool RL>
auto nm3_kernel(int flags) {
    if (flags & LG_F_BF16) return k_gcn_fwd_nm3<D, DR, RL, true, 4, true>;
    return (flags & LG_F_F32_MFMA) ? k_gcn_fwd_nm3<D, DR, RL, false, 4> : k_gcn_fwd_nm3<D, DR, RL, true, 4>;
}
template <int D, bool DR, bool RL, bool X0>
auto pc_kernel(bool bf16, bool f16) {
    return bf16 ? k_gcn_fwd_pc<D, DR, RL, true, false, kPcProdN, kPcNC, X0>
                : (f16 ? k_gcn_fwd_pc<D, DR, RL, false, true, kPcProdN, kPcNC, X0>
                       : k_gcn_fwd_pc<D, DR, RL, false, false, kPcProdN, kPcNC, X0>);
}

// lg_gcn_fwd_nm_bits (x0 == NULL) and lg_gcn_fwd_nm_x0 (x the sensor rows, *x0 the rest)
int nm_fwd(const int32_t* nodetab, const int32_t* pairs, const float* x, const float* W, const float* bias, float* y,
           int64_t B, int64_t N, int64_t D, int flags, float dropout_p, uint64_t seed, uint32_t salt,
           lg_stream_t stream, uint16_t* ymask, const PcX0* x0) {
    if (B < 0 || N <= 0 || !nodetab || !pairs || !x || !W || !y || x == y) return LG_EINVAL;
    if ((flags & LG_F_BIAS) && !bias) return LG_EINVAL;
    const bool drop = (flags & LG_F_DROPOUT) != 0;
    if (drop && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    if (B == 0) return LG_OK;
    if (!nm_fits(B, N, D) || N * ((B + 15) / 16) >= kLgMaxRows) return LG_EUNSUPPORTED;
    const int64_t ngroups = (B + 15) / 16, ntiles = ngroups * N;
    const float scale = drop ? 1.0f / (1.0f - dropout_p) : 1.0f;
    const float* bp = (flags & LG_F_BIAS) ? bias : nullptr;
    const bool relu = (flags & LG_F_RELU) != 0;
    const bool bf16 = (flags & LG_F_BF16) != 0;
    // Kernel and transform (results: see include/leakgnn.h):
    //   fp32 tier, default: the producer / consumer pipeline k_gcn_fwd_pc with the 2-way fp16
    //     transform; LG_F_BF16X3: the same pipeline on the 3-way bf16 split;
    //   LG_F_NM3: the per-wave pipeline k_gcn_fwd_nm3 (3-way bf16 split; LG_F_F32_MFMA: exact
    //     fp32 MFMA, bit-identical to lg_gcn_fwd);
    //   bf16 tier (LG_F_BF16): nm3's single bf16 product, or pc's with LG_F_PC.
    // The compressed layer-0 input runs on pc only.
    const bool nm3 = !x0 && ((flags & (LG_F_NM3 | LG_F_F32_MFMA)) != 0 || (bf16 && !(flags & LG_F_PC)));
    const bool f16 = !bf16 && !(flags & LG_F_BF16X3);
    const int2* pr = reinterpret_cast<const int2*>(pairs);
    const lg_fastdiv fd = lg_make_fastdiv(static_cast<uint32_t>(N));
    hipStream_t s = lg_stream(stream);
    const uint32_t N32 = static_cast<uint32_t>(N), B32 = static_cast<uint32_t>(B), G32 = static_cast<uint32_t>(ngroups);
    const PcX0 xz = x0 ? *x0 : PcX0{nullptr, nullptr, 1.f, 0u};
    auto launch = [&](auto dc, auto drc) {
        constexpr int DD = decltype(dc)::value;
        constexpr bool DR = decltype(drc)::value;
        if (nm3) {
            auto kern = relu ? nm3_kernel<DD, DR, true>(flags) : nm3_kernel<DD, DR, false>(flags);
            const size_t dyn = (flags & LG_F_F32_MFMA) && !bf16 ? Nm3Lds<DD, false, 4>::BYTES : Nm3Lds<DD, true, 4>::BYTES;
            const int grid = nm_grid(kern, 64 * 4, dyn, ntiles, 4, 3);
            lg_launch(kern, grid, 64 * 4, dyn, s, nodetab, pr, x, W, bp, y, N32, B32, G32, fd, dropout_p, scale, seed,
                      salt, ymask);
        } else {
            auto kern = x0 ? (relu ? pc_kernel<DD, DR, true, true>(bf16, f16) : pc_kernel<DD, DR, false, true>(bf16, f16))
                           : (relu ? pc_kernel<DD, DR, true, false>(bf16, f16) : pc_kernel<DD, DR, false, false>(bf16, f16));
            const size_t dyn = PcLds<DD, kPcProdN, kPcNC>::BYTES;
            const int thr = 64 * kPcProdN * (1 + kPcNC);
            const int grid = nm_grid(kern, thr, dyn, ntiles, 4, 1);
            lg_launch(kern, grid, thr, dyn, s, nodetab, pr, x, W, bp, y, N32, B32, G32, fd, dropout_p, scale, seed,
                      salt, ymask, xz);
        }
    };
    using I32 = std::integral_constant<int, 32>;
    using I64 = std::integral_constant<int, 64>;
    using T = std::true_type;
    using F = std::false_type;
    if (D == 64) {
        if (drop) launch(I64{}, T{});
        else launch(I64{}, F{});
    } else {
        if (drop) launch(I32{}, T{});
        else launch(I32{}, F{});
    }
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

}  // namespace

extern "C" int lg_gcn_fwd_nm_bits(const int32_t* nodetab, const int32_t* pairs, const float* x, const float* W,
                             const float* bias, float* y, int64_t B, int64_t N, int64_t D, int64_t nnz_cap, int flags,
                             float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream, uint16_t* ymask) {
    (void)nnz_cap;
    return nm_fwd(nodetab, pairs, x, W, bias, y, B, N, D, flags, dropout_p, seed, salt, stream, ymask, nullptr);
}

extern "C" int lg_gcn_fwd_nm_x0(const int32_t* nodetab_s, const int32_t* pairs_s, const float* xs0,
                                const uint16_t* x0bits, const float* node_bias, const float* W, const float* bias,
                                float* y, int64_t B, int64_t N, int64_t S, int64_t D, int flags, float dropout_p,
                                uint64_t seed, uint32_t salt, lg_stream_t stream) {
    if (S < 0 || S > 0xFFFF || !x0bits || !node_bias || !xs0) return LG_EINVAL;
    if (S * B * D * 4 > static_cast<int64_t>(kNm3MaxBytes)) return LG_EUNSUPPORTED;
    // the compressed layer-0 input runs on the producer / consumer kernel only: the nm3 and exact
    // fp32 forms are refused rather than silently replaced
    if (flags & (LG_F_NM3 | LG_F_F32_MFMA)) return LG_EUNSUPPORTED;
    const bool drop = (flags & LG_F_DROPOUT) != 0;
    const float scale = drop && dropout_p >= 0.f && dropout_p < 1.f ? 1.0f / (1.0f - dropout_p) : 1.0f;
    const PcX0 x0{x0bits, node_bias, scale, static_cast<uint32_t>(S)};
    return nm_fwd(nodetab_s, pairs_s, xs0, W, bias, y, B, N, D, flags, dropout_p, seed, salt, stream, nullptr, &x0);
}

#if defined(LG_NM3_STAMPS) || defined(LG_PC_PROBE)
// kernel-lab timeline readout (LG_NM3_STAMPS / LG_PC_PROBE builds only; see g_nm3_stamps)
extern "C" int lg_lab_nm3_stamps(uint64_t* host, int64_t n) {
    if (n > static_cast<int64_t>(8192) * kNm3Stamps) return LG_EINVAL;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_nm3_stamps), static_cast<size_t>(n) * 8) == hipSuccess ? LG_OK
                                                                                                         : LG_EHIP;
}
extern "C" int lg_lab_nm3_stamps_clear(void) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_nm3_stamps)) != hipSuccess) return LG_EHIP;
    return hipMemset(p, 0, sizeof(uint64_t) * 8192 * kNm3Stamps) == hipSuccess ? LG_OK : LG_EHIP;
}
#endif

extern "C" int lg_gcn_fwd_nm(const int32_t* nodetab, const int32_t* pairs, const float* x, const float* W,
                             const float* bias, float* y, int64_t B, int64_t N, int64_t D, int64_t nnz_cap, int flags,
                             float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream) {
    return lg_gcn_fwd_nm_bits(nodetab, pairs, x, W, bias, y, B, N, D, nnz_cap, flags, dropout_p, seed, salt, stream,
                              nullptr);
}

extern "C" int64_t lg_gcn_bwd_nm_workspace_bytes(int64_t D) {
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    return static_cast<int64_t>(2) * lg_num_cus() * (D * D + 2 * D) * static_cast<int64_t>(sizeof(float));
}

namespace {
// lg_gcn_bwd_nm_bits (x0 == NULL) and lg_gcn_bwd_nm_x0 (x the sensor rows, *x0 the rest)
int nm_bwd(const int32_t* nodetab_t, const int32_t* pairs_t, const float* dy, const float* y, const float* x,
           const float* W, float* dx_out, float* dW, float* db, const int32_t* node_slot, float* dnode_bias, int64_t B,
           int64_t N, int64_t D, int flags, float scale_in, float scale_out, void* workspace, int64_t ws_bytes,
           lg_stream_t stream, const uint16_t* ymask, const NbX0* x0) {
    if (B < 0 || N <= 0 || !nodetab_t || !pairs_t || !dy || !x || !W || !dx_out || !dW || !workspace) return LG_EINVAL;
    if ((node_slot == nullptr) != (dnode_bias == nullptr)) return LG_EINVAL;
    const bool mask_in = (flags & LG_F_MASK_IN) != 0;
    if (mask_in && !y && !ymask) return LG_EINVAL;
    if (x0 && mask_in) return LG_EUNSUPPORTED;  // layer 0: its output mask is the next layer's input mask
    const bool mbits = mask_in && ymask != nullptr;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    if (!nm_fits(B, N, D) || N * ((B + 15) / 16) >= kLgMaxRows) return LG_EUNSUPPORTED;
    const int64_t ngroups = (B + 15) / 16, ntiles = std::max<int64_t>(ngroups * N, 0);
    // bit 0: MASK_OUT; bit 1: LG_F_DX_SENSOR_ROWS
    const int mask_out = ((flags & LG_F_MASK_OUT) ? 1 : 0) | ((node_slot && (flags & LG_F_DX_SENSOR_ROWS)) ? 2 : 0);
    const int2* pr = reinterpret_cast<const int2*>(pairs_t);
    const lg_fastdiv fd = lg_make_fastdiv(static_cast<uint32_t>(N));
    // the launch grid is at most 2 x CUs workgroups, one slab row each
    if (ws_bytes < lg_gcn_bwd_nm_workspace_bytes(D)) return LG_EINVAL;
    float* slab = static_cast<float*>(workspace);
    hipStream_t s = lg_stream(stream);
    const bool bf = (flags & LG_F_BF16) != 0;
    // fp32 tier: the f16x2 transform unless LG_F_BF16X3 asks for the 3-way bf16 split
    const bool f16 = !bf && !(flags & LG_F_BF16X3);
    const NbX0 xz = x0 ? *x0 : NbX0{nullptr, nullptr, 1.f, 0u, nullptr};
    // k_gcn_bwd_nm3: the 3-way bf16 split (fp32 tier) or the single bf16 product (LG_F_BF16)
    int grid = 1;
    // B == 0 still runs one (empty) launch so the slab holds zeros
    auto launch = [&](auto kern, size_t dyn3) {
        grid = std::min<int>(nm_grid(kern, 64 * kNmBwdWaves3, dyn3, std::max<int64_t>(ntiles, 1), kNmBwdWaves3, 2),
                             2 * lg_num_cus());
        lg_launch(kern, grid, 64 * kNmBwdWaves3, dyn3, s, nodetab_t, pr, dy, y, x, W, node_slot, dx_out, slab,
                  static_cast<uint32_t>(N), static_cast<uint32_t>(B), static_cast<uint32_t>(ngroups), fd, mask_out,
                  scale_in, scale_out, ymask, xz);
    };
#define LG_NM_BWD_P(DD, MI, NBB, MBB, X0B)                                                                        \
    launch(bf ? k_gcn_bwd_nm3<DD, MI, NBB, true, MBB, X0B>                                                        \
              : (f16 ? k_gcn_bwd_nm3<DD, MI, NBB, false, MBB, X0B, true> : k_gcn_bwd_nm3<DD, MI, NBB, false, MBB, X0B>), \
           Nb3Lds<DD, MI>::BYTES)
#define LG_NM_BWD(DD, MI, NBB)                                                                                     \
    do {                                                                                                           \
        if constexpr (!MI) {                                                                                       \
            if (x0) {                                                                                              \
                LG_NM_BWD_P(DD, false, NBB, false, true);                                                          \
                break;                                                                                             \
            }                                                                                                      \
        }                                                                                                          \
        if (MI && mbits) LG_NM_BWD_P(DD, MI, NBB, MI, false);                                                      \
        else LG_NM_BWD_P(DD, MI, NBB, false, false);                                                               \
    } while (0)
#define LG_NM_BWD_D(DD)                                  \
    do {                                                 \
        if (mask_in) {                                   \
            if (node_slot) LG_NM_BWD(DD, true, true);    \
            else LG_NM_BWD(DD, true, false);             \
        } else {                                         \
            if (node_slot) LG_NM_BWD(DD, false, true);   \
            else LG_NM_BWD(DD, false, false);            \
        }                                                \
    } while (0)
    if (D == 64) LG_NM_BWD_D(64);
    else LG_NM_BWD_D(32);
#undef LG_NM_BWD_D
#undef LG_NM_BWD
#undef LG_NM_BWD_P
    LG_RET_IF_LAUNCH_FAILED();
    const int64_t L = D * D + 2 * D;
    const LgSlabSeg segs[3] = {{0, D * D, dW}, {D * D, D, db}, {D * D + D, D, dnode_bias}};
    return lg_launch_slab_reduce_multi(slab, grid, L, segs, 3, nullptr, nullptr, s);
}
}  // namespace

extern "C" int lg_gcn_bwd_nm_bits(const int32_t* nodetab_t, const int32_t* pairs_t, const float* dy, const float* y,
                             const float* x, const float* W, float* dx_out, float* dW, float* db,
                             const int32_t* node_slot, float* dnode_bias, int64_t B, int64_t N, int64_t D, int flags,
                             float scale_in, float scale_out, void* workspace, int64_t ws_bytes, lg_stream_t stream,
                             const uint16_t* ymask) {
    return nm_bwd(nodetab_t, pairs_t, dy, y, x, W, dx_out, dW, db, node_slot, dnode_bias, B, N, D, flags, scale_in,
                  scale_out, workspace, ws_bytes, stream, ymask, nullptr);
}

extern "C" int lg_gcn_bwd_nm_x0(const int32_t* nodetab_t, const int32_t* pairs_t, const int32_t* pos_slot_t,
                                const float* dy, const float* xs0, const uint16_t* x0bits, const float* node_bias,
                                const float* W, float* dx_out, float* dW, float* db, const int32_t* node_slot,
                                float* dnode_bias, int64_t B, int64_t N, int64_t S, int64_t D, int flags,
                                float dropout_p, float scale_out, void* workspace, int64_t ws_bytes,
                                lg_stream_t stream) {
    if (S < 0 || S > 0xFFFF || !x0bits || !node_bias || !xs0 || !pos_slot_t) return LG_EINVAL;
    if (S * B * D * 4 > static_cast<int64_t>(kNm3MaxBytes)) return LG_EUNSUPPORTED;
    const bool drop = (flags & LG_F_DROPOUT) != 0;
    if (drop && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    const NbX0 x0{x0bits, node_bias, drop ? 1.0f / (1.0f - dropout_p) : 1.0f, static_cast<uint32_t>(S), pos_slot_t};
    return nm_bwd(nodetab_t, pairs_t, dy, nullptr, xs0, W, dx_out, dW, db, node_slot, dnode_bias, B, N, D,
                  flags & ~LG_F_DROPOUT, 1.0f, scale_out, workspace, ws_bytes, stream, nullptr, &x0);
}

extern "C" int lg_gcn_bwd_nm(const int32_t* nodetab_t, const int32_t* pairs_t, const float* dy, const float* y,
                             const float* x, const float* W, float* dx_out, float* dW, float* db,
                             const int32_t* node_slot, float* dnode_bias, int64_t B, int64_t N, int64_t D, int flags,
                             float scale_in, float scale_out, void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    return lg_gcn_bwd_nm_bits(nodetab_t, pairs_t, dy, y, x, W, dx_out, dW, db, node_slot, dnode_bias, B, N, D, flags,
                              scale_in, scale_out, workspace, ws_bytes, stream, nullptr);
}

extern "C" int lg_gcn_fwd_rows(const int32_t* nodetab, const int32_t* pairs, const float* x, const float* W,
                               const float* bias, float* y, int64_t N, int64_t D, int flags, lg_stream_t stream) {
    if (N <= 0 || !nodetab || !pairs || !x || !W || !y || x == y) return LG_EINVAL;
    if ((flags & LG_F_BIAS) && !bias) return LG_EINVAL;
    if (flags & ~LG_F_BIAS) return LG_EUNSUPPORTED;
    if (D != 64 || !nm_fits(1, N, D)) return LG_EUNSUPPORTED;
    const int64_t ntiles = (N + 15) / 16;
    hipStream_t s = lg_stream(stream);
    const size_t dyn = RowsLds::fwd_bytes();
    const int2* pr = reinterpret_cast<const int2*>(pairs);
    if (flags & LG_F_BIAS) {
        auto kern = k_gcn_fwd_rows<true>;
        const int grid = nm_grid(kern, 64 * kRowWaves, dyn, ntiles, kRowWaves, 4);
        lg_launch(kern, grid, 64 * kRowWaves, dyn, s, nodetab, pr, x, W, bias, y, static_cast<uint32_t>(N));
    } else {
        auto kern = k_gcn_fwd_rows<false>;
        const int grid = nm_grid(kern, 64 * kRowWaves, dyn, ntiles, kRowWaves, 4);
        lg_launch(kern, grid, 64 * kRowWaves, dyn, s, nodetab, pr, x, W, bias, y, static_cast<uint32_t>(N));
    }
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_gcn_bwd_rows(const int32_t* nodetab_t, const int32_t* pairs_t, const float* dy, const float* x,
                               const float* W, float* dx, float* dW, float* db, int64_t N, int64_t D, void* workspace, int64_t ws_bytes,
                               lg_stream_t stream) {
    if (N <= 0 || !nodetab_t || !pairs_t || !dy || !x || !W || !dx || !dW || !workspace) return LG_EINVAL;
    if (D != 64 || !nm_fits(1, N, D)) return LG_EUNSUPPORTED;
    if (ws_bytes < lg_gcn_bwd_nm_workspace_bytes(D)) return LG_EINVAL;  // <= 2 x CUs slab rows
    const int64_t ntiles = (N + 15) / 16;
    hipStream_t s = lg_stream(stream);
    const size_t dyn = RowsLds::bwd_bytes();
    auto kern = k_gcn_bwd_rows;
    // the slab holds lg_gcn_bwd_nm_workspace_bytes(D) / (4 L) = 2 x CUs rows
    const int grid = std::min<int>(nm_grid(kern, 64 * kRowWaves, dyn, ntiles, kRowWaves, 2), 2 * lg_num_cus());
    float* slab = static_cast<float*>(workspace);
    lg_launch(kern, grid, 64 * kRowWaves, dyn, s, nodetab_t, reinterpret_cast<const int2*>(pairs_t), dy, x, W, dx, slab,
              static_cast<uint32_t>(N));
    LG_RET_IF_LAUNCH_FAILED();
    const int64_t L = D * D + 2 * D;
    const LgSlabSeg segs[2] = {{0, D * D, dW}, {D * D, D, db}};
    return lg_launch_slab_reduce_multi(slab, grid, L, segs, 2, nullptr, nullptr, s);
}

extern "C" int lg_spin_errors(uint32_t* out, int reset) {
    if (!out) return LG_EINVAL;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pc_spin_err), sizeof(uint32_t)) != hipSuccess) return LG_EHIP;
    if (reset) {
        const uint32_t z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pc_spin_err), &z, sizeof(uint32_t)) != hipSuccess) return LG_EHIP;
    }
    return LG_OK;
}
