// K1+K2 node init, K8 pipe-endpoint gather / incidence scatter, K10 mean pool.
// All HBM-bound row kernels: D/4 lanes per row, one float4 per lane, rows read
// and written as whole 4*D-byte lines.
#include <algorithm>
#include <deque>
#include <mutex>
#include <vector>

#include "common.h"
#include "reduce.h"

namespace {

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Node init dropout: the row-stream rule of the fused GCN forward (common.h
// lg_row_stream_seed, oracle/dropout_ref.py row_stream_mask) with the window-major row id,
// so both layouts draw the same mask.  The bulk rows are written by lane groups (row, q):
// lane q owns channels 16 mt + 4 q .. + 3 of its row, i.e. exactly one stream, so a row
// costs one seed and D / 8 xorshift32 steps per lane instead of a multiply hash per element.
constexpr int kNiRowsPerBlock = 64;  // 256 threads, 4 lanes per row

// v[mt] = keep(channel 16 mt + 4 q + reg) ? t[mt] : 0 over the (row, q) stream
template <int CH>
__device__ __forceinline__ void ni_stream_select(uint32_t key, uint64_t rw, uint32_t q, uint32_t thr,
                                                 const f32x4 (&t)[CH], f32x4 (&v)[CH]) {
    uint32_t st = lg_row_stream_seed(key, rw, q);
#pragma unroll
    for (int mt = 0; mt < CH; ++mt) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            if ((reg & 1) == 0) st = lg_xorshift32(st);
            const uint32_t u16 = (reg & 1) ? (st >> 16) : (st & 0xFFFFu);
            v[mt][reg] = u16 >= thr ? t[mt][reg] : 0.0f;
        }
    }
}

// Output row r of x0: window-major r = b N + n, node-major (nm) r = n B + b; fdM divides by
// the fast index's extent (N, resp. B).  x0 = dropout(relu(sensor row ? proj[b][slot] : bias)).
template <int D>
__global__ void __launch_bounds__(256)
k_node_init(const int32_t* __restrict__ slot, const float* __restrict__ proj, const float* __restrict__ bias,
            float* __restrict__ x0, int64_t N, lg_fastdiv fdM, int nm, int64_t S, int64_t R, int dropout, float p,
            float scale, uint64_t seed, uint32_t salt) {
    constexpr int CH = D / 16;
    const int rl = threadIdx.x >> 2, q = threadIdx.x & 3;
    const uint32_t key = lg_dropout_key_dev(seed, salt);
    const uint32_t thr = lg_keep_threshold16(p);
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * kNiRowsPerBlock + rl; r < R;
         r += static_cast<int64_t>(gridDim.x) * kNiRowsPerBlock) {
        const uint32_t hi = lg_div(static_cast<uint32_t>(r), fdM), lo = static_cast<uint32_t>(r) - hi * fdM.d;
        const uint32_t b = nm ? lo : hi, n = nm ? hi : lo;
        const int32_t s = slot[n];
        const float* src = s >= 0 ? proj + (static_cast<int64_t>(b) * S + s) * D : bias;
        f32x4 t[CH], v[CH];
#pragma unroll
        for (int mt = 0; mt < CH; ++mt) {
            t[mt] = ld4(src + 16 * mt + 4 * q);
#pragma unroll
            for (int i = 0; i < 4; ++i) t[mt][i] = fmaxf(t[mt][i], 0.f) * (dropout ? scale : 1.0f);
        }
        if (dropout) ni_stream_select<CH>(key, static_cast<uint64_t>(b) * N + n, q, thr, t, v);
        else
#pragma unroll
            for (int mt = 0; mt < CH; ++mt) v[mt] = t[mt];
#pragma unroll
        for (int mt = 0; mt < CH; ++mt) st4(x0 + r * D + 16 * mt + 4 * q, v[mt]);
    }
}

// k_node_init with the sensor projection folded in (detector.py:160, 184-190): a sensor
// row's pre-activation is h_s[b][s] . W[o][:Ds] + (W[o][Ds] + bias[o]) (its Linear input is
// [h_s, 1]), every other row's is bias (input [0, 0]).  The first GS workgroups stage W^T
// and the folded bias in LDS and form the S*B sensor rows (a lane group per row, 4 outputs
// per lane, 4 * Ds fmas in ascending k); the workgroups after them write the non-sensor rows
// (kNiRowsPerBlock each), so no other workgroup pays for W.
template <int D, int DS>
__global__ void __launch_bounds__(256)
k_node_init_proj(const int32_t* __restrict__ slot, const int64_t* __restrict__ sidx, const float* __restrict__ hs,
                 const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ x0, int64_t B,
                 int64_t N, lg_fastdiv fdM, int nm, int64_t S, int64_t R, int GS, int dropout, float p, float scale,
                 uint64_t seed, uint32_t salt) {
    constexpr int LPR = D / 4, RPB = 256 / LPR, CH = D / 16;
    __shared__ __attribute__((aligned(16))) float wt[DS][D];  // W^T[k][o]
    __shared__ __attribute__((aligned(16))) float bf[D];      // W[o][DS] + bias[o]
    const uint32_t key = lg_dropout_key_dev(seed, salt);
    const uint32_t thr = lg_keep_threshold16(p);
    if (static_cast<int>(blockIdx.x) < GS) {
        const int rl = threadIdx.x / LPR, fg = threadIdx.x % LPR;
        for (int i = threadIdx.x; i < D * (DS + 1); i += 256) {  // o fastest: conflict-free LDS writes
            const int k = i / D, o = i % D;
            if (k < DS) wt[k][o] = W[o * (DS + 1) + k];
            else bf[o] = W[o * (DS + 1) + DS] + bias[o];
        }
        __syncthreads();
        const f32x4 bs = ld4(bf + 4 * fg);
        for (int64_t q = static_cast<int64_t>(blockIdx.x) * RPB + rl; q < S * B; q += static_cast<int64_t>(GS) * RPB) {
            const int64_t sc = q / B, b = q - sc * B, n = sidx[sc];
            if (slot[n] != sc) continue;  // a duplicated sensor id: the last one's row wins (detector.py:181)
            const float* hrow = hs + (b * S + sc) * DS;
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
            for (int k4 = 0; k4 < DS / 4; ++k4) {
                const f32x4 h4 = ld4(hrow + 4 * k4);
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const f32x4 w = ld4(&wt[4 * k4 + kk][4 * fg]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i] = fmaf(h4[kk], w[i], acc[i]);
                }
            }
            f32x4 v = acc + bs;
            const uint32_t kb = dropout ? lg_row_stream_keep4(key, static_cast<uint64_t>(b * N + n), 4 * fg, thr) : 0xFu;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = ((kb >> i) & 1u) ? fmaxf(v[i], 0.f) * (dropout ? scale : 1.0f) : 0.0f;
            st4(x0 + (nm ? n * B + b : b * N + n) * D + 4 * fg, v);
        }
    }
    // every row without a sensor: dropout(relu(bias)).  Flat grid: the workgroups after the
    // first GS own kNiRowsPerBlock rows each.  The keep bits are drawn in (row, q) lane groups
    // (one stream per group, as above) and posted to LDS; the rows are then stored as whole
    // lines (at D = 64 a wave's store covers 4 whole rows, 1 KiB contiguous, instead of 64-byte
    // pieces of 16 rows).
    if (static_cast<int>(blockIdx.x) < GS) return;
    __shared__ uint32_t kbits[kNiRowsPerBlock][4];  // keep bits of (row, q): bit 4 mt + reg
    const int64_t r0 = static_cast<int64_t>(static_cast<int>(blockIdx.x) - GS) * kNiRowsPerBlock;
    {
        const int rl = threadIdx.x >> 2, q = threadIdx.x & 3;
        const int64_t r = r0 + rl;
        uint32_t kb = 0xFFFFFFFFu;
        if (dropout && r < R) {
            const uint32_t hi = lg_div(static_cast<uint32_t>(r), fdM), lo = static_cast<uint32_t>(r) - hi * fdM.d;
            const uint32_t b = nm ? lo : hi, n = nm ? hi : lo;
            uint32_t st = lg_row_stream_seed(key, static_cast<uint64_t>(b) * N + n, q);
            kb = 0;
#pragma unroll
            for (int mt = 0; mt < CH; ++mt)
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) {
                    if ((reg & 1) == 0) st = lg_xorshift32(st);
                    const uint32_t u16 = (reg & 1) ? (st >> 16) : (st & 0xFFFFu);
                    kb |= static_cast<uint32_t>(u16 >= thr) << (4 * mt + reg);
                }
        }
        kbits[rl][q] = kb;
    }
    __syncthreads();
    // store phase: lane -> (row, float4 group fg), LPR lanes per row
    const int fg = threadIdx.x % LPR, mt = fg >> 2, q = fg & 3;
    f32x4 t = ld4(bias + 4 * fg);
#pragma unroll
    for (int i = 0; i < 4; ++i) t[i] = fmaxf(t[i], 0.f) * (dropout ? scale : 1.0f);
#pragma unroll
    for (int it = 0; it < kNiRowsPerBlock / RPB; ++it) {
        const int rl = it * RPB + static_cast<int>(threadIdx.x) / LPR;
        const int64_t r = r0 + rl;
        if (r >= R) break;
        const uint32_t hi = lg_div(static_cast<uint32_t>(r), fdM), lo = static_cast<uint32_t>(r) - hi * fdM.d;
        const uint32_t n = nm ? hi : lo;
        if (slot[n] >= 0) continue;
        const uint32_t kb = kbits[rl][q] >> (4 * mt);
        f32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = ((kb >> i) & 1u) ? t[i] : 0.0f;
        st4(x0 + r * D + 4 * fg, v);
    }
}

// Compressed node init (lg_node_init_bits_fwd): x0 never materialised.  Output:
//   xs0   [S][B][D]: the sensor rows dropout(relu([h_s, 1] W^T + b)) of every LIVE slot s
//                    (the node's last slot, detector.py:181), node-major per slot;
//   x0bits          : [x0 > 0] of EVERY row in the node-major mask layout of lg_gcn_fwd_nm_bits
//                    (per 16-row tile (node n, window group g) one uint16 per lane l of the
//                    gather layout: bit 4 k + i = row 16 g + RPI k + l / LPR, channel
//                    4 (l % LPR) + i);
// a non-sensor element is then x0 = bit ? relu(b) * scale : 0 exactly (relu(b) * scale > 0
// <=> b > 0 kept).  The first GS workgroups stage W^T and form the sensor tiles (16 rows
// each: the same per-row arithmetic as k_node_init_proj, so the rows are bit-identical),
// posting each row's nibbles to LDS and storing the tile's mask words; the workgroups after
// them write the non-sensor tiles' mask words, one lane of one tile per thread.
// non-sensor tiles per thread of k_node_init_bits: 1 (r04m: 4 measured 14.1 us against 11.7)
constexpr int kNibTiles = 1;
template <int D, int DS>
__global__ void __launch_bounds__(256)
k_node_init_bits(const int32_t* __restrict__ slot, const int64_t* __restrict__ sidx, const float* __restrict__ hs,
                 const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ xs0,
                 uint16_t* __restrict__ bits, uint32_t B, uint32_t N, uint32_t S, uint32_t ngroups, lg_fastdiv fdG,
                 int GS, int dropout, float p, float scale, uint64_t seed, uint32_t salt) {
    constexpr int LPR = D / 4, RPI = 64 / LPR, K = 16 / RPI, TPI = 256 / (16 * LPR);
    const uint32_t key = lg_dropout_key_dev(seed, salt);
    const uint32_t thr = lg_keep_threshold16(p);
    if (static_cast<int>(blockIdx.x) < GS) {
        // one tile (16 rows) of TPI sensor tiles per iteration.  Latency first: W's rows and the
        // tiles' h_s rows are requested together, coalesced (a float4 per thread), and meet in LDS
        // behind one barrier; each lane then forms 4 outputs of one row from LDS (the h_s element
        // is a broadcast read), the same ascending-k fmaf chain as k_node_init_proj.
        __shared__ __attribute__((aligned(16))) float wt[DS][D];        // W^T[k][o]
        __shared__ __attribute__((aligned(16))) float bf[D];            // W[o][DS] + bias[o]
        __shared__ __attribute__((aligned(16))) float hl[TPI][16][DS];  // the tiles' h_s rows
        __shared__ uint8_t nib[TPI][16][LPR];
        const int rr = threadIdx.x / LPR, fg = threadIdx.x % LPR, ti = rr / 16, r = rr % 16;
        constexpr int WF4 = D * (DS + 1) / 4;  // W is [D][DS + 1] row-major: float4 i = elements 4i..4i+3
        constexpr int WPT = (WF4 + 255) / 256;
        f32x4 wv[WPT];
#pragma unroll
        for (int u = 0; u < WPT; ++u) wv[u] = ld4(W + 4 * min(u * 256 + static_cast<int>(threadIdx.x), WF4 - 1));
        const uint32_t T = S * ngroups;
        constexpr int HF4 = TPI * 16 * DS / 4, HPT = (HF4 + 255) / 256;  // h_s float4 per iteration
        auto load_h = [&](uint32_t t0, f32x4 (&hv)[HPT]) {
#pragma unroll
            for (int u = 0; u < HPT; ++u) {
                const int e = u * 256 + static_cast<int>(threadIdx.x);  // (tile j, row rj, float4 kk)
                const int j = e / (16 * DS / 4), rj = (e / (DS / 4)) % 16, kk = e % (DS / 4);
                const uint32_t t = t0 + j;
                const uint32_t sc = t < T ? lg_div(t, fdG) : 0u, g = t < T ? t - sc * ngroups : 0u;
                const uint32_t b = min(16 * g + rj, B - 1);
                hv[u] = e < HF4 ? ld4(hs + (static_cast<size_t>(b) * S + sc) * DS + 4 * kk) : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        };
        f32x4 hv[HPT];
        load_h(blockIdx.x * TPI, hv);
#pragma unroll
        for (int u = 0; u < WPT; ++u) {
            const int i4 = u * 256 + static_cast<int>(threadIdx.x);
            if (i4 >= WF4) continue;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int e = 4 * i4 + c, o = e / (DS + 1), k = e % (DS + 1);
                if (k < DS) wt[k][o] = wv[u][c];
                else bf[o] = wv[u][c] + bias[o];  // the constant-1 column's weight + the bias
            }
        }
        for (uint32_t t0 = blockIdx.x * TPI; t0 < T; t0 += static_cast<uint32_t>(GS) * TPI) {
#pragma unroll
            for (int u = 0; u < HPT; ++u) {
                const int e = u * 256 + static_cast<int>(threadIdx.x);
                if (e < HF4) st4(&hl[0][0][0] + 4 * e, hv[u]);
            }
            __syncthreads();
            if (t0 + static_cast<uint32_t>(GS) * TPI < T) load_h(t0 + static_cast<uint32_t>(GS) * TPI, hv);  // next iteration's rows
            const uint32_t t = t0 + ti;
            const uint32_t sc = t < T ? lg_div(t, fdG) : 0u, grp = t < T ? t - sc * ngroups : 0u;
            const uint32_t n = static_cast<uint32_t>(sidx[sc]);
            const bool live = t < T && slot[n] == static_cast<int32_t>(sc);
            const uint32_t b = 16 * grp + r;
            uint32_t nb = 0;
            if (live && b < B) {
                f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
                for (int k = 0; k < DS; ++k) {
                    const float hk = hl[ti][r][k];
                    const f32x4 w = ld4(&wt[k][4 * fg]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i] = fmaf(hk, w[i], acc[i]);
                }
                f32x4 v = acc + ld4(bf + 4 * fg);
                const uint32_t kb =
                    dropout ? lg_row_stream_keep4(key, static_cast<uint64_t>(b) * N + n, 4 * fg, thr) : 0xFu;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    v[i] = ((kb >> i) & 1u) ? fmaxf(v[i], 0.f) * (dropout ? scale : 1.0f) : 0.0f;
                    nb |= static_cast<uint32_t>(v[i] > 0.f) << i;
                }
                st4(xs0 + (static_cast<size_t>(sc) * B + b) * D + 4 * fg, v);
            }
            nib[ti][r][fg] = static_cast<uint8_t>(nb);
            __syncthreads();
            if (threadIdx.x < 64 * TPI) {
                const int tj = threadIdx.x / 64, l = threadIdx.x % 64, rl = l / LPR, fl = l % LPR;
                const uint32_t tt = t0 + tj;
                const uint32_t sc2 = tt < T ? lg_div(tt, fdG) : 0u, g2 = tt < T ? tt - sc2 * ngroups : 0u;
                const uint32_t n2 = static_cast<uint32_t>(sidx[sc2]);
                if (tt < T && slot[n2] == static_cast<int32_t>(sc2)) {
                    uint32_t w = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k) w |= static_cast<uint32_t>(nib[tj][RPI * k + rl][fl]) << (4 * k);
                    bits[(static_cast<size_t>(n2) * ngroups + g2) * 64 + l] = static_cast<uint16_t>(w);
                }
            }
            __syncthreads();
        }
        return;
    }
    // non-sensor tiles: one lane of kNibTiles tiles per thread (the workgroup's 4 x kNibTiles
    // tiles, strided by 4): the tiles' slots, the bias and (with a device seed) the dropout key
    // are independent loads, all in flight before the first use.
    const uint32_t t0 = (blockIdx.x - static_cast<uint32_t>(GS)) * 4 * kNibTiles + threadIdx.x / 64;
    const int l = threadIdx.x % 64, rl = l / LPR, fg = l % LPR;
    uint32_t tn[kNibTiles], tg[kNibTiles];
    int32_t tsl[kNibTiles];
#pragma unroll
    for (int u = 0; u < kNibTiles; ++u) {
        const uint32_t t = t0 + 4 * u;
        const bool tv = t < N * ngroups;
        tn[u] = tv ? lg_div(t, fdG) : 0u;
        tg[u] = t - tn[u] * ngroups;
        tsl[u] = tv ? slot[tn[u]] : 0;
    }
    const f32x4 bv = ld4(bias + 4 * fg);
    uint32_t pos = 0;  // [relu(b) * scale > 0] of the lane's four channels
#pragma unroll
    for (int i = 0; i < 4; ++i) pos |= static_cast<uint32_t>(fmaxf(bv[i], 0.f) * (dropout ? scale : 1.0f) > 0.f) << i;
#pragma unroll
    for (int u = 0; u < kNibTiles; ++u) {
        const uint32_t t = t0 + 4 * u;
        if (t >= N * ngroups || tsl[u] >= 0) continue;  // past the end, or a sensor node's tile
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t b = 16 * tg[u] + RPI * k + rl;
            if (b < B) {
                const uint32_t kb = dropout ? lg_row_stream_keep4(key, static_cast<uint64_t>(b) * N + tn[u], 4 * fg, thr) : 0xFu;
                w |= (kb & pos) << (4 * k);
            }
        }
        bits[static_cast<size_t>(t) * 64 + l] = static_cast<uint16_t>(w);
    }
}

// x0 materialised from its compressed form (lg_node_init_expand; diagnostics and tests):
// node-major [N][B][D], a row per LPR lanes.
template <int D>
__global__ void __launch_bounds__(256)
k_node_init_expand(const int32_t* __restrict__ slot, const float* __restrict__ xs0, const uint16_t* __restrict__ bits,
                   const float* __restrict__ bias, float* __restrict__ x0, int64_t B, int64_t N, int64_t ngroups,
                   float vscale) {
    constexpr int LPR = D / 4, RPI = 64 / LPR;
    const int64_t r = static_cast<int64_t>(blockIdx.x) * (256 / LPR) + threadIdx.x / LPR;
    const int fg = threadIdx.x % LPR;
    if (r >= N * B) return;
    const int64_t n = r / B, b = r - n * B;
    f32x4 v;
    if (slot[n] >= 0) {
        v = ld4(xs0 + (static_cast<int64_t>(slot[n]) * B + b) * D + 4 * fg);
    } else {
        const int64_t grp = b / 16, rb = b % 16;
        const int k = static_cast<int>(rb) / RPI, rl = static_cast<int>(rb) % RPI;
        const uint32_t w = bits[(n * ngroups + grp) * 64 + rl * LPR + fg] >> (4 * k);
        const f32x4 bv = ld4(bias + 4 * fg);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = ((w >> i) & 1u) ? fmaxf(bv[i], 0.f) * vscale : 0.0f;
    }
    st4(x0 + r * D + 4 * fg, v);
}

// Backward of the sensor projection from the node-init pre-activation gradient dx0 (the
// layer-0 backward's output, already masked by the node init's ReLU/dropout):
//   dproj[b][s] = dx0[row(sensor_node[s], b)] * live[s]
//   dh_s[b][s][k] = sum_o dproj[b][s][o] W[o][k]                          (written)
//   slab row: dW[o][k] = sum dproj[.][o] [h_s, 1][.][k],  db[o] = sum dproj[.][o] (+ dbias_in
//   from workgroup 0: the non-sensor rows' sum the layer-0 backward already formed)
// One workgroup per kSpRows (b, s) rows, staged in LDS; every sum in a fixed order.
constexpr int kSpRows = 32;
template <int D, int DS>
__global__ void __launch_bounds__(256)
k_sensor_proj_bwd(const float* __restrict__ dx0, const int64_t* __restrict__ sidx, const float* __restrict__ live,
                  const float* __restrict__ hs, const float* __restrict__ W, const float* __restrict__ dbias_in,
                  float* __restrict__ dhs, float* __restrict__ slab, int64_t B, int64_t N, int64_t S, int nm) {
    constexpr int SL = D * (DS + 1) + D;
    __shared__ __attribute__((aligned(16))) float dp[kSpRows][D + 4];
    __shared__ __attribute__((aligned(16))) float hx[kSpRows][DS + 4];  // column DS = 1 (the bias input)
    __shared__ __attribute__((aligned(16))) float wl[D][DS];
    const int64_t K = B * S, k0 = static_cast<int64_t>(blockIdx.x) * kSpRows;
    for (int i = threadIdx.x; i < D * DS / 4; i += 256) {
        const int o = i / (DS / 4), c4 = 4 * (i % (DS / 4));
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = W[o * (DS + 1) + c4 + j];
        st4(&wl[o][c4], v);
    }
    for (int i = threadIdx.x; i < kSpRows * (D / 4); i += 256) {
        const int rr = i / (D / 4), c4 = 4 * (i % (D / 4));
        const int64_t kr = k0 + rr;
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (kr < K) {
            const int64_t b = kr / S, sc = kr - b * S, n = sidx[sc];
            const int64_t row = nm ? n * B + b : b * N + n;
            v = ld4(dx0 + row * D + c4);
            if (live) v = v * live[sc];
        }
        st4(&dp[rr][c4], v);
    }
    for (int i = threadIdx.x; i < kSpRows * (DS / 4); i += 256) {
        const int rr = i / (DS / 4), c4 = 4 * (i % (DS / 4));
        const int64_t kr = k0 + rr;
        st4(&hx[rr][c4], kr < K ? ld4(hs + kr * DS + c4) : f32x4{0.f, 0.f, 0.f, 0.f});
        if (c4 == 0) hx[rr][DS] = 1.f;
    }
    __syncthreads();
    // dh_s: thread -> (row, 4 consecutive k); the wave's lanes share o, so the W reads broadcast
    {
        constexpr int TPR = DS / 4;  // threads per row
        for (int t = threadIdx.x; t < kSpRows * TPR; t += 256) {
            const int rr = t / TPR, kc = 4 * (t % TPR);
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
            for (int o4 = 0; o4 < D / 4; ++o4) {
                const f32x4 g = ld4(&dp[rr][4 * o4]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x4 w = ld4(&wl[4 * o4 + j][kc]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i] = fmaf(g[j], w[i], acc[i]);
                }
            }
            const int64_t kr = k0 + rr;
            if (kr < K) st4(dhs + kr * DS + kc, acc);
        }
    }
    // slab: dW[o][k] over this block's rows; thread -> (o, KW consecutive k), KW independent
    // accumulator chains; the k = DS column (the constant-1 input) is db[o]
    float* out = slab + static_cast<int64_t>(blockIdx.x) * SL;
    {
        constexpr int KQ = 256 / D, KW = DS / KQ;
        const int o = threadIdx.x / KQ, kb = (threadIdx.x % KQ) * KW;
        float acc[KW];
#pragma unroll
        for (int j = 0; j < KW; ++j) acc[j] = 0.f;
        float a1 = 0.f;
        for (int rr = 0; rr < kSpRows; ++rr) {
            const float g = dp[rr][o];
#pragma unroll
            for (int j = 0; j < KW; j += 4) {
                const f32x4 hv = ld4(&hx[rr][kb + j]);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[j + i] = fmaf(g, hv[i], acc[j + i]);
            }
            a1 += g;
        }
#pragma unroll
        for (int j = 0; j < KW; ++j) out[o * (DS + 1) + kb + j] = acc[j];
        if (kb == 0) {
            out[o * (DS + 1) + DS] = a1;
            out[D * (DS + 1) + o] = a1 + ((blockIdx.x == 0 && dbias_in) ? dbias_in[o] : 0.f);
        }
    }
}

template <int D>
__global__ void __launch_bounds__(256)
k_pipe_gather(const int64_t* __restrict__ ends, const float* __restrict__ h, float* __restrict__ feat, int64_t N,
              lg_fastdiv fdP, int64_t BP) {
    constexpr int LPR = D / 4, RPB = 256 / LPR;
    const int rl = threadIdx.x / LPR, fg = threadIdx.x % LPR;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * RPB + rl; i < BP; i += static_cast<int64_t>(gridDim.x) * RPB) {
        const uint32_t b = lg_div(static_cast<uint32_t>(i), fdP), p = static_cast<uint32_t>(i) - b * fdP.d;
        const int64_t u = ends[2 * p], v = ends[2 * p + 1];
        const f32x4 hu = ld4(h + (static_cast<int64_t>(b) * N + u) * D + 4 * fg);
        const f32x4 hv = ld4(h + (static_cast<int64_t>(b) * N + v) * D + 4 * fg);
        f32x4 ad;
#pragma unroll
        for (int k = 0; k < 4; ++k) ad[k] = fabsf(hu[k] - hv[k]);
        float* f = feat + i * (3 * D) + 4 * fg;
        st4(f, hu);
        st4(f + D, hv);
        st4(f + 2 * D, ad);
    }
}

// dh[b][n] = dpool[b]/N + sum over incidences (p, role) of n, in item order, of dpipe[b][p][role]
template <int D>
__global__ void __launch_bounds__(256)
k_pipe_scatter(const int32_t* __restrict__ inc_rowptr, const int32_t* __restrict__ inc_item,
               const float* __restrict__ dpipe, const float* __restrict__ dpool, float* __restrict__ dh, int64_t N,
               lg_fastdiv fdM, int nm, int64_t P, int64_t R) {
    constexpr int LPR = D / 4, RPB = 256 / LPR;
    const int rl = threadIdx.x / LPR, fg = threadIdx.x % LPR;
    const float fN = static_cast<float>(N);
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * RPB + rl; r < R; r += static_cast<int64_t>(gridDim.x) * RPB) {
        const uint32_t hi = lg_div(static_cast<uint32_t>(r), fdM), lo = static_cast<uint32_t>(r) - hi * fdM.d;
        const int64_t b = nm ? lo : hi;
        const uint32_t n = nm ? hi : lo;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        if (dpool) {
            const f32x4 g = ld4(dpool + b * D + 4 * fg);
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[k] = g[k] / fN;
        }
        // incidences in item order, kScatterBatch items and their rows requested before
        // the first add (a node has few incidences: one round trip instead of one per item)
        constexpr int kScatterBatch = 4;
        const int32_t e0 = inc_rowptr[n], e1 = inc_rowptr[n + 1];
        for (int32_t e = e0; e < e1; e += kScatterBatch) {
            int32_t it[kScatterBatch];
#pragma unroll
            for (int u = 0; u < kScatterBatch; ++u) it[u] = e + u < e1 ? inc_item[e + u] : -1;  // 2*p + role
            f32x4 v[kScatterBatch];
#pragma unroll
            for (int u = 0; u < kScatterBatch; ++u)
                v[u] = it[u] >= 0 ? ld4(dpipe + ((b * P + (it[u] >> 1)) * 2 + (it[u] & 1)) * D + 4 * fg)
                                  : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < kScatterBatch; ++u)
                if (it[u] >= 0) acc += v[u];
        }
        st4(dh + r * D + 4 * fg, acc);
    }
}


// Weight gradient of a Linear whose input rows are [x_k, 1]:
//   slab row g: [M][N+1] block partial of dW[m][n] = sum_k dy[k][m] x[k][n], dW[m][N] = sum_k dy[k][m],
//   then [M] the same column sums (the bias gradient).  One wave per 16-row m-tile; K split
//   over blocks of kLinRows rows; v_mfma_f32_16x16x4_f32 with the column sums as an extra
//   MFMA against a constant-1 B operand.  Split-K partials are reduced in fixed order.
constexpr int kLinRows = 32;  // 8 k-steps per block: every operand load is issued before the MFMAs

template <int M, int N>
__global__ void __launch_bounds__(64 * (M / 16))
k_linear_dw(const float* __restrict__ dy, const float* __restrict__ x, int64_t K, float* __restrict__ slab) {
    constexpr int NT = N / 16, SL = M * (N + 1) + M, KS = kLinRows / 4;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const int64_t k0 = static_cast<int64_t>(blockIdx.x) * kLinRows;
    float a[KS], bv[KS][NT];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int64_t kr = k0 + 4 * ks + q;
        const bool ok = kr < K;
        const int64_t kc = ok ? kr : 0;
        a[ks] = ok ? dy[kc * M + 16 * w + j] : 0.f;  // A[m = j][k = q]
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bv[ks][nt] = ok ? x[kc * N + 16 * nt + j] : 0.f;  // B[k = q][n = j]
    }
    f32x4 acc[NT], cs = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ks], bv[ks][nt], acc[nt], 0, 0, 0);
        cs = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ks], 1.f, cs, 0, 0, 0);
    }
    float* out = slab + static_cast<int64_t>(blockIdx.x) * SL;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int m = 16 * w + 4 * q + reg;  // D layout: row 4q + reg, column j
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) out[m * (N + 1) + 16 * nt + j] = acc[nt][reg];
        if (j == 0) {
            out[m * (N + 1) + N] = cs[reg];
            out[M * (N + 1) + m] = cs[reg];
        }
    }
}

int linear_dw_grid(int64_t K) { return static_cast<int>(std::max<int64_t>(1, ceil_div(K, kLinRows))); }

inline unsigned ni_grid(int64_t rows) {
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(rows, kNiRowsPerBlock), 16LL * lg_num_cus())));
}

inline unsigned row_grid(int64_t rows, int D) {
    const int64_t rpb = 256 / (D / 4);
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(rows, rpb), 16LL * lg_num_cus())));
}

}  // namespace

extern "C" int lg_node_init_fwd(const int32_t* sensor_slot, const float* proj, const float* bias, float* x0,
                                int64_t B, int64_t N, int64_t S, int64_t D, int flags, float dropout_p,
                                uint64_t seed, uint32_t salt, lg_stream_t stream) {
    if (B < 0 || N <= 0 || S < 0) return LG_EINVAL;
    if (!sensor_slot || !bias || !x0 || (S > 0 && B > 0 && !proj)) return LG_EINVAL;
    const int dropout = (flags & LG_F_DROPOUT) ? 1 : 0;
    if (dropout && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    const int64_t R = B * N;
    if (R == 0) return LG_OK;
    if (R >= kLgMaxRows) return LG_EUNSUPPORTED;
    const int nm = (flags & LG_F_NODE_MAJOR) ? 1 : 0;
    const lg_fastdiv fdM = lg_make_fastdiv(static_cast<uint32_t>(nm ? B : N));
    const float scale = dropout ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
    switch (D) {
        case 64:
            lg_launch(k_node_init<64>, ni_grid(R), 256, 0, s, sensor_slot, proj, bias, x0, N, fdM, nm, S, R, dropout,
                                                            dropout_p, scale, seed, salt);
            break;
        case 32:
            lg_launch(k_node_init<32>, ni_grid(R), 256, 0, s, sensor_slot, proj, bias, x0, N, fdM, nm, S, R, dropout,
                                                            dropout_p, scale, seed, salt);
            break;
        default:
            return LG_EUNSUPPORTED;
    }
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_pipe_gather_fwd(const int64_t* ends, const float* h, float* feat, int64_t B, int64_t N,
                                  int64_t P, int64_t D, lg_stream_t stream) {
    if (B < 0 || N <= 0 || P < 0) return LG_EINVAL;
    const int64_t BP = B * P;
    if (BP == 0) return LG_OK;
    if (!ends || !h || !feat) return LG_EINVAL;
    if (BP >= kLgMaxRows) return LG_EUNSUPPORTED;
    const lg_fastdiv fdP = lg_make_fastdiv(static_cast<uint32_t>(P));
    hipStream_t s = lg_stream(stream);
    switch (D) {
        case 64: lg_launch(k_pipe_gather<64>, row_grid(BP, 64), 256, 0, s, ends, h, feat, N, fdP, BP); break;
        case 32: lg_launch(k_pipe_gather<32>, row_grid(BP, 32), 256, 0, s, ends, h, feat, N, fdP, BP); break;
        default: return LG_EUNSUPPORTED;
    }
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_pipe_scatter_bwd(const int32_t* inc_rowptr, const int32_t* inc_item, const float* dpipe,
                                   const float* dpool, float* dh, int64_t B, int64_t N, int64_t P, int64_t D,
                                   int flags, lg_stream_t stream) {
    if (B < 0 || N <= 0 || P < 0) return LG_EINVAL;
    const int64_t R = B * N;
    if (R == 0) return LG_OK;
    if (!inc_rowptr || !dh || (P > 0 && (!inc_item || !dpipe))) return LG_EINVAL;
    if (R >= kLgMaxRows) return LG_EUNSUPPORTED;
    const int nm = (flags & LG_F_NODE_MAJOR) ? 1 : 0;
    const lg_fastdiv fdM = lg_make_fastdiv(static_cast<uint32_t>(nm ? B : N));
    hipStream_t s = lg_stream(stream);
    switch (D) {
        case 64:
            lg_launch(k_pipe_scatter<64>, row_grid(R, 64), 256, 0, s, inc_rowptr, inc_item, dpipe, dpool, dh, N, fdM, nm, P, R);
            break;
        case 32:
            lg_launch(k_pipe_scatter<32>, row_grid(R, 32), 256, 0, s, inc_rowptr, inc_item, dpipe, dpool, dh, N, fdM, nm, P, R);
            break;
        default: return LG_EUNSUPPORTED;
    }
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_node_init_proj_fwd(const int32_t* sensor_slot, const int64_t* sensor_idx, const float* h_s,
                                     const float* W, const float* bias, float* x0, int64_t B, int64_t N, int64_t S,
                                     int64_t Ds, int64_t D, int flags, float dropout_p, uint64_t seed, uint32_t salt,
                                     lg_stream_t stream) {
    if (B < 0 || N <= 0 || S < 0) return LG_EINVAL;
    if (!sensor_slot || !W || !bias || !x0 || (S > 0 && B > 0 && (!h_s || !sensor_idx))) return LG_EINVAL;
    if (!((D == 64 && Ds == 64) || (D == 32 && Ds == 32))) return LG_EUNSUPPORTED;
    const int dropout = (flags & LG_F_DROPOUT) ? 1 : 0;
    if (dropout && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    const int64_t R = B * N;
    if (R == 0) return LG_OK;
    if (R >= kLgMaxRows) return LG_EUNSUPPORTED;
    const int nm = (flags & LG_F_NODE_MAJOR) ? 1 : 0;
    const lg_fastdiv fdM = lg_make_fastdiv(static_cast<uint32_t>(nm ? B : N));
    const float scale = dropout ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
    const int RPBD = 256 / (static_cast<int>(D) / 4);
    const int GS = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(S * B, RPBD), lg_num_cus())));
    // the first GS workgroups form the sensor rows, one workgroup per kNiRowsPerBlock rows after
    const unsigned grid = static_cast<unsigned>(GS + ceil_div(R, kNiRowsPerBlock));
    if (D == 64)
        lg_launch(k_node_init_proj<64, 64>, grid, 256, 0, s, sensor_slot, sensor_idx, h_s, W, bias, x0, B, N, fdM, nm,
                  S, R, GS, dropout, dropout_p, scale, seed, salt);
    else
        lg_launch(k_node_init_proj<32, 32>, grid, 256, 0, s, sensor_slot, sensor_idx, h_s, W, bias, x0, B, N, fdM, nm,
                  S, R, GS, dropout, dropout_p, scale, seed, salt);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_node_init_bits_fwd(const int32_t* sensor_slot, const int64_t* sensor_idx, const float* h_s,
                                     const float* W, const float* bias, float* xs0, uint16_t* x0bits, int64_t B,
                                     int64_t N, int64_t S, int64_t Ds, int64_t D, int flags, float dropout_p,
                                     uint64_t seed, uint32_t salt, lg_stream_t stream) {
    if (B < 0 || N <= 0 || S < 0) return LG_EINVAL;
    if (!sensor_slot || !W || !bias || !x0bits || (S > 0 && B > 0 && (!h_s || !sensor_idx || !xs0))) return LG_EINVAL;
    if (!((D == 64 && Ds == 64) || (D == 32 && Ds == 32))) return LG_EUNSUPPORTED;
    const int dropout = (flags & LG_F_DROPOUT) ? 1 : 0;
    if (dropout && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (B == 0) return LG_OK;
    const int64_t ngroups = (B + 15) / 16;
    if (B * N >= kLgMaxRows || N * ngroups * 64 >= kLgMaxRows) return LG_EUNSUPPORTED;
    const float scale = dropout ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
    const int64_t tpi = 256 / (16 * (D / 4));
    const int GS = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(S * ngroups, tpi), 2 * lg_num_cus())));
    const unsigned grid = static_cast<unsigned>(GS + ceil_div(N * ngroups, 4 * kNibTiles));
    const lg_fastdiv fdG = lg_make_fastdiv(static_cast<uint32_t>(ngroups));
    const uint32_t B32 = static_cast<uint32_t>(B), N32 = static_cast<uint32_t>(N), S32 = static_cast<uint32_t>(S),
                   G32 = static_cast<uint32_t>(ngroups);
    if (D == 64)
        lg_launch(k_node_init_bits<64, 64>, grid, 256, 0, s, sensor_slot, sensor_idx, h_s, W, bias, xs0, x0bits, B32, N32,
                  S32, G32, fdG, GS, dropout, dropout_p, scale, seed, salt);
    else
        lg_launch(k_node_init_bits<32, 32>, grid, 256, 0, s, sensor_slot, sensor_idx, h_s, W, bias, xs0, x0bits, B32, N32,
                  S32, G32, fdG, GS, dropout, dropout_p, scale, seed, salt);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_node_init_expand(const int32_t* sensor_slot, const float* xs0, const uint16_t* x0bits,
                                   const float* bias, float* x0, int64_t B, int64_t N, int64_t D, int flags,
                                   float dropout_p, lg_stream_t stream) {
    if (B < 0 || N <= 0 || !sensor_slot || !x0bits || !bias || !x0) return LG_EINVAL;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    const int dropout = (flags & LG_F_DROPOUT) ? 1 : 0;
    if (dropout && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (B == 0) return LG_OK;
    const int64_t ngroups = (B + 15) / 16, R = B * N, rpb = 256 / (D / 4);
    const float scale = dropout ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
    const unsigned grid = static_cast<unsigned>(ceil_div(R, rpb));
    if (D == 64)
        lg_launch(k_node_init_expand<64>, grid, 256, 0, s, sensor_slot, xs0, x0bits, bias, x0, B, N, ngroups, scale);
    else
        lg_launch(k_node_init_expand<32>, grid, 256, 0, s, sensor_slot, xs0, x0bits, bias, x0, B, N, ngroups, scale);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int64_t lg_sensor_proj_bwd_workspace_bytes(int64_t B, int64_t S, int64_t Ds, int64_t D) {
    if (B < 0 || S < 0 || !((D == 64 && Ds == 64) || (D == 32 && Ds == 32))) return LG_EUNSUPPORTED;
    const int64_t G = std::max<int64_t>(1, ceil_div(B * S, kSpRows));
    return G * (D * (Ds + 1) + D) * static_cast<int64_t>(sizeof(float));
}

extern "C" int lg_sensor_proj_bwd(const float* dx0, const int64_t* sensor_idx, const float* live, const float* h_s,
                                  const float* W, const float* dbias_in, float* dh_s, float* dW, float* db, int64_t B,
                                  int64_t N, int64_t S, int64_t Ds, int64_t D, int flags, void* workspace, int64_t ws_bytes,
                                  lg_stream_t stream) {
    if (B < 0 || N <= 0 || S < 0 || !W || !dW || !db || !workspace) return LG_EINVAL;
    if (B * S > 0 && (!dx0 || !sensor_idx || !h_s || !dh_s)) return LG_EINVAL;
    if (!((D == 64 && Ds == 64) || (D == 32 && Ds == 32))) return LG_EUNSUPPORTED;
    const int nm = (flags & LG_F_NODE_MAJOR) ? 1 : 0;
    const int G = static_cast<int>(std::max<int64_t>(1, ceil_div(B * S, kSpRows)));
    const int64_t SL = D * (Ds + 1) + D;
    if (ws_bytes < G * SL * static_cast<int64_t>(sizeof(float))) return LG_EINVAL;
    float* slab = static_cast<float*>(workspace);
    hipStream_t s = lg_stream(stream);
    // inside a reduce batch dbias_in may still be pending (the layer-0 backward's reduction
    // not yet launched): its partials are then summed into db by the batch instead of being
    // read by workgroup 0
    LgSlabSeg dbseg{D * (Ds + 1), D, db};
    if (lg_reduce_batch_pending(dbias_in, &dbseg.slab2, &dbseg.G2, &dbseg.stride2, &dbseg.off2)) dbias_in = nullptr;
    if (D == 64)
        lg_launch(k_sensor_proj_bwd<64, 64>, G, 256, 0, s, dx0, sensor_idx, live, h_s, W, dbias_in, dh_s, slab, B, N, S,
                  nm);
    else
        lg_launch(k_sensor_proj_bwd<32, 32>, G, 256, 0, s, dx0, sensor_idx, live, h_s, W, dbias_in, dh_s, slab, B, N, S,
                  nm);
    LG_RET_IF_LAUNCH_FAILED();
    const LgSlabSeg segs[2] = {{0, D * (Ds + 1), dW}, dbseg};
    return lg_launch_slab_reduce_multi(slab, G, SL, segs, 2, nullptr, nullptr, s);
}

extern "C" int64_t lg_linear_dw_workspace_bytes(int64_t K, int64_t M, int64_t N) {
    if (K < 0 || (M != 32 && M != 64) || (N != 32 && N != 64)) return LG_EUNSUPPORTED;
    return static_cast<int64_t>(linear_dw_grid(K)) * (M * (N + 1) + M) * static_cast<int64_t>(sizeof(float));
}

extern "C" int lg_linear_dw(const float* dy, const float* x, int64_t K, int64_t M, int64_t N, float* dw, float* db,
                            void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    if (K < 0 || !dw || !workspace || (K > 0 && (!dy || !x))) return LG_EINVAL;
    if ((M != 32 && M != 64) || (N != 32 && N != 64)) return LG_EUNSUPPORTED;
    hipStream_t s = lg_stream(stream);
    const int G = linear_dw_grid(K);
    float* slab = static_cast<float*>(workspace);
    const int64_t SL = M * (N + 1) + M;
    if (ws_bytes < G * SL * static_cast<int64_t>(sizeof(float))) return LG_EINVAL;
    if (K == 0) {
        if (hipMemsetAsync(slab, 0, SL * sizeof(float), s) != hipSuccess) return LG_EHIP;
    } else {
#define LG_LDW(MM, NN) lg_launch(k_linear_dw<MM, NN>, G, 64 * (MM / 16), 0, s, dy, x, K, slab)
        if (M == 64) {
            if (N == 64) LG_LDW(64, 64); else LG_LDW(64, 32);
        } else {
            if (N == 64) LG_LDW(32, 64); else LG_LDW(32, 32);
        }
#undef LG_LDW
        LG_RET_IF_LAUNCH_FAILED();
    }
    const LgSlabSeg segs[2] = {{0, M * (N + 1), dw}, {M * (N + 1), M, db}};
    return lg_launch_slab_reduce_multi(slab, G, SL, segs, 2, nullptr, nullptr, s);
}

extern "C" int lg_abi_version(void) { return 26; }

// ------------------------------------------------------------------ kernel timing
// The event pairs are process-wide (a backward op runs on autograd's worker thread, the
// timer reads the pairs back on the caller's); only the armed slot is per host thread.
// std::deque: growing it never moves the pairs already handed out.
namespace {
std::mutex g_timing_mu;
std::deque<LgTimingPair> g_timing_pool;
thread_local int t_timing_armed = -1;
}  // namespace

LgTimingPair* lg_timing_take() {
    if (t_timing_armed < 0) return nullptr;
    std::lock_guard<std::mutex> lk(g_timing_mu);
    LgTimingPair* t = &g_timing_pool[t_timing_armed];
    t_timing_armed = -1;
    return t;
}

extern "C" int lg_timing_arm(int slot) {
    if (slot < 0 || slot > (1 << 20)) return LG_EINVAL;
    {
        std::lock_guard<std::mutex> lk(g_timing_mu);
        while (static_cast<int>(g_timing_pool.size()) <= slot) {
            LgTimingPair t{};
            if (hipEventCreate(&t.start) != hipSuccess) return LG_EHIP;
            if (hipEventCreate(&t.stop) != hipSuccess) {
                (void)hipEventDestroy(t.start);
                return LG_EHIP;
            }
            g_timing_pool.push_back(t);
        }
    }
    t_timing_armed = slot;
    return LG_OK;
}

extern "C" int lg_timing_disarm(void) {
    const int was = t_timing_armed >= 0 ? 1 : 0;
    t_timing_armed = -1;
    return was;
}

extern "C" int lg_timing_elapsed(int slot, float* ms) {
    if (!ms || slot < 0) return LG_EINVAL;
    hipEvent_t a, z;
    {
        std::lock_guard<std::mutex> lk(g_timing_mu);
        if (slot >= static_cast<int>(g_timing_pool.size())) return LG_EINVAL;
        a = g_timing_pool[slot].start;
        z = g_timing_pool[slot].stop;
    }
    return hipEventElapsedTime(ms, a, z) == hipSuccess ? LG_OK : LG_EHIP;
}

extern "C" const char* lg_strerror(int code) {
    switch (code) {
        case LG_OK: return "ok";
        case LG_EINVAL: return "invalid argument";
        case LG_EUNSUPPORTED: return "unsupported feature width or flags";
        case LG_EHIP: return "HIP launch/runtime error";
        default: return "unknown error";
    }
}
