// SharedSensorGRUEncoder (reference detector.py:28-73) as two fused HIP kernels.
//
// One nn.GRU(input 1 [+9 time features], hidden H in {32, 64}, 1 layer) runs over B*S
// independent sequences (sequence q = b*S + s) of L steps; the encoder keeps h_L.
// PyTorch gate order / formulas:
//   r = sig(W_ir x + b_ir + W_hr h + b_hr)     z = sig(W_iz x + b_iz + W_hz h + b_hz)
//   n = tanh(W_in x + b_in + r * (W_hn h + b_hn))     h' = (1 - z) * n + z * h
//
// Work split: one workgroup = 16 sequences x H/16 waves; wave w owns hidden units
// [16w, 16w+16), i.e. one 16-row tile of each gate.  Gates are computed transposed,
// G^T (3H x 16 seq) = W (3H x K) [h; x]^T on v_mfma_f32_16x16x4_f32 (exact fp32).
// With the K index permuted as k = fk(ks, q) = 16*(ks>>2) + 4q + (ks&3), the
// accumulator layout of the new h IS the B-operand layout of the next step's h, so
// the recurrence stays in registers; waves swap their quarters of h through LDS once
// per step.  x = [residual, tfeat] is staged into LDS 32 steps at a time straight
// from (B, L, S) / (B, L, 9) (the (B*S, L, 10) concatenation of detector.py:62-67 is
// never built) with a constant-1 column that the backward uses for the bias sums.
//
// Training forward also stores the gate values (r, z, n, W_hn h + b_hn) per step, so
// the backward does not recompute them: its serial critical path per step is the
// elementwise gate backward, one LDS exchange and the dh MFMAs (W_hh^T fragments held
// in registers, four independent accumulator chains).  dW_hh / dW_ih / db are
// accumulated in the same loop from the exchanged dG (the MFMA pipe fills the
// recurrence's bubbles), gates and h_{t-1} are prefetched two steps ahead, and each
// workgroup writes its partial sums once to a slab reduced in fixed order
// (deterministic).
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include "common.h"

#ifndef LG_GRU_AUX
// Cache policy of the forward's h / gate stores (342 MB at B = 256, read by the backward ~0.3 ms
// and ~400 MB of other traffic later): 18 = sc1 | nt, past the Infinity Cache.  Write-back let them
// evict the trunk's and the heads' working sets from the 256 MB Infinity Cache: under sc1 | nt
// every later kernel of the step ran faster (trunk backward 48.2 -> 45.5 us, GRU backward 101.5
// -> 96.7, EdgeHead 56.1 / 130.0 -> 53.2 / 127.2) for 5 us more in this kernel; step sum 561 ->
// 552 us (r06t, same box).  nt alone took this kernel to 124 us (64-byte row pieces per store).
#define LG_GRU_AUX 18
#endif
#ifndef LG_GRU_LAUX
#define LG_GRU_LAUX 0  // cache policy of the backward's h / gate loads (lab: 2 = nt)
#endif
#include "reduce.h"
#include "split_bf16.h"

namespace {

constexpr int TS = 16;  // sequences per workgroup
constexpr int kLC = 32;  // x staging chunk (steps), forward
constexpr int kLB = 16;  // x staging chunk (steps), backward (keeps 2 workgroups/CU in LDS)

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int fk(int ks, int q) { return 16 * (ks >> 2) + 4 * q + (ks & 3); }
// Gate nonlinearities on the hardware transcendentals (v_exp_f32, v_rcp_f32, ~1 ulp each)
// instead of libm's IEEE expf / division / tanhf sequences: the recurrence's per-step
// critical path runs through them (MI355X, B = 256: GRU training forward 139 -> 116 us).
// sigma: ~3 ulp.  tanh: e^{-2|x|} form for |x| >= 1/16 (the 1 - t cancellation costs at
// most a factor 8 there, ~5e-7 relative), odd Taylor polynomial below it (truncation
// < 1e-9 relative).
__device__ __forceinline__ float sigm(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}
__device__ __forceinline__ float gru_tanh(float x) {
    const float ax = fabsf(x);
    const float t = __builtin_amdgcn_exp2f(-2.88539008177792682f * ax);  // e^{-2|x|}
    const float big = (1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t);
    const float x2 = x * x;
    const float small = ax * fmaf(x2, fmaf(x2, 0.133333333333f, -0.333333333333f), 1.0f);
    return copysignf(ax < 0.0625f ? small : big, x);
}
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// xs[tt][seq][0..15] (row stride XR) = [x_0 .. x_{I-1}, 0.., 1 (col 10), 0..] for steps
// t0 .. t0+nt-1 of the block's 16 sequences (all zero for padded sequences).  The odd
// row stride keeps the per-lane (seq, k) reads of both kernels bank-conflict free.  All
// loads are issued before the first LDS store of each batch.
constexpr int XR = 17;
template <bool UT, int PER = 8>
__device__ __forceinline__ void stage_x(float* __restrict__ xs, const float* __restrict__ resid,
                                        const float* __restrict__ tfeat, int t0, int nt, uint32_t seq0,
                                        uint32_t Nseq, int L, int S, const lg_fastdiv& fdS) {
    const int total = nt * TS * 16;
    for (int base = 0; base < total; base += blockDim.x * PER) {
        float v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = base + u * blockDim.x + threadIdx.x;
            const int tt = idx >> 8, sq = (idx >> 4) & 15, k = idx & 15;
            const uint32_t sg = seq0 + sq;
            const bool ok = idx < total && sg < Nseq;
            const uint32_t sgc = ok ? sg : 0u;
            const uint32_t b = lg_div(sgc, fdS), s = sgc - b * fdS.d;
            const int64_t row = static_cast<int64_t>(b) * L + (t0 + (ok ? tt : 0));
            float x = 0.f;
            if (k == 0) x = resid[row * S + s];
            else if (UT && k <= 9) x = tfeat[row * 9 + (k - 1)];
            else if (k == 10) x = 1.f;
            v[u] = ok ? x : 0.f;
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = base + u * blockDim.x + threadIdx.x;
            if (idx < total) xs[(idx >> 4) * XR + (idx & 15)] = v[u];
        }
    }
}

// two floats (already scaled) -> the packed hi and lo f16 parts of the f16x2 split:
// hi = v_cvt_pk_f16_f32, each lo = f16(x - hi) one v_fma_mix{lo,hi}_f16 reading hi's half
// (3 instructions a pair; the compiler's form converts hi back and subtracts: 5-7)
__device__ __forceinline__ void split2_pair_mix(float a, float b, uint32_t& p0, uint32_t& p1) {
    const lg_f32x2 v = {a, b};
    p0 = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, lg_f16x2));
    uint32_t lo;
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lo) : "v"(a), "v"(p0));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo) : "v"(b), "v"(p0));
    p1 = lo;
}

// ------------------------------------------------------------------ forward
// One wave per 16-row gate tile: 3 * H/16 waves per 16 sequences (12 at H = 64).  Wave
// (g, u), g in {r, z, n}, u = unit group: the r and z waves post sigma(.) tiles to LDS; the
// n wave u keeps W_in x + b_in and W_hn h + b_hn, forms n = tanh(.), h' = (1-z) n + z h for
// units [16u, 16u+16) (h of its own units stays in registers, fp32) and posts h' to LDS,
// from where every wave reads the next step's B operand.  Two barriers per step.
// The recurrent product W_hh h runs on v_mfma_f32_16x16x32_f16 with f16x2 split operands
// (split_bf16.h: two parts, three products, fp32-level accuracy): 6 MFMAs of 16 cycles per
// wave and step (12 on round 3's 3-way bf16 split, 16 v_mfma_f32_16x16x4_f32 of 32 before).
// The scales need no bookkeeping: W_hh's per wave (its 16 rows, all of K), h' at the fixed
// 2^14 (|h| <= 1).  W_hh is split once into registers; h' is split ONCE, by the n wave that
// produces it (4 values per lane), and posted as f16 parts.  The K order of chunk c is permuted, k = 8q + p <-> unit 16(2c + p/4) + 4q + p%4,
// so a lane's B fragment is exactly the lane's own outputs of n waves 2c and 2c+1: the
// exchange is lane-major (reader lane == writer lane), one b128 read per chunk and part.
// The x part (K = I <= 12) stays on v_mfma_f32_16x16x4_f32 (exact, off the critical path).
// Measured and dropped (MI355X, B = 256): one wave per unit group owning all three gates
// (one barrier per step, no sigma exchange) — 114 vs 116 us with fp32 MFMA; PMC
// (profiles/pmc/r02m_pmc_summary.txt): 51% of its wave time in dependency stalls.
// The node init fused into the training forward's epilogue (lg_gru_node_init_fwd, NI): the
// GRU's h_L of the block's 16 sequences (window b, sensor slot s) are the sensor rows of the
// node init (detector.py:181-190), so the block forms them right there:
//   xs0[s][b] = dropout(relu([h_L, 1] W^T + b))     for the slot's node if s is its live slot
// with the arithmetic of k_node_init_bits (heads.hip: W^T staged in LDS, the ascending-k fmaf
// chain, the same row-stream dropout), so xs0 is bit-identical to lg_node_init_bits_fwd's; and
// the NON-sensor tiles' [x0 > 0] words (the bias sign and the dropout stream alone; the sensor
// tiles' words are never read: layer 0 takes those nodes' rows from xs0) are written by extra
// workgroups past the sequence blocks (GruNi::nseqblk), which need nothing from the recurrence:
// they fill the CU slots the sequence blocks leave free (48 of 512 at B = 256) and run beside
// the serial loop instead of after it (r05d: every block's grid-strided share in the epilogue,
// the fused forward 92.8 us in the step).  Node init and its launch leave the step.
struct GruNi {
    const int32_t* slot;  // [N] node -> its live sensor slot, or -1
    const int64_t* sidx;  // [S] slot -> node
    const float* W;       // [D][H + 1] sensor_to_node.weight (D = H)
    const float* bias;    // [D]
    float* xs0;           // [S][B][D]
    uint16_t* bits;       // [N][ngroups][64]
    uint32_t B, N, ngroups;
    lg_fastdiv fdG;       // division by ngroups
    int dropout;
    float p, scale;
    uint64_t seed;
    uint32_t salt;
    uint32_t nseqblk;     // blocks [0, nseqblk) run the GRU, the rest write the bits words
};

// [x0 > 0] words of the non-sensor tiles, block `blk` of `nblk` (D = H)
template <int H>
__device__ __forceinline__ void gru_ni_bits(const GruNi& ni, uint32_t blk, uint32_t nblk) {
    constexpr int D = H, LPR = D / 4, RPI = 64 / LPR, K = 16 / RPI;
    const uint32_t key = ni.dropout ? lg_dropout_key_dev(ni.seed, ni.salt) : 0u;
    const uint32_t thr = lg_keep_threshold16(ni.p);
    const float vs = ni.dropout ? ni.scale : 1.0f;
    // one lane word per thread (blockDim.x is a multiple of 64, so a thread keeps its lane and
    // its four channels over the stride)
    const uint32_t l = threadIdx.x & 63, rl = l / LPR, fg = l % LPR;
    const f32x4 bv = ld4(ni.bias + 4 * fg);
    uint32_t pos = 0;  // [relu(b) * scale > 0] of the lane's four channels
#pragma unroll
    for (int i = 0; i < 4; ++i) pos |= static_cast<uint32_t>(fmaxf(bv[i], 0.f) * vs > 0.f) << i;
    const uint32_t words = ni.N * ni.ngroups * 64u, stride = nblk * blockDim.x;
    for (uint32_t e = blk * blockDim.x + threadIdx.x; e < words; e += stride) {
        const uint32_t t = e >> 6, n = lg_div(t, ni.fdG), gg = t - n * ni.ngroups;
        uint32_t wd = 0;  // a sensor node's tile: never read, written 0 (a deterministic output)
        if (ni.slot[n] < 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t b = 16 * gg + RPI * k + rl;
                if (b < ni.B) {
                    const uint32_t kb =
                        ni.dropout ? lg_row_stream_keep4(key, static_cast<uint64_t>(b) * ni.N + n, 4 * fg, thr) : 0xFu;
                    wd |= (kb & pos) << (4 * k);
                }
            }
        }
        ni.bits[e] = static_cast<uint16_t>(wd);
    }
}

// gates (optional) [L][Nseq][4][H]: r, z, n, W_hn h_{t-1} + b_hn
template <int H, bool UT, bool SAVE, bool NI = false>
__global__ void __launch_bounds__(12 * H) __attribute__((amdgpu_waves_per_eu(6, 8)))  // 2 workgroups / CU
k_gru_fwd(const float* __restrict__ resid, const float* __restrict__ tfeat, const float* __restrict__ Wih,
          const float* __restrict__ Whh, const float* __restrict__ bih, const float* __restrict__ bhh,
          float* __restrict__ hs, float* __restrict__ gates, float* __restrict__ hout, uint32_t Nseq, int L, int S,
          lg_fastdiv fdS, GruNi ni) {
    constexpr int NU = H / 16, NC = H / 32, I = UT ? 10 : 1;
    constexpr int LC = H == 64 ? kLC : 30;  // H = 32: four workgroups per CU fit in LDS
    if constexpr (NI) {
        if (blockIdx.x >= ni.nseqblk) {  // a bits block (uniform: before any barrier)
            gru_ni_bits<H>(ni, blockIdx.x - ni.nseqblk, gridDim.x - ni.nseqblk);
            return;
        }
    }
    __shared__ __attribute__((aligned(16))) float xs[LC * TS * XR];
    __shared__ __attribute__((aligned(16))) f32x4 grz[2][NU][64];   // [r|z][unit group][lane]: sigma tiles
    __shared__ __attribute__((aligned(16))) lg_u32x4 hbs[2][NC][64];  // h_t split parts: [part][chunk][lane]
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = w / NU, u = w % NU;  // gate (0 r, 1 z, 2 n), unit group
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const uint32_t seq0 = blockIdx.x * TS, seq = seq0 + j;
    const bool valid = seq < Nseq;

    // the h / gate stores go through buffer descriptors over one step's rows (base advanced per
    // step in SGPRs, 32-bit offsets within the step: Nseq * 4H * 4 bytes < 2^31, checked on the
    // host): 10 fewer VGPRs than 64-bit addresses.  Write-back policy (common.h kLgActAux: these
    // stores write 64-byte pieces of rows)
    const int row = g * H + 16 * u + j;  // A-operand row of this lane
    lg_f16x8 ah[NC][2];
    float hunsc;  // 2^-(sW + 14): the h product's unscale
    {
        f32x4 v[NC][2];
        float m = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                v[c][0][p] = Whh[row * H + 32 * c + 4 * q + p];
                v[c][1][p] = Whh[row * H + 32 * c + 16 + 4 * q + p];
                m = fmaxf(m, fmaxf(fabsf(v[c][0][p]), fabsf(v[c][1][p])));
            }
        }
        const int sW = lg_f16_scale_exp_c(lg_wave_max_bits(__float_as_uint(m)));
        const float sc = lg_pow2f(sW);
        hunsc = lg_pow2f(-(sW + 14));
#pragma unroll
        for (int c = 0; c < NC; ++c) split2_f16_x8(v[c][0] * sc, v[c][1] * sc, ah[c][0], ah[c][1]);
    }
    // x-side A operand; column 10 meets x's constant-1 column: the x-side bias (r, z: both
    // biases) rides in the x product, exactly (x = 1)
    float ax[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
        const int k = 4 * kx + q;
        ax[kx] = k < I ? Wih[row * I + k] : (k == 10 ? (g < 2 ? bih[row] + bhh[row] : bih[row]) : 0.f);
    }
    __shared__ __attribute__((aligned(16))) float bhn[H];  // b_hn (n waves add it to W_hn h)
    for (int i = threadIdx.x; i < H; i += blockDim.x) bhn[i] = bhh[2 * H + i];
    // NI: W^T [H][D] and W[o][H] + bias[o], staged now (their loads overlap the first x chunk's),
    // read by the epilogue
    __shared__ __attribute__((aligned(16))) float niw[NI ? H * H + H : 1];
    if constexpr (NI) {
        constexpr int D = H, NW1 = D * (H + 1), NTT = 12 * H, PER = (NW1 + NTT - 1) / NTT;
        float v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = u * NTT + static_cast<int>(threadIdx.x);
            v[u] = i < NW1 ? ni.W[i] : 0.f;
        }
        float bo[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = u * NTT + static_cast<int>(threadIdx.x);
            bo[u] = (i < NW1 && i % (H + 1) == H) ? ni.bias[i / (H + 1)] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = u * NTT + static_cast<int>(threadIdx.x);
            if (i < NW1) {
                const int o = i / (H + 1), k = i - o * (H + 1);
                if (k < H) niw[k * D + o] = v[u];
                else niw[H * D + o] = v[u] + bo[u];  // the constant-1 column's weight + the bias
            }
        }
    }
    f32x4 hcur = zero4();  // n waves: h of units 16u + 4q + reg, fp32
    if (g == 2) {  // h_{-1} = 0 (published by the first staging barrier)
        lg_u32x2* dst = reinterpret_cast<lg_u32x2*>(&hbs[0][u >> 1][lane]) + (u & 1);
#pragma unroll
        for (int p = 0; p < 2; ++p) dst[2 * NC * 64 * p] = lg_u32x2{0u, 0u};
    }

    for (int t0 = 0; t0 < L; t0 += LC) {
        const int nt = min(LC, L - t0);
        __syncthreads();
        stage_x<UT, 2>(xs, resid, tfeat, t0, nt, seq0, Nseq, L, S, fdS);
        __syncthreads();
        for (int tt = 0; tt < nt; ++tt) {
            const int t = t0 + tt;
            f32x4 a0 = zero4();  // x part
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) a0 = mfma(ax[kx], xs[(tt * TS + j) * XR + 4 * kx + q], a0);
            // h part: B fragments read just before their chunk's MFMAs (register budget of
            // two workgroups per CU)
            f32x4 hp = zero4();
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                lg_f16x8 hf[2];
#pragma unroll
                for (int p = 0; p < 2; ++p) hf[p] = __builtin_bit_cast(lg_f16x8, hbs[p][c][lane]);
                hp = mfma_f16x2(ah[c], hf, hp);
            }
            hp *= hunsc;
            if (g < 2) {
                f32x4 sg;
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) sg[reg] = sigm(a0[reg] + hp[reg]);
                grz[g][u][lane] = sg;
                // the r / z waves store their own gate (the n waves' phase between the barriers is
                // the step's critical path; it keeps the n, W_hn h + b_hn and h stores)
                if (SAVE && valid)
                    st4_act<LG_GRU_AUX>(lg_act_rsrc(gates + static_cast<int64_t>(t) * Nseq * 4 * H, static_cast<int64_t>(Nseq) * 4 * H),
                            seq * 4 * H + g * H + 16 * u + 4 * q, sg);
            }
            __syncthreads();  // (A) sigma(r), sigma(z) posted; every wave is done reading hbs
            if (g == 2) {
                hp += *reinterpret_cast<const f32x4*>(&bhn[16 * u + 4 * q]);
                const f32x4 r = grz[0][u][lane], z = grz[1][u][lane];
                f32x4 n;
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) {
                    n[reg] = gru_tanh(a0[reg] + r[reg] * hp[reg]);
                    hcur[reg] = (1.f - z[reg]) * n[reg] + z[reg] * hcur[reg];
                }
                if (valid) {
                    const int64_t rw = static_cast<int64_t>(t) * Nseq + seq;
                    (void)rw;
                    if (hs)
                        st4_act<LG_GRU_AUX>(lg_act_rsrc(hs + static_cast<int64_t>(t) * Nseq * H, static_cast<int64_t>(Nseq) * H),
                                seq * H + 16 * u + 4 * q, hcur);
                    if constexpr (SAVE) {  // r, z: stored by their waves
                        const __amdgpu_buffer_rsrc_t gr =
                            lg_act_rsrc(gates + static_cast<int64_t>(t) * Nseq * 4 * H, static_cast<int64_t>(Nseq) * 4 * H);
                        st4_act<LG_GRU_AUX>(gr, seq * 4 * H + 2 * H + 16 * u + 4 * q, n);
                        st4_act<LG_GRU_AUX>(gr, seq * 4 * H + 3 * H + 16 * u + 4 * q, hp);
                    }
                }
                const f32x4 hsc = hcur * 16384.f;  // |h| <= 1 at the fixed scale 2^14
                uint32_t a0, a1, b0, b1;
                split2_pair_mix(hsc[0], hsc[1], a0, a1);
                split2_pair_mix(hsc[2], hsc[3], b0, b1);
                lg_u32x2* dst = reinterpret_cast<lg_u32x2*>(&hbs[0][u >> 1][lane]) + (u & 1);
                dst[0] = lg_u32x2{a0, b0};
                dst[2 * NC * 64] = lg_u32x2{a1, b1};
            }
            __syncthreads();  // (B) h_t posted; sigma slots free again
        }
    }
    if (g == 2 && valid) st4(hout + static_cast<int64_t>(seq) * H + 16 * u + 4 * q, hcur);
    if constexpr (NI) {
        constexpr int D = H, LPR = D / 4, HS = H + 4;
        static_assert(TS * HS <= LC * TS * XR, "node-init staging fits the x buffer");
        float* hl = xs;             // [TS][HS] h_L of the block's sequences (fp32)
        const float* wt = niw;      // W^T [H][D] (staged at the start)
        const float* bfv = niw + H * D;  // [D] W[o][H] + bias[o]
        __syncthreads();            // the last step's reads of xs are done
        if (g == 2) st4(hl + j * HS + 16 * u + 4 * q, hcur);
        __syncthreads();
        const uint32_t key = ni.dropout ? lg_dropout_key_dev(ni.seed, ni.salt) : 0u;
        const uint32_t thr = lg_keep_threshold16(ni.p);
        const float vs = ni.dropout ? ni.scale : 1.0f;
        if (static_cast<int>(threadIdx.x) < TS * LPR) {
            const int r = threadIdx.x / LPR, fg = threadIdx.x % LPR;
            const uint32_t sq = seq0 + r;
            if (sq < Nseq) {
                const uint32_t b = lg_div(sq, fdS), sl = sq - b * fdS.d;
                const uint32_t n = static_cast<uint32_t>(ni.sidx[sl]);
                if (ni.slot[n] == static_cast<int32_t>(sl)) {
                    f32x4 acc = zero4();
#pragma unroll 8
                    for (int k = 0; k < H; ++k) {
                        const float hk = hl[r * HS + k];
                        const f32x4 w = ld4(wt + k * D + 4 * fg);
#pragma unroll
                        for (int i = 0; i < 4; ++i) acc[i] = fmaf(hk, w[i], acc[i]);
                    }
                    f32x4 v = acc + ld4(bfv + 4 * fg);
                    const uint32_t kb =
                        ni.dropout ? lg_row_stream_keep4(key, static_cast<uint64_t>(b) * ni.N + n, 4 * fg, thr) : 0xFu;
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[i] = ((kb >> i) & 1u) ? fmaxf(v[i], 0.f) * vs : 0.0f;
                    st4(ni.xs0 + (static_cast<size_t>(sl) * ni.B + b) * D + 4 * fg, v);
                }
            }
        }
    }
}

// ------------------------------------------------------------------ backward
// slab layout per workgroup: [dWhh 3H*H][dWih 3H*I][dbih 3H][dbhh 3H]
template <int H>
struct GB {
    static constexpr int NW = H / 16;
    static constexpr int RW = 16 * NW;     // dG floats per lane row: 4 gates x NW waves x 4 regs
    static constexpr int DS = RW + 4;      // dg row stride (16 B aligned rows)
    static constexpr int HS = H + 16;      // h tile row stride (== 16 mod 64: conflict-free B' reads)
    static constexpr int KG = 3 * H / 4;   // k-steps of the dh contraction (3H gate rows)
};

// Physical column of logical dG column c in the row of lane `src`: a 16-float rotation by
// (src >> 4) keeps the cross-lane dW operand reads bank-conflict free.
template <int H>
__device__ __forceinline__ int dg_col(int src, int c) {
    return (c + 16 * ((src >> 4) & 3)) & (GB<H>::RW - 1);
}

template <int H, bool UT, bool NEED_DX>
__global__ void __launch_bounds__(4 * H)
k_gru_bwd(const float* __restrict__ resid, const float* __restrict__ tfeat, const float* __restrict__ Wih,
          const float* __restrict__ Whh, const float* __restrict__ hs, const float* __restrict__ gates,
          const float* __restrict__ dhL, float* __restrict__ dx, float* __restrict__ slab, uint32_t Nseq, int L,
          int S, lg_fastdiv fdS) {
    using G = GB<H>;
    constexpr int NW = G::NW, I = UT ? 10 : 1, G3 = 3 * H;
    constexpr int SLAB = G3 * H + G3 * I + 2 * G3;
    constexpr int NTH = 64 * NW;
    __shared__ __attribute__((aligned(16))) float xs[kLB * TS * XR];
    __shared__ __attribute__((aligned(16))) float hl[3][TS * G::HS];
    __shared__ __attribute__((aligned(16))) float dg[2][64 * G::DS];
    __shared__ __attribute__((aligned(16))) float wih[NEED_DX ? G3 * 16 : 1];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const uint32_t seq0 = blockIdx.x * TS, seq = seq0 + j;
    const bool valid = seq < Nseq;
    const uint32_t seqc = valid ? seq : 0u;

    if constexpr (NEED_DX) {
        for (int i = threadIdx.x; i < G3 * 16; i += NTH) wih[i] = (i % 16) < I ? Wih[(i / 16) * I + (i % 16)] : 0.f;
    }
    // W_hh^T fragments: A[row j = unit 16w + j][k = gate row fk(ks, q)]
    float at[G::KG];
#pragma unroll
    for (int ks = 0; ks < G::KG; ++ks) at[ks] = Whh[fk(ks, q) * H + 16 * w + j];

    // h_{t-1} tile rows: thread -> (row = seq, float4 column)
    const int hrow = threadIdx.x / (H / 4), hc4 = threadIdx.x % (H / 4);
    const uint32_t hseq = seq0 + hrow;
    const bool hvalid = hseq < Nseq;
    auto load_h = [&](int t) -> f32x4 {  // h_t row of this thread (zero for t < 0 / padded)
        if (t < 0) return zero4();
        const f32x4 v = ld4(hs + (static_cast<int64_t>(t) * Nseq + (hvalid ? hseq : 0u)) * H + 4 * hc4);
        return hvalid ? v : zero4();
    };
    auto load_g = [&](int t, f32x4 (&g)[4]) {  // gates of step t for this lane's 4 units
        const float* p = gates + (static_cast<int64_t>(t) * Nseq + seqc) * 4 * H + 16 * w + 4 * q;
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] = valid ? ld4(p + k * H) : zero4();
    };

    f32x4 dh = valid ? ld4(dhL + static_cast<int64_t>(seq) * H + 16 * w + 4 * q) : zero4();
    f32x4 dwh[3][NW], dwx[3], dbhn = zero4();
#pragma unroll
    for (int gi = 0; gi < 3; ++gi) {
        dwx[gi] = zero4();
#pragma unroll
        for (int nt = 0; nt < NW; ++nt) dwh[gi][nt] = zero4();
    }

    // prologue: hl for step L-1 (= h_{L-2}), prefetch h_{L-3}, h_{L-4}; gates of L-1, L-2
    f32x4 g_cur[4], g_n1[4];
    load_g(L - 1, g_cur);
    if (L >= 2) load_g(L - 2, g_n1);
    f32x4 h_n1 = load_h(L - 3), h_n2 = load_h(L - 4);
    st4(&hl[(L - 1) % 3][hrow * G::HS + 4 * hc4], load_h(L - 2));

    for (int t = L - 1; t >= 0; --t) {
        if (t == L - 1 || t % kLB == kLB - 1) {  // stage the x chunk containing t (descending)
            const int t0 = t - t % kLB;
            __syncthreads();
            stage_x<UT>(xs, resid, tfeat, t0, min(kLB, L - t0), seq0, Nseq, L, S, fdS);
        }
        const int tt = t % kLB;
        // One barrier per step (below).  hl[t%3] and this step's x were published by the
        // previous step's barrier (or the staging barrier); hl[(t-1)%3] and dg[t&1] were
        // last read two steps ago, which every wave finished before that barrier.
        // (b) h tile for step t-1 (= h_{t-2}) into the buffer nobody can be reading
        if (t >= 1) st4(&hl[(t - 1) % 3][hrow * G::HS + 4 * hc4], h_n1);
        // (a) elementwise gate backward for this lane's 4 units
        const f32x4 hp = ld4(&hl[t % 3][j * G::HS + 16 * w + 4 * q]);
        const f32x4 r = g_cur[0], z = g_cur[1], n = g_cur[2], hnp = g_cur[3];
        f32x4 gr, gz, ghn, gin, dhp;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const float d = dh[reg];
            const float dn = d * (1.f - z[reg]);
            const float dzv = d * (hp[reg] - n[reg]);
            dhp[reg] = d * z[reg];
            const float dnp = dn * (1.f - n[reg] * n[reg]);
            gin[reg] = dnp;
            ghn[reg] = dnp * r[reg];
            gr[reg] = dnp * hnp[reg] * r[reg] * (1.f - r[reg]);
            gz[reg] = dzv * z[reg] * (1.f - z[reg]);
        }
        dbhn += ghn;
        float* dgb = dg[t & 1];
        st4(&dgb[lane * G::DS + dg_col<H>(lane, 4 * (0 * NW + w))], gr);
        st4(&dgb[lane * G::DS + dg_col<H>(lane, 4 * (1 * NW + w))], gz);
        st4(&dgb[lane * G::DS + dg_col<H>(lane, 4 * (2 * NW + w))], ghn);
        st4(&dgb[lane * G::DS + dg_col<H>(lane, 4 * (3 * NW + w))], gin);
        // prefetch: gates of t-2, h_{t-4} (consumed two iterations from now)
#pragma unroll
        for (int k = 0; k < 4; ++k) g_cur[k] = g_n1[k];
        if (t >= 2) load_g(t - 2, g_n1);
        h_n1 = h_n2;
        h_n2 = load_h(t - 4);
        __syncthreads();  // dG of all waves visible

        // dh_{t-1}[c] = dh z + sum_g W_hh[g][c] dG_h[g]   (4 independent chains)
        f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
        for (int a = 0; a < G::KG / 4; ++a) {
            const f32x4 bv = ld4(&dgb[lane * G::DS + dg_col<H>(lane, 4 * a)]);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = mfma(at[4 * a + i], bv[i], acc[i]);
        }
        dh = dhp + ((acc[0] + acc[1]) + (acc[2] + acc[3]));

        // dW over this step's 16 sequences: A'[unit j][seq 4ks + q] from the exchanged dG
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int src = (4 * ks + q) + 16 * (j >> 2);
            const float* row = &dgb[src * G::DS];
            const float a0 = row[dg_col<H>(src, 4 * (0 * NW + w) + (j & 3))];
            const float a1 = row[dg_col<H>(src, 4 * (1 * NW + w) + (j & 3))];
            const float a2 = row[dg_col<H>(src, 4 * (2 * NW + w) + (j & 3))];
            const float a3 = row[dg_col<H>(src, 4 * (3 * NW + w) + (j & 3))];
            const float* hrow_p = &hl[t % 3][(4 * ks + q) * G::HS];
#pragma unroll
            for (int nt = 0; nt < NW; ++nt) {
                const float hb = hrow_p[16 * nt + j];
                dwh[0][nt] = mfma(a0, hb, dwh[0][nt]);
                dwh[1][nt] = mfma(a1, hb, dwh[1][nt]);
                dwh[2][nt] = mfma(a2, hb, dwh[2][nt]);
            }
            const float xb = xs[(tt * TS + 4 * ks + q) * XR + j];
            dwx[0] = mfma(a0, xb, dwx[0]);
            dwx[1] = mfma(a1, xb, dwx[1]);
            dwx[2] = mfma(a3, xb, dwx[2]);
        }
        if (NEED_DX && w == 0) {
            // dx^T[k][seq] = sum_g W_ih[g][k] dG_i[g][seq]   (gates r, z, in; k = 4q + reg < I)
            f32x4 dxa = zero4();
#pragma unroll
            for (int ks = 0; ks < G::KG; ++ks) {
                const int c = ks < 2 * 4 * NW ? ks : ks + 4 * NW;  // skip the hn block
                dxa = mfma(wih[fk(ks, q) * 16 + j], dgb[lane * G::DS + dg_col<H>(lane, c)], dxa);
            }
            if (valid) {
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) {
                    const int k = 4 * q + reg;
                    if (k < I) dx[(static_cast<int64_t>(seq) * L + t) * I + k] = dxa[reg];
                }
            }
        }
    }

    // per-workgroup slab: waves own disjoint gate rows
    float* out = slab + static_cast<int64_t>(blockIdx.x) * SLAB;
    float* oWhh = out;
    float* oWih = out + G3 * H;
    float* obih = oWih + G3 * I;
    float* obhh = obih + G3;
#pragma unroll
    for (int gi = 0; gi < 3; ++gi)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int g = gi * H + 16 * w + 4 * q + reg;
#pragma unroll
            for (int nt = 0; nt < NW; ++nt) oWhh[g * H + 16 * nt + j] = dwh[gi][nt][reg];
            if (j < I) oWih[g * I + j] = dwx[gi][reg];
            if (j == 10) obih[g] = dwx[gi][reg];             // constant-1 column: sum of dG_i
            if (j == 10 && gi < 2) obhh[g] = dwx[gi][reg];   // r, z: dG_h == dG_i
        }
    // db_hh(n) = sum over sequences of dG_hn: fold the 16 sequence lanes of each row
#pragma unroll
    for (int off = 1; off < 16; off <<= 1)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) dbhn[reg] += __shfl_xor(dbhn[reg], off);
    if (j == 0) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) obhh[2 * H + 16 * w + 4 * q + reg] = dbhn[reg];
    }
}

// ------------------------------------------------------------------ backward, split MFMA
// The training step's backward (no dx: the residual is data).  One workgroup = 32
// sequences x 2 H/16 waves: wave (w, s) owns hidden units [16w, 16w+16) of sequences
// [16s, 16s+16).  Per step t (descending), one barrier:
//   1. elementwise gate backward for the lane's 4 units (gates, h_{t-1} and x_t prefetched
//      two steps ahead from global); dG = (dG_r, dG_z, dG_hn, dG_in), h_{t-1} and x_t are
//      split (below) and posted row-major [seq][column] to a double-buffered LDS image
//   2. dh_{t-1} = d z + W_hh^T dG_h on 16x16x32 MFMAs (K = the 3H gate rows read straight
//      from the [seq][rho] rows: one b128 per chunk and part), W_hh^T split once into
//      registers
//   3. dW_hh += dG_h^T h_{t-1} and dW_ih += dG_i^T x_t over the 32 sequences (K = 32: one
//      16x16x32 per tile and product); both operands come from the row-major images through
//      ds_read_b64_tr_b16 (transposing 4 x 16 blocks), wave (w, s) owning the dW_hh column
//      tiles of its half
//
// Two splits of the fp32 operands, both at fp32-level accuracy:
//  - F16 (default): the f16x2 transform (split_bf16.h: 2 parts, 3 products per operand pair),
//    with power-of-two scales that are uniform along every MFMA's K: W_hh^T per wave (the
//    wave's unit rows), h_{t-1} fixed at 2^14 (|h| <= 1), x_t and dG_t one scale per step for
//    the whole workgroup.  A workgroup-wide scale needs a bound on the step's largest |dG|
//    before any wave has computed it, and a second barrier per step would cost what the
//    halved MFMAs save; the bound comes from the previous step instead.  With d = dh_t,
//      |dG_in|, |dG_hn| <= |d|,  |dG_z| <= |d| / 2,  |dG_r| <= |d| |W_hn h + b_hn| / 4
//    (r, z, n, h in [0, 1] / [-1, 1]), and dh_t = z dh_{t+1} + W_hh^T dG_h,t+1, so
//      max |dG_t| <= (max |dh_{t+1}| + |W_hh^T|_inf max |dG_h,t+1|) max(1, max |hn_t| / 4)
//    and, as hn = W_hn h + b_hn with |h| <= 1, max |hn_t| <= max |hn_{L-1}| + 2 H max |W_hn|
//    for every t (one factor per launch).  Each step posts max |dh| and max |dG_h| into a
//    3-slot LDS ring (ds_max over the four row leaders of each wave); the following step reads
//    them after the barrier.  x is data: its scale is the workgroup's max |x| over all steps,
//    scanned once before the loop.  The
//    bound only ever overshoots, which f16x2 tolerates (block max placed at [2^14, 2^15):
//    values down to 2^-17 of it keep both parts normal).  A scale is kept while the bound
//    stays within 2^6 of it, so the dW accumulators (in units of the product scale) are
//    rescaled only when it moves; they are unscaled once at the end.
//  - 3-way bf16 (LG_KERNEL_LAB builds, LG_LAB_GRU_BF16X3=1, for A/B runs): six products
//    per operand pair, no scales.
// MFMA cycles per wave and step: 18 x 16 (dh) + 18-24 x 16 (dW) on the f16x2 split against
// 36 x 16 + 36-48 x 16 on the 3-way bf16 split and 108 x 32 for the fp32
// v_mfma_f32_16x16x4_f32 kernel above, which stays for the dx variant.
constexpr int TS2 = 32;  // sequences per workgroup
template <int H>
struct GB2 {
    static constexpr int NW = H / 16;         // unit groups
    static constexpr int NWAVE = 2 * NW;      // x 2 sequence halves
    static constexpr int NTH = 64 * NWAVE;
    static constexpr int DGS = 4 * H + 16;    // dG row (16-bit): [r | z | hn | in], 8 dwords mod 64: conflict-free
    static constexpr int HLS = H + 16;        // h row (16-bit)
    static constexpr int XLS = 16;            // x row (16-bit): 16 columns (I <= 10, col 10 = 1)
    static constexpr int NCH = 3 * H / 32;    // dh contraction chunks
    static constexpr int NTS = NW / 2;        // dW_hh column tiles per wave
};
constexpr int kGruKeep = 6;  // f16x2: a step scale is kept while the new bound is within 2^6 of it

[[maybe_unused]] __device__ __forceinline__ void split3_1(float x, uint16_t& p0, uint16_t& p1, uint16_t& p2) {
    const uint32_t a = pk_bf16(x, 0.f);
    const float r = x - bf_lo(a);
    const uint32_t b = pk_bf16(r, 0.f);
    const uint32_t c = pk_bf16(r - bf_lo(b), 0.f);
    p0 = static_cast<uint16_t>(a);
    p1 = static_cast<uint16_t>(b);
    p2 = static_cast<uint16_t>(c);
}
// one float -> the two f16 parts of the f16x2 split (already scaled)
__device__ __forceinline__ void split2_1(float x, uint16_t& p0, uint16_t& p1) {
    const _Float16 h = static_cast<_Float16>(x);
    p0 = __builtin_bit_cast(uint16_t, h);
    p1 = __builtin_bit_cast(uint16_t, static_cast<_Float16>(x - static_cast<float>(h)));
}
// max of a non-negative float's bits over each row of 16 lanes (every lane of the row; every
// source lane of these patterns exists, so bound_ctrl only lets the move fold into the max)
__device__ __forceinline__ uint32_t gru_row_max_bits(uint32_t m) {
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0xB1, 0xF, 0xF, true)));  // xor 1
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x4E, 0xF, 0xF, true)));  // xor 2
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x124, 0xF, 0xF, true)));  // row_ror 4
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x128, 0xF, 0xF, true)));  // row_ror 8
    return m;
}
// ds_max_u32 on an LDS word from the lanes that call it.  The offset is hidden from the
// compiler so that its atomic optimizer does not wrap a (provably) uniform address in a
// readlane loop over the active lanes (~30 instructions per atomic).
__device__ __forceinline__ void lds_max_u32(uint32_t* p, uint32_t v) {
    int off = 0;
    asm volatile("" : "+v"(off));
    atomicMax(p + off, v);
}
__device__ __forceinline__ float absmax4(const f32x4& v) {
    return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
}

#ifdef LG_NM3_STAMPS
// kernel-lab timeline (stamps builds only): per wave, for steps t = kGruStampT0 .. +7, clock at
// the step's start, before its barrier, after it, once dh is formed, once the gate backward is
// done (its loads waited for), after the LDS image and the refill are issued
constexpr int kGruStampT0 = 20, kGruStamps = 48;
__device__ uint64_t g_gru_stamps[256 * 8 * kGruStamps];
#define LG_GRU_STAMP(t, k)                                                                                 \
    do {                                                                                                   \
        const int st_ = kGruStampT0 + 7 - (t);                                                             \
        if (lane == 0 && st_ >= 0 && st_ < 8 && blockIdx.x < 256)                                          \
            g_gru_stamps[(static_cast<size_t>(blockIdx.x) * 8 + wid) * kGruStamps + 6 * st_ + (k)] =       \
                __builtin_amdgcn_s_memtime();                                                              \
    } while (0)
#else
#define LG_GRU_STAMP(t, k) \
    do {                   \
    } while (0)
#endif

// The sensor projection's backward fused into the training backward (lg_gru_node_init_bwd, NI;
// the arithmetic of k_sensor_proj_bwd, heads.hip, with the same 32-row groups, so every value
// is bit-identical to lg_sensor_proj_bwd's):
//   prologue: dh_L of the lane's sequence (window b, slot s) = dproj W[:, :H], dproj = the
//             layer-0 backward's dx at node sidx[s], row b (already masked by the node init's
//             ReLU / dropout), times live[s]; W staged in the dG image before its first use;
//   epilogue: the workgroup's slab row of dW (D x (H + 1): [h_L, 1] columns) and db, after the
//             GRU's own slab row.
struct GruNiB {
    const float* dx0;     // node-major [N][B][D] (the sensor nodes' rows)
    const int64_t* sidx;  // [S] slot -> node
    const float* live;    // [S] 1 / 0, or null (every slot live)
    const float* W;       // [D][H + 1]
    const float* dbias_in;  // [D] added to db by workgroup 0 (the non-sensor rows' sum), or null
    uint32_t B;
};

template <int H, bool UT, bool F16, bool DEFER, bool NI = false>
__global__ void __launch_bounds__(GB2<H>::NTH)
k_gru_bwd2(const float* __restrict__ resid, const float* __restrict__ tfeat, const float* __restrict__ Whh,
           const float* __restrict__ hs, const float* __restrict__ gates, const float* __restrict__ dhL,
           float* __restrict__ slab, uint32_t Nseq, int L, int S, lg_fastdiv fdS, GruNiB ni) {
    using G = GB2<H>;
    using AF = std::conditional_t<F16, lg_f16x8, lg_bf16x8>;
    constexpr int NP = F16 ? 2 : 3;  // split parts
    constexpr int I = UT ? 10 : 1, G3 = 3 * H;
    constexpr int SLAB = G3 * H + G3 * I + 2 * G3;
    constexpr int XPT = TS2 * 16 / G::NTH;  // x values staged per thread and step
    __shared__ __attribute__((aligned(16))) uint16_t dgs[2][NP][TS2][G::DGS];
    __shared__ __attribute__((aligned(16))) uint16_t hls[2][NP][TS2][G::HLS];
    __shared__ __attribute__((aligned(16))) uint16_t xls[2][NP][TS2][G::XLS];
    __shared__ __attribute__((aligned(16))) float dbh[H];
    // F16: per-step maxima (float bits) {max |dh|, max |dG_h|}, ring of 3 (written at step t,
    // read at t-1, cleared at t-2); |W_hh^T|_inf, max |W_hn|, max |hn_{L-1}|, max |x|
    __shared__ __attribute__((aligned(8))) uint32_t gmx[3][2];
    __shared__ uint32_t wnm[4];
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = wid % G::NW, sh = wid / G::NW;
    const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const int sl = 16 * sh + j;  // local sequence of this lane (elementwise, dh)
    const uint32_t seq0 = blockIdx.x * TS2, seq = seq0 + sl;
    const bool valid = seq < Nseq;
    const int u0 = 16 * w + 4 * q;  // this lane's 4 units

    auto frag_row = [](const uint16_t* p) { return __builtin_bit_cast(AF, lds_frag_row(p)); };
    auto frag_tr = [](const uint16_t* r0, const uint16_t* r1) {
        return __builtin_bit_cast(AF, lds_frag_tr16(r0, r1));
    };
    auto mm = [](const AF (&a)[NP], const AF (&b)[NP], f32x4 c) {
        if constexpr (F16) return mfma_f16x2(a, b, c);
        else return mfma_split(a, b, c);
    };
    // value -> its NP 16-bit parts (F16: already scaled)
    auto split_x4 = [](const f32x4& v, lg_u32x2 (&f)[NP]) {
        if constexpr (F16) {
            uint32_t a0, a1, b0, b1;
            split2_pair_mix(v[0], v[1], a0, a1);
            split2_pair_mix(v[2], v[3], b0, b1);
            f[0] = lg_u32x2{a0, b0};
            f[1] = lg_u32x2{a1, b1};
        } else {
            split3_x4(v, f[0], f[1], f[2]);
        }
    };

    // W_hh^T A fragments: row = unit 16w + j, k = gate row 32c + 8q + p
    AF adh[G::NCH][NP];
    float sWinv = 1.f;  // F16: 2^-sW, the wave's W_hh^T scale
    {
        f32x4 wv[G::NCH][2];
#pragma unroll
        for (int c = 0; c < G::NCH; ++c)
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                wv[c][0][p] = Whh[(32 * c + 8 * q + p) * H + 16 * w + j];
                wv[c][1][p] = Whh[(32 * c + 8 * q + 4 + p) * H + 16 * w + j];
            }
        if constexpr (F16) {
            // max |W| of the wave, of its W_hn rows, |W| sum of column 16w + j (this lane's rows)
            float m = 0.f, mn = 0.f, cs = 0.f;
#pragma unroll
            for (int c = 0; c < G::NCH; ++c) {
                m = fmaxf(m, fmaxf(absmax4(wv[c][0]), absmax4(wv[c][1])));
                if (32 * c >= 2 * H) mn = fmaxf(mn, fmaxf(absmax4(wv[c][0]), absmax4(wv[c][1])));
#pragma unroll
                for (int p = 0; p < 4; ++p) cs += fabsf(wv[c][0][p]) + fabsf(wv[c][1][p]);
            }
            cs += __shfl_xor(cs, 16);
            cs += __shfl_xor(cs, 32);
            const int sW = lg_f16_scale_exp_c(lg_wave_max_bits(__float_as_uint(m)));
            const float sc = lg_pow2f(sW);
            sWinv = lg_pow2f(-sW);
#pragma unroll
            for (int c = 0; c < G::NCH; ++c) split2_f16_x8(wv[c][0] * sc, wv[c][1] * sc, adh[c][0], adh[c][1]);
            if (threadIdx.x < 6) (&gmx[0][0])[threadIdx.x] = 0u;
            if (threadIdx.x < 4) wnm[threadIdx.x] = 0u;
            __syncthreads();
            const uint32_t cm = gru_row_max_bits(__float_as_uint(cs)), nm = gru_row_max_bits(__float_as_uint(mn));
            if (j == 0) {
                lds_max_u32(&wnm[0], cm);
                lds_max_u32(&wnm[1], nm);
            }
        } else {
#pragma unroll
            for (int c = 0; c < G::NCH; ++c) split3_x8(wv[c][0], wv[c][1], adh[c][0], adh[c][1], adh[c][2]);
        }
    }

    // Prefetch loads are unconditional and raw: addresses clamped in range (a padded
    // sequence's x is the last sequence's, its gates and h read 0, t < 0 reads step 0) and nothing selected on the loaded
    // value until it is consumed — a load under a divergent branch, or a select on its
    // result, makes the compiler wait for it (vmcnt) in the iteration that issued it, which
    // serialises the two-step prefetch.  A padded sequence needs no masking: its dh is zero,
    // every dG term is proportional to dh, and its h / x rows only ever multiply its own dG
    // (its gates read as 0 leave the F16 bounds alone; its x lies in the scanned windows, so it
    // cannot overflow the x scale and make 0 x inf).
    // gates / h through buffer loads: the base (step t, the workgroup's first sequence) is
    // scalar, the lane's offset fixed, and a padded sequence's rows lie past the resource's
    // end (read as 0)
    const int nsq = static_cast<int>(min(Nseq - seq0, static_cast<uint32_t>(TS2)));
    auto load_g = [&](int t, f32x4 (&g)[4]) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(gates + (static_cast<int64_t>(max(t, 0)) * Nseq + seq0) * 4 * H), static_cast<short>(0),
            nsq * 4 * H * 4, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            g[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (sl * 4 * H + u0 + k * H) * 4, 0, LG_GRU_LAUX));
    };
    auto load_h = [&](int t) -> f32x4 {  // h_t of this lane's units (h_0 for t < 0: masked at use)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(hs + (static_cast<int64_t>(max(t, 0)) * Nseq + seq0) * H), static_cast<short>(0),
            nsq * H * 4, 0x00020000);
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (sl * H + u0) * 4, 0, LG_GRU_LAUX));
    };
    // x value i of this thread: step 0's element and the per-step stride (hoisted out of the loop)
    const float* xp0[XPT];
    int xst[XPT];
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
        const int e = threadIdx.x + i * G::NTH, xs = e >> 4, k = e & 15;
        const uint32_t sg = seq0 + xs;
        const uint32_t sgc = sg < Nseq ? sg : Nseq - 1;  // the last sequence's x: inside the F16 x scan
        const uint32_t b = lg_div(sgc, fdS), s = sgc - b * fdS.d;
        const int64_t row0 = static_cast<int64_t>(b) * L;
        const bool from_t = UT && k >= 1 && k <= 9;
        xp0[i] = from_t ? tfeat + row0 * 9 + (k - 1) : resid + row0 * S + s;
        xst[i] = from_t ? 9 : S;
    }
    auto load_x = [&](int t, float (&x)[XPT]) {  // raw residual / tfeat value (see x_val)
#pragma unroll
        for (int i = 0; i < XPT; ++i) x[i] = xp0[i][static_cast<int64_t>(max(t, 0)) * xst[i]];
    };
    auto x_val = [&](int i, float raw) {  // x row column k: residual, tfeat, the constant 1, 0
        const int k = (threadIdx.x + i * G::NTH) & 15;
        return (k == 0 || (UT && k >= 1 && k <= 9)) ? raw : (k == 10 ? 1.f : 0.f);
    };
    // F16: post this wave's maxima into ring slot `slot` (the four row leaders, ds_max)
    auto post = [&](int slot, float md, float mg) {
        const uint32_t a = gru_row_max_bits(__float_as_uint(md)), b = gru_row_max_bits(__float_as_uint(mg));
        if (j == 0) {
            lds_max_u32(&gmx[slot][0], a);
            lds_max_u32(&gmx[slot][1], b);
        }
    };
    if constexpr (F16) {
        // the x scale: max |x| over every step of the workgroup's windows (a superset of its
        // sequences' values, contiguous in memory: coalesced, all loads of a round in flight)
        const uint32_t b0 = lg_div(seq0, fdS), b1 = lg_div(min(seq0 + TS2, Nseq) - 1, fdS);
        float m = 1.f;  // the constant-1 column
        auto scan = [&](const float* base, int64_t n) {
            for (int64_t i0 = threadIdx.x; i0 < n; i0 += 8 * G::NTH)
#pragma unroll
                for (int u = 0; u < 8; ++u) m = fmaxf(m, fabsf(base[min(i0 + u * G::NTH, n - 1)]));
        };
        const int64_t nb = static_cast<int64_t>(b1 - b0 + 1) * L;
        scan(resid + static_cast<int64_t>(b0) * L * S, nb * S);
        if (UT) scan(tfeat + static_cast<int64_t>(b0) * L * 9, nb * 9);
        const uint32_t xm = gru_row_max_bits(__float_as_uint(m));
        if (j == 0) lds_max_u32(&wnm[3], xm);
    }

    f32x4 dh = zero4();
    if constexpr (NI) {
        // W[:, :H] as [D][H] and the block's 32 dproj rows (times live) in the dG image, which is
        // unused until step L-1; every load of both in flight at once (coalesced)
        constexpr int D = H, DP = D + 4;
        float* wl = reinterpret_cast<float*>(&dgs[0][0][0][0]);
        float* dpl = wl + D * H;  // [TS2][DP]
        static_assert(sizeof(dgs) >= sizeof(float) * (D * H + TS2 * DP), "staging fits the dG image");
        static_assert((D * H) % G::NTH == 0, "W staging: whole rounds");
        {
            constexpr int PER = D * H / G::NTH;
            float v[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {  // every load in flight before the first store
                const int i = u * G::NTH + static_cast<int>(threadIdx.x), o = i / H, k = i - o * H;
                v[u] = ni.W[o * (H + 1) + k];
            }
#pragma unroll
            for (int u = 0; u < PER; ++u) wl[u * G::NTH + threadIdx.x] = v[u];
        }
        for (int i = threadIdx.x; i < TS2 * (D / 4); i += G::NTH) {
            const int rr = i / (D / 4), c4 = 4 * (i % (D / 4));
            const uint32_t sq = seq0 + rr;
            f32x4 v = zero4();
            if (sq < Nseq) {
                const uint32_t b = lg_div(sq, fdS), sl2 = sq - b * fdS.d;
                v = ld4(ni.dx0 + (static_cast<int64_t>(ni.sidx[sl2]) * ni.B + b) * D + c4);
                if (ni.live) v = v * ni.live[sl2];
            }
            st4(dpl + rr * DP + c4, v);
        }
        __syncthreads();
#pragma unroll 4
        for (int o4 = 0; o4 < D / 4; ++o4) {
            const f32x4 gz = ld4(dpl + sl * DP + 4 * o4);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const f32x4 wv = ld4(wl + (4 * o4 + jj) * H + u0);
#pragma unroll
                for (int i = 0; i < 4; ++i) dh[i] = fmaf(gz[jj], wv[i], dh[i]);
            }
        }
        if (!valid) dh = zero4();
        __syncthreads();  // the staging area is the dG image of step L-1
    } else {
        dh = valid ? ld4(dhL + static_cast<int64_t>(seq) * H + u0) : zero4();
    }
    f32x4 dwh[3][G::NTS], dwx[2], dbhn = zero4();
#pragma unroll
    for (int gi = 0; gi < 3; ++gi)
#pragma unroll
        for (int n = 0; n < G::NTS; ++n) dwh[gi][n] = zero4();
    dwx[0] = dwx[1] = zero4();

    // Two prefetch slots (steps of one parity each), each consumed and refilled with the
    // step two earlier by the same unrolled copy of the step: no register rotation, whose
    // moves would wait for the loads just issued.
    // Issued slot by slot in the refill's order (x, gates, h): the loop's first step then
    // waits for slot A and slot B's x only, as every later step does.
    f32x4 gA[4], gB[4], hA, hB;
    float xA[XPT], xB[XPT];
    load_x(L - 1, xA);
    load_g(L - 1, gA);
    hA = load_h(L - 2);
    load_x(L - 2, xB);
    load_g(L - 2, gB);
    hB = load_h(L - 3);

    lg_u32x2 mcur = {0u, 0u};  // F16: the maxima the next step's bound is built from (read early)
    float Wn = 0.f, Cg = 1.f;  // F16: |W_hh^T|_inf, max(1, max |hn| / 4) of the workgroup
    float xsc = 1.f;           // F16: the x scale 2^sx
    int sg_cur = 0, sx = 0;    // F16: current dG scale exponent (uniform), the x scale exponent
    if constexpr (F16) {
        // the bound for step L-1: max |dh_L|, no dG; max |hn_{L-1}|
        post(L % 3, absmax4(dh), 0.f);
        const uint32_t hm = gru_row_max_bits(__float_as_uint(absmax4(gA[3])));
        if (j == 0) lds_max_u32(&wnm[2], hm);
        __syncthreads();
        Wn = __uint_as_float(__builtin_amdgcn_readfirstlane(wnm[0]));
        const float mhn = __uint_as_float(__builtin_amdgcn_readfirstlane(wnm[2]));
        Cg = fmaxf(1.f, 0.25f * fmaf(static_cast<float>(2 * H), __uint_as_float(__builtin_amdgcn_readfirstlane(wnm[1])), mhn));
        sx = lg_f16_scale_exp_c(__builtin_amdgcn_readfirstlane(wnm[3]));
        xsc = lg_pow2f(sx);
        mcur = *reinterpret_cast<const lg_u32x2*>(&gmx[L % 3][0]);
    }

    // (3) dW over the 32 sequences of LDS image bf: A = dG^T tiles (rows = gate rows 16w..,
    // K = seq), B = h_{t-1} / x_t (K = seq, columns = units / x columns)
    auto dw_products = [&](const int bf) {
        // tr16 addressing of this lane.  K = the 32 sequences, lane group q taking rows
        // 4q..4q+3 (elements 0-3) and 16+4q..16+4q+3 (elements 4-7), the same in both
        // operands: a 32-lane half then reads 8 consecutive rows, whose 8-dword windows meet
        // distinct banks at these row strides (rows 8q.. and 8q+4.. did 2-way:
        // MI355X_MICROARCH.md §LDS, 54 % of LDS-active cycles were conflicts)
        const int tr = 4 * q + (j >> 2), tc = 4 * (j & 3);
        AF bh[G::NTS][NP], bx[NP];
#pragma unroll
        for (int n = 0; n < G::NTS; ++n)
#pragma unroll
            for (int p = 0; p < NP; ++p)
                bh[n][p] = frag_tr(&hls[bf][p][tr][16 * (sh * G::NTS + n) + tc],
                                   &hls[bf][p][tr + 16][16 * (sh * G::NTS + n) + tc]);
#pragma unroll
        for (int p = 0; p < NP; ++p) bx[p] = frag_tr(&xls[bf][p][tr][tc], &xls[bf][p][tr + 16][tc]);
#pragma unroll
        for (int gi = 0; gi < 3; ++gi) {
            AF a[NP];
#pragma unroll
            for (int p = 0; p < NP; ++p)
                a[p] = frag_tr(&dgs[bf][p][tr][gi * H + 16 * w + tc], &dgs[bf][p][tr + 16][gi * H + 16 * w + tc]);
#pragma unroll
            for (int n = 0; n < G::NTS; ++n) dwh[gi][n] = mm(a, bh[n], dwh[gi][n]);
            if (sh == 0 && gi < 2) dwx[gi] = mm(a, bx, dwx[gi]);  // r, z: dG_i == dG_h
        }
        if (sh == 1) {  // n gate's input side: dG_in
            AF a[NP];
#pragma unroll
            for (int p = 0; p < NP; ++p)
                a[p] = frag_tr(&dgs[bf][p][tr][3 * H + 16 * w + tc], &dgs[bf][p][tr + 16][3 * H + 16 * w + tc]);
            dwx[0] = mm(a, bx, dwx[0]);
        }
    };
    auto step = [&](const int t, f32x4 (&g_cur)[4], f32x4& h_cur, float (&x_cur)[XPT]) {
        const int bf = t & 1;
        LG_GRU_STAMP(t, 0);
        float gsc = 1.f, gin_ = 1.f;  // F16: this step's dG scale and its inverse
        int sg = 0;                   // F16: its exponent
        if constexpr (F16) {
            // this step's scales from the bound posted by step t+1 (or the prologue), read right
            // after that step's barrier
            const float md = __uint_as_float(__builtin_amdgcn_readfirstlane(mcur[0]));
            const float mg = __uint_as_float(__builtin_amdgcn_readfirstlane(mcur[1]));
            const uint32_t bound = __builtin_amdgcn_readfirstlane(__float_as_uint(fmaf(Wn, mg, md) * Cg));
            int s = lg_f16_scale_exp_c(bound);
            sg = (s < sg_cur || s > sg_cur + kGruKeep) ? s : sg_cur;
            gsc = lg_pow2f(sg);
            gin_ = lg_pow2f(-sg);
            if (threadIdx.x < 2) gmx[(t + 2) % 3][threadIdx.x] = 0u;  // read by step t+1, written next by t-1
        }
        // (1) elementwise gate backward (h_cur = h_{t-1})
        {
            const f32x4 r = g_cur[0], z = g_cur[1], n = g_cur[2], hnp = g_cur[3];
            const f32x4 hp = t >= 1 ? h_cur : zero4();  // h_{-1} = 0
            f32x4 gr, gz, ghn, gin, dhp;
            // dG is linear in dh: F16 forms it at the step's scale straight away
            const f32x4 ds = F16 ? dh * gsc : dh;
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const float d = ds[reg];
                const float dn = d * (1.f - z[reg]);
                const float dzv = d * (hp[reg] - n[reg]);
                dhp[reg] = dh[reg] * z[reg];
                const float dnp = dn * (1.f - n[reg] * n[reg]);
                gin[reg] = dnp;
                ghn[reg] = dnp * r[reg];
                gr[reg] = dnp * hnp[reg] * r[reg] * (1.f - r[reg]);
                gz[reg] = dzv * z[reg] * (1.f - z[reg]);
            }
#ifdef LG_NM3_STAMPS
            asm volatile("" ::"v"(gr[0]), "v"(gz[3]), "v"(ghn[1]), "v"(gin[2]));
#endif
            LG_GRU_STAMP(t, 4);
            if constexpr (F16) {
                post(t % 3, absmax4(dh), fmaxf(absmax4(gr), fmaxf(absmax4(gz), absmax4(ghn))) * gin_);
                dbhn += ghn * gin_;
            } else {
                dbhn += ghn;
            }
            // d z materialised here: left to the compiler it is formed in (2), which keeps z live
            // across the slot's refill and costs a register move at the loop's back edge that
            // waits for the loads just issued
            asm volatile("" : "+v"(dhp[0]), "+v"(dhp[1]), "+v"(dhp[2]), "+v"(dhp[3]));
            dh = dhp;
            const f32x4 blk[4] = {gr, gz, ghn, gin};
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                lg_u32x2 f[NP];
                split_x4(blk[b], f);
#pragma unroll
                for (int p = 0; p < NP; ++p) *reinterpret_cast<lg_u32x2*>(&dgs[bf][p][sl][b * H + u0]) = f[p];
            }
            lg_u32x2 f[NP];
            split_x4(F16 ? hp * 16384.f : hp, f);  // F16: |h| <= 1 at the fixed scale 2^14
#pragma unroll
            for (int p = 0; p < NP; ++p) *reinterpret_cast<lg_u32x2*>(&hls[bf][p][sl][u0]) = f[p];
#pragma unroll
            for (int i = 0; i < XPT; ++i) {
                const int e = threadIdx.x + i * G::NTH;
                uint16_t pp[3];
                if constexpr (F16) split2_1(x_val(i, x_cur[i]) * xsc, pp[0], pp[1]);
                else split3_1(x_val(i, x_cur[i]), pp[0], pp[1], pp[2]);
#pragma unroll
                for (int p = 0; p < NP; ++p) xls[bf][p][e >> 4][e & 15] = pp[p];
            }
        }
        // refill this slot: step t-2's x / gates and h_{t-3}
        load_x(t - 2, x_cur);
        load_g(t - 2, g_cur);
        h_cur = load_h(t - 3);
        LG_GRU_STAMP(t, 5);
        // DEFER: step t+1's dW (image bf ^ 1, rewritten only after this step's barrier) in the
        // MFMA pipe while this step's LDS writes land and the workgroup gathers at the barrier
        if constexpr (DEFER)
            if (t < L - 1) dw_products(bf ^ 1);
        if constexpr (F16) {
            if (sg != sg_cur) {  // dW in units of 2^(sg + 14) / 2^(sg + sx) from here on
                const float f = lg_pow2f(sg - sg_cur);
#pragma unroll
                for (int gi = 0; gi < 3; ++gi)
#pragma unroll
                    for (int n = 0; n < G::NTS; ++n) dwh[gi][n] *= f;
                dwx[0] *= f;
                dwx[1] *= f;
            }
            sg_cur = sg;
        }
        // dgs/hls/xls[bf] complete.  Buffer bf was last read at step t+2, which every wave
        // finished before arriving at step t+1's barrier: one barrier per step suffices.
        LG_GRU_STAMP(t, 1);
        __syncthreads();
        LG_GRU_STAMP(t, 2);
        if constexpr (F16) mcur = *reinterpret_cast<const lg_u32x2*>(&gmx[t % 3][0]);  // cleared at t-2

        // (2) dh_{t-1} = d z + W_hh^T dG_h: two accumulator chains
        {
            f32x4 acc[2] = {zero4(), zero4()};
#pragma unroll
            for (int c = 0; c < G::NCH; ++c) {
                AF b[NP];
#pragma unroll
                for (int p = 0; p < NP; ++p) b[p] = frag_row(&dgs[bf][p][sl][32 * c + 8 * q]);
                acc[c & 1] = mm(adh[c], b, acc[c & 1]);
            }
            if constexpr (F16) dh += (acc[0] + acc[1]) * (sWinv * lg_pow2f(-sg_cur));
            else dh += acc[0] + acc[1];
#ifdef LG_NM3_STAMPS
            asm volatile("" ::"v"(dh[0]));  // the stamp after dh exists
#endif
        }
        LG_GRU_STAMP(t, 3);
        if constexpr (!DEFER) dw_products(bf);
    };
    int t = L - 1;
    for (; t >= 1; t -= 2) {     // unconditional pairs: a conditional second half would merge
        step(t, gA, hA, xA);      // the slot registers in a phi, i.e. moves that wait for loads
        step(t - 1, gB, hB, xB);
    }
    if (t == 0) step(0, gA, hA, xA);
    if constexpr (DEFER) dw_products(0);  // step 0's dW
    if constexpr (F16) {  // back to plain units
        const float fh = lg_pow2f(-(sg_cur + 14)), fx = lg_pow2f(-(sg_cur + sx));
#pragma unroll
        for (int gi = 0; gi < 3; ++gi)
#pragma unroll
            for (int n = 0; n < G::NTS; ++n) dwh[gi][n] *= fh;
        dwx[0] *= fx;
        dwx[1] *= fx;
    }

    // per-workgroup slab (the layout of k_gru_bwd): C rows = gate rows 16w + 4q + reg, columns j;
    // NI: each row then carries the projection's dW and db (lg_gru_node_init_bwd_workspace_bytes)
    constexpr int SLROW = SLAB + (NI ? H * (H + 1) + H : 0);
    float* out = slab + static_cast<int64_t>(blockIdx.x) * SLROW;
    float* oWhh = out;
    float* oWih = out + G3 * H;
    float* obih = oWih + G3 * I;
    float* obhh = obih + G3;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
#pragma unroll
        for (int gi = 0; gi < 3; ++gi)
#pragma unroll
            for (int n = 0; n < G::NTS; ++n)
                oWhh[(gi * H + u0 + reg) * H + 16 * (sh * G::NTS + n) + j] = dwh[gi][n][reg];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            if (sh == 1 && x == 1) break;
            const int gi = sh == 0 ? x : 2;
            const int g = gi * H + u0 + reg;
            if (j < I) oWih[g * I + j] = dwx[x][reg];
            if (j == 10) obih[g] = dwx[x][reg];            // constant-1 column: sum of dG_i
            if (j == 10 && gi < 2) obhh[g] = dwx[x][reg];  // r, z: dG_h == dG_i
        }
    }
    // db_hh(n) = sum over sequences of dG_hn: 16 lanes, then the two sequence halves
#pragma unroll
    for (int off = 1; off < 16; off <<= 1)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) dbhn[reg] += __shfl_xor(dbhn[reg], off);
    if (sh == 1 && j == 0) st4(&dbh[u0], dbhn);
    __syncthreads();
    if (sh == 0 && j == 0) st4(obhh + 2 * H + u0, dbhn + ld4(&dbh[u0]));
    if constexpr (NI) {
        // the projection's slab row: dW[o][k] = sum over the block's 32 rows of dproj[o] [h_L, 1][k]
        // (rows in order, one fmaf chain per output), db[o] = the same sum of dproj[o]
        constexpr int D = H, DP = D + 4, HP = H + 4;
        float* dpl = reinterpret_cast<float*>(&dgs[0][0][0][0]);  // [TS2][DP] dproj rows
        float* hx = dpl + TS2 * DP;                               // [TS2][HP] [h_L, 1]
        static_assert(sizeof(dgs) >= sizeof(float) * TS2 * (DP + HP), "projection staging fits the dG image");
        // (every read of the images ended before the db_hh barrier above)
        for (int i = threadIdx.x; i < TS2 * (D / 4); i += G::NTH) {
            const int rr = i / (D / 4), c4 = 4 * (i % (D / 4));
            const uint32_t sq = seq0 + rr;
            f32x4 v = zero4(), hv = zero4();
            if (sq < Nseq) {
                const uint32_t b = lg_div(sq, fdS), sl2 = sq - b * fdS.d;
                v = ld4(ni.dx0 + (static_cast<int64_t>(ni.sidx[sl2]) * ni.B + b) * D + c4);
                if (ni.live) v = v * ni.live[sl2];
                hv = ld4(hs + (static_cast<int64_t>(L - 1) * Nseq + sq) * H + c4);
            }
            st4(dpl + rr * DP + c4, v);
            st4(hx + rr * HP + c4, hv);
            if (c4 == 0) hx[rr * HP + H] = 1.f;
        }
        __syncthreads();
        float* outp = out + SLAB;  // [D][H + 1] dW, then [D] db
        constexpr int KQ = G::NTH / D, KW = H / KQ;
        static_assert(KW % 4 == 0, "float4 columns");
        const int o = threadIdx.x / KQ, kb = (threadIdx.x % KQ) * KW;
        float acc[KW];
#pragma unroll
        for (int jj = 0; jj < KW; ++jj) acc[jj] = 0.f;
        float a1 = 0.f;
        for (int rr = 0; rr < TS2; ++rr) {
            const float gz = dpl[rr * DP + o];
#pragma unroll
            for (int jj = 0; jj < KW; jj += 4) {
                const f32x4 hv = ld4(hx + rr * HP + kb + jj);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[jj + i] = fmaf(gz, hv[i], acc[jj + i]);
            }
            a1 += gz;
        }
#pragma unroll
        for (int jj = 0; jj < KW; ++jj) outp[o * (H + 1) + kb + jj] = acc[jj];
        if (kb == 0) {
            outp[o * (H + 1) + H] = a1;
            outp[D * (H + 1) + o] = a1 + ((blockIdx.x == 0 && ni.dbias_in) ? ni.dbias_in[o] : 0.f);
        }
    }
}

inline int64_t nblocks_seq(int64_t nseq) { return (nseq + TS - 1) / TS; }
inline int64_t nblocks_seq2(int64_t nseq) { return (nseq + TS2 - 1) / TS2; }

template <int H>
int launch_fwd(bool ut, bool save, const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
               const float* b_ih, const float* b_hh, float* h_seq, float* gates, float* h_last, int64_t B,
               int64_t L, int64_t S, hipStream_t s) {
    const uint32_t Nseq = static_cast<uint32_t>(B * S);
    const unsigned grid = static_cast<unsigned>(nblocks_seq(B * S));
    const lg_fastdiv fdS = lg_make_fastdiv(static_cast<uint32_t>(S));
#define LG_GRU_FWD(UT, SV)                                                                                        \
    lg_launch(k_gru_fwd<H, UT, SV>, grid, 12 * H, 0, s, residual, tfeat, w_ih, w_hh, b_ih, b_hh, h_seq, gates, h_last, \
              Nseq, static_cast<int>(L), static_cast<int>(S), fdS, GruNi{})
    if (ut) {
        if (save) LG_GRU_FWD(true, true); else LG_GRU_FWD(true, false);
    } else {
        if (save) LG_GRU_FWD(false, true); else LG_GRU_FWD(false, false);
    }
#undef LG_GRU_FWD
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

template <int H>
int launch_bwd(bool ut, bool need_dx, const float* residual, const float* tfeat, const float* w_ih,
               const float* w_hh, const float* h_seq, const float* gates, const float* dh_last, float* dx,
               float* slab, int64_t B, int64_t L, int64_t S, hipStream_t s) {
    const uint32_t Nseq = static_cast<uint32_t>(B * S);
    const unsigned grid = static_cast<unsigned>(nblocks_seq(B * S));
    const lg_fastdiv fdS = lg_make_fastdiv(static_cast<uint32_t>(S));
#define LG_GRU_BWD(UT, DX)                                                                                       \
    lg_launch(k_gru_bwd<H, UT, DX>, grid, 4 * H, 0, s, residual, tfeat, w_ih, w_hh, h_seq, gates, dh_last, dx, slab,   \
                                                 Nseq, static_cast<int>(L), static_cast<int>(S), fdS)
#define LG_GRU_BWD2(UT, F, DF)                                                                                   \
    lg_launch(k_gru_bwd2<H, UT, F, DF>, static_cast<unsigned>(nblocks_seq2(B * S)), GB2<H>::NTH, 0, s, residual,    \
              tfeat, w_hh, h_seq, gates, dh_last, slab, Nseq, static_cast<int>(L), static_cast<int>(S), fdS, GruNiB{})
#ifdef LG_KERNEL_LAB
    // lab A/B: LG_LAB_GRU_BF16X3 the 3-way bf16 split, LG_LAB_GRU_NODEFER each step's dW after its dh
    if (!need_dx && (getenv("LG_LAB_GRU_BF16X3") || getenv("LG_LAB_GRU_NODEFER"))) {
        const bool x3 = getenv("LG_LAB_GRU_BF16X3") != nullptr, nd = getenv("LG_LAB_GRU_NODEFER") != nullptr;
        if (ut) {
            if (x3) { if (nd) LG_GRU_BWD2(true, false, false); else LG_GRU_BWD2(true, false, true); }
            else LG_GRU_BWD2(true, true, false);
        } else {
            if (x3) { if (nd) LG_GRU_BWD2(false, false, false); else LG_GRU_BWD2(false, false, true); }
            else LG_GRU_BWD2(false, true, false);
        }
        LG_RET_IF_LAUNCH_FAILED();
        return LG_OK;
    }
#endif
    if (need_dx) {
        if (ut) LG_GRU_BWD(true, true); else LG_GRU_BWD(false, true);
    } else if (ut) {
        LG_GRU_BWD2(true, true, true);
    } else {
        LG_GRU_BWD2(false, true, true);
    }
#undef LG_GRU_BWD
#undef LG_GRU_BWD2
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

// ------------------------------------------------------------------ any hidden width
// The encoder at a hidden width the tiled kernels above do not cover (H not 32 / 64; ABI 26):
// the same recurrence (detector.py:60-73 through nn.GRU) with one hidden unit per thread and a
// workgroup per sequence (grid-stride over the B*S sequences), h_{t-1} and x_t in LDS, W read
// through the caches.  Same saved layouts as the tiled kernels: h_seq [t][seq][H] = h_t and
// gates [t][seq][4][H] = sigma(r), sigma(z), n, W_hn h_{t-1} + b_hn.  A generality path (the
// reference's widths run the tiled kernels), sized for correctness at any H <= 1024.
constexpr int kGenMaxH = 1024;
constexpr int kGenBwdBlocks = 512;  // slab rows of the generic backward

inline int gen_threads(int64_t H) { return static_cast<int>((H + 63) / 64 * 64); }

__global__ void __launch_bounds__(kGenMaxH) k_gru_gen_fwd(const float* __restrict__ residual,
                                                          const float* __restrict__ tfeat, const float* __restrict__ w_ih,
                                                          const float* __restrict__ w_hh, const float* __restrict__ b_ih,
                                                          const float* __restrict__ b_hh, float* __restrict__ h_seq,
                                                          float* __restrict__ gates, float* __restrict__ h_last, int B,
                                                          int L, int S, int I, int H) {
    extern __shared__ float gsm[];
    float* hs = gsm;      // h_{t-1} [H]
    float* xs = gsm + H;  // x_t [I]
    const int u = threadIdx.x;
    const int64_t nseq = static_cast<int64_t>(B) * S;
    for (int64_t seq = blockIdx.x; seq < nseq; seq += gridDim.x) {
        const int64_t b = seq / S, sn = seq % S;
        if (u < H) hs[u] = 0.f;
        for (int t = 0; t < L; ++t) {
            if (u < I) xs[u] = u == 0 ? residual[(b * L + t) * S + sn] : tfeat[(b * L + t) * (I - 1) + u - 1];
            __syncthreads();
            float hn = 0.f, g[4] = {0.f, 0.f, 0.f, 0.f};
            if (u < H) {
                float a[3], c[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const int row = k * H + u;
                    a[k] = b_ih[row];
                    for (int i = 0; i < I; ++i) a[k] = fmaf(w_ih[static_cast<int64_t>(row) * I + i], xs[i], a[k]);
                    c[k] = b_hh[row];
                    const float* wr = w_hh + static_cast<int64_t>(row) * H;
                    for (int i = 0; i < H; ++i) c[k] = fmaf(wr[i], hs[i], c[k]);
                }
                g[0] = sigm(a[0] + c[0]);
                g[1] = sigm(a[1] + c[1]);
                g[2] = gru_tanh(a[2] + g[0] * c[2]);
                g[3] = c[2];
                hn = (1.f - g[1]) * g[2] + g[1] * hs[u];
            }
            __syncthreads();
            if (u < H) {
                hs[u] = hn;
                const int64_t r = static_cast<int64_t>(t) * nseq + seq;
                if (h_seq) h_seq[r * H + u] = hn;
                if (gates) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) gates[(r * 4 + k) * H + u] = g[k];
                }
            }
        }
        if (u < H) h_last[seq * H + u] = hs[u];
        __syncthreads();
    }
}

// BPTT per sequence; the weight gradients accumulate into the workgroup's own slab row
// [dW_hh 3H x H | dW_ih 3H x I | db_ih 3H | db_hh 3H] (every element read-modified-written by
// one fixed thread: no races, no atomics), reduced over the rows in row order afterwards.
__global__ void __launch_bounds__(kGenMaxH) k_gru_gen_bwd(const float* __restrict__ residual,
                                                          const float* __restrict__ tfeat, const float* __restrict__ w_ih,
                                                          const float* __restrict__ w_hh, const float* __restrict__ h_seq,
                                                          const float* __restrict__ gates,
                                                          const float* __restrict__ dh_last, float* __restrict__ dx,
                                                          float* __restrict__ slab, int B, int L, int S, int I, int H) {
    extern __shared__ float gsm[];
    float* dh = gsm;            // dL/dh_t [H]
    float* hp = dh + H;         // h_{t-1} [H]
    float* dgh = hp + H;        // d(W_h. h + b_h.) [3H]
    float* dgn = dgh + 3 * H;   // d(W_in x + b_in) [H] (the r and z parts equal dgh's)
    float* xs = dgn + H;        // x_t [I]
    const int u = threadIdx.x, nt = blockDim.x;
    const int G3 = 3 * H;
    const int64_t nseq = static_cast<int64_t>(B) * S, len = static_cast<int64_t>(G3) * (H + I) + 2 * G3;
    float* row = slab + blockIdx.x * len;
    float* dwhh = row;
    float* dwih = row + static_cast<int64_t>(G3) * H;
    float* dbih = dwih + static_cast<int64_t>(G3) * I;
    float* dbhh = dbih + G3;
    // each element is zeroed by the thread that accumulates it
    if (u < H)
        for (int j = 0; j < G3; ++j) dwhh[static_cast<int64_t>(j) * H + u] = 0.f;
    if (u < I)
        for (int j = 0; j < G3; ++j) dwih[static_cast<int64_t>(j) * I + u] = 0.f;
    for (int j = u; j < G3; j += nt) dbih[j] = dbhh[j] = 0.f;
    auto dgi = [&](int j) { return j < 2 * H ? dgh[j] : dgn[j - 2 * H]; };
    for (int64_t seq = blockIdx.x; seq < nseq; seq += gridDim.x) {
        const int64_t b = seq / S, sn = seq % S;
        if (u < H) dh[u] = dh_last[seq * H + u];
        for (int t = L - 1; t >= 0; --t) {
            const int64_t r = static_cast<int64_t>(t) * nseq + seq;
            if (u < I) xs[u] = u == 0 ? residual[(b * L + t) * S + sn] : tfeat[(b * L + t) * (I - 1) + u - 1];
            float dz_keep = 0.f;
            if (u < H) {
                const float h0 = t > 0 ? h_seq[(r - nseq) * H + u] : 0.f;
                hp[u] = h0;
                const float rg = gates[(r * 4 + 0) * H + u], zg = gates[(r * 4 + 1) * H + u];
                const float ng = gates[(r * 4 + 2) * H + u], ghn = gates[(r * 4 + 3) * H + u];
                const float d = dh[u];
                const float dnp = d * (1.f - zg) * (1.f - ng * ng);
                const float dzp = d * (h0 - ng) * zg * (1.f - zg);
                const float drp = dnp * ghn * rg * (1.f - rg);
                dgh[u] = drp;
                dgh[H + u] = dzp;
                dgh[2 * H + u] = dnp * rg;
                dgn[u] = dnp;
                dz_keep = d * zg;
            }
            __syncthreads();
            float acc = dz_keep;
            if (u < H) {
                for (int j = 0; j < G3; ++j) {
                    const float gj = dgh[j];
                    acc = fmaf(w_hh[static_cast<int64_t>(j) * H + u], gj, acc);
                    dwhh[static_cast<int64_t>(j) * H + u] += gj * hp[u];
                }
            }
            if (u < I) {
                float dxi = 0.f;
                for (int j = 0; j < G3; ++j) {
                    const float gj = dgi(j);
                    dxi = fmaf(w_ih[static_cast<int64_t>(j) * I + u], gj, dxi);
                    dwih[static_cast<int64_t>(j) * I + u] += gj * xs[u];
                }
                if (dx) dx[(seq * L + t) * I + u] = dxi;
            }
            for (int j = u; j < G3; j += nt) {
                dbih[j] += dgi(j);
                dbhh[j] += dgh[j];
            }
            __syncthreads();
            if (u < H) dh[u] = acc;
        }
        __syncthreads();
    }
}

bool dims_ok(int64_t B, int64_t L, int64_t S) {
    return B >= 0 && L > 0 && S > 0 && L <= INT32_MAX && S <= INT32_MAX && B * S < (int64_t{1} << 31);
}
// the forward's h / gate stores address one step's rows of gates by 32-bit byte offsets
bool fwd_rows_ok(int64_t B, int64_t S, int64_t H) { return B * S * 4 * H * 4 < (int64_t{1} << 31); }

}  // namespace

#ifdef LG_NM3_STAMPS
extern "C" int lg_lab_gru_stamps(uint64_t* host, int64_t n) {
    if (n > static_cast<int64_t>(256) * 8 * kGruStamps) return LG_EINVAL;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gru_stamps), static_cast<size_t>(n) * 8) == hipSuccess ? LG_OK
                                                                                                         : LG_EHIP;
}
extern "C" int lg_lab_gru_stamps_clear(void) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_gru_stamps)) != hipSuccess) return LG_EHIP;
    return hipMemset(p, 0, sizeof(uint64_t) * 256 * 8 * kGruStamps) == hipSuccess ? LG_OK : LG_EHIP;
}
#endif

extern "C" int64_t lg_gru_bwd_workspace_bytes(int64_t B, int64_t S, int64_t I, int64_t H) {
    if (B < 0 || S < 0 || (I != 1 && I != 10) || H < 1 || H > kGenMaxH) return LG_EINVAL;
    const int64_t slab = 3 * H * H + 3 * H * I + 6 * H;
    if (H != 32 && H != 64)
        return std::max<int64_t>(1, std::min<int64_t>(B * S, kGenBwdBlocks)) * slab * static_cast<int64_t>(sizeof(float));
    return std::max<int64_t>(1, nblocks_seq(B * S)) * slab * static_cast<int64_t>(sizeof(float));
}

extern "C" int lg_gru_fwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
                          const float* b_ih, const float* b_hh, float* h_seq, float* gates, float* h_last, int64_t B,
                          int64_t L, int64_t S, int64_t I, int64_t H, lg_stream_t stream) {
    if (!dims_ok(B, L, S)) return LG_EINVAL;
    if (H < 1 || H > kGenMaxH || (I != 1 && I != 10)) return LG_EUNSUPPORTED;
    if (!residual || !w_ih || !w_hh || !b_ih || !b_hh || !h_last || (I == 10 && !tfeat)) return LG_EINVAL;
    if (gates && !h_seq) return LG_EINVAL;  // the backward needs both
    if (B == 0) return LG_OK;
    hipStream_t s = lg_stream(stream);
    if (H != 32 && H != 64) {  // any other width: the generic kernel
        const unsigned grid = static_cast<unsigned>(std::min<int64_t>(B * S, 4096));
        lg_launch(k_gru_gen_fwd, grid, gen_threads(H), sizeof(float) * (H + I), s, residual, tfeat, w_ih, w_hh, b_ih,
                  b_hh, h_seq, gates, h_last, static_cast<int>(B), static_cast<int>(L), static_cast<int>(S),
                  static_cast<int>(I), static_cast<int>(H));
        LG_RET_IF_LAUNCH_FAILED();
        return LG_OK;
    }
    if (!fwd_rows_ok(B, S, H)) return LG_EUNSUPPORTED;
    return H == 64 ? launch_fwd<64>(I == 10, gates != nullptr, residual, tfeat, w_ih, w_hh, b_ih, b_hh, h_seq, gates,
                                    h_last, B, L, S, s)
                   : launch_fwd<32>(I == 10, gates != nullptr, residual, tfeat, w_ih, w_hh, b_ih, b_hh, h_seq, gates,
                                    h_last, B, L, S, s);
}

extern "C" int lg_gru_bwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
                          const float* h_seq, const float* gates, const float* dh_last, float* dx, float* dw_ih,
                          float* dw_hh, float* db_ih, float* db_hh, int64_t B, int64_t L, int64_t S, int64_t I,
                          int64_t H, void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    if (!dims_ok(B, L, S)) return LG_EINVAL;
    if (H < 1 || H > kGenMaxH || (I != 1 && I != 10)) return LG_EUNSUPPORTED;
    if (!residual || !w_ih || !w_hh || !h_seq || !gates || !dh_last || !dw_ih || !dw_hh || !db_ih || !db_hh ||
        !workspace || (I == 10 && !tfeat))
        return LG_EINVAL;
    hipStream_t s = lg_stream(stream);
    const bool gen = H != 32 && H != 64;
    // slabs written: one per workgroup (16 sequences with dx, 32 without; the generic kernel:
    // one per workgroup of its grid-stride)
    const int nb = static_cast<int>(std::max<int64_t>(
        1, gen ? std::min<int64_t>(B * S, kGenBwdBlocks) : (dx ? nblocks_seq(B * S) : nblocks_seq2(B * S))));
    float* slab = static_cast<float*>(workspace);
    const int64_t G3 = 3 * H, len = G3 * H + G3 * I + 2 * G3;
    if (ws_bytes < nb * len * static_cast<int64_t>(sizeof(float))) return LG_EINVAL;
    if (B == 0) {
        if (hipMemsetAsync(slab, 0, sizeof(float) * len, s) != hipSuccess) return LG_EHIP;
    } else if (gen) {
        lg_launch(k_gru_gen_bwd, static_cast<unsigned>(nb), gen_threads(H), sizeof(float) * (6 * H + I), s, residual,
                  tfeat, w_ih, w_hh, h_seq, gates, dh_last, dx, slab, static_cast<int>(B), static_cast<int>(L),
                  static_cast<int>(S), static_cast<int>(I), static_cast<int>(H));
        LG_RET_IF_LAUNCH_FAILED();
    } else {
        const int rc = H == 64 ? launch_bwd<64>(I == 10, dx != nullptr, residual, tfeat, w_ih, w_hh, h_seq, gates,
                                                dh_last, dx, slab, B, L, S, s)
                               : launch_bwd<32>(I == 10, dx != nullptr, residual, tfeat, w_ih, w_hh, h_seq, gates,
                                                dh_last, dx, slab, B, L, S, s);
        if (rc != LG_OK) return rc;
    }
    const int64_t nWhh = G3 * H, nWih = G3 * I;
    const LgSlabSeg segs[4] = {{0, nWhh, dw_hh}, {nWhh, nWih, dw_ih}, {nWhh + nWih, G3, db_ih},
                               {nWhh + nWih + G3, G3, db_hh}};
    return lg_launch_slab_reduce_multi(slab, nb, len, segs, 4, nullptr, nullptr, s);
}

// ------------------------------------------------------------------ GRU + node init, fused
extern "C" int lg_gru_node_init_fwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
                                    const float* b_ih, const float* b_hh, float* h_seq, float* gates, float* h_last,
                                    const int32_t* sensor_slot, const int64_t* sensor_idx, const float* proj_w,
                                    const float* node_bias, float* xs0, uint16_t* x0bits, int64_t B, int64_t L,
                                    int64_t S, int64_t I, int64_t H, int64_t N, int flags, float dropout_p,
                                    uint64_t seed, uint32_t salt, lg_stream_t stream) {
    if (!dims_ok(B, L, S) || N <= 0 || N >= (int64_t{1} << 24)) return LG_EINVAL;
    if ((H != 32 && H != 64) || (I != 1 && I != 10)) return LG_EUNSUPPORTED;
    if (!residual || !w_ih || !w_hh || !b_ih || !b_hh || !h_last || (I == 10 && !tfeat)) return LG_EINVAL;
    if (!sensor_slot || !sensor_idx || !proj_w || !node_bias || !xs0 || !x0bits) return LG_EINVAL;
    if (gates && !h_seq) return LG_EINVAL;
    if (!fwd_rows_ok(B, S, H)) return LG_EUNSUPPORTED;
    const bool drop = (flags & LG_F_DROPOUT) != 0;
    if (drop && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (B == 0) return LG_OK;
    const int64_t ngroups = (B + 15) / 16;
    if (N * ngroups * 64 >= (int64_t{1} << 32) || B * N >= kLgMaxRows) return LG_EUNSUPPORTED;
    hipStream_t s = lg_stream(stream);
    const uint32_t Nseq = static_cast<uint32_t>(B * S);
    // the sequence blocks, then the bits blocks: the CU slots the sequence blocks leave free (two
    // workgroups per CU at H = 64, four at H = 32), at least 16
    const int64_t nseqblk = nblocks_seq(B * S), slots = (H == 64 ? 2 : 4) * static_cast<int64_t>(lg_num_cus());
    const int64_t nbits = std::max<int64_t>(16, nseqblk < slots ? slots - nseqblk : 0);
    const unsigned grid = static_cast<unsigned>(nseqblk + nbits);
    const lg_fastdiv fdS = lg_make_fastdiv(static_cast<uint32_t>(S));
    const GruNi ni{sensor_slot, sensor_idx, proj_w, node_bias, xs0, x0bits, static_cast<uint32_t>(B),
                   static_cast<uint32_t>(N), static_cast<uint32_t>(ngroups),
                   lg_make_fastdiv(static_cast<uint32_t>(ngroups)), drop ? 1 : 0, dropout_p,
                   drop ? 1.0f / (1.0f - dropout_p) : 1.0f, seed, salt, static_cast<uint32_t>(nseqblk)};
#define LG_GRU_NI(HH, UT, SV)                                                                                     \
    lg_launch(k_gru_fwd<HH, UT, SV, true>, grid, 12 * HH, 0, s, residual, tfeat, w_ih, w_hh, b_ih, b_hh, h_seq, gates, \
              h_last, Nseq, static_cast<int>(L), static_cast<int>(S), fdS, ni)
    const bool ut = I == 10, save = gates != nullptr;
    if (H == 64) {
        if (ut) { if (save) LG_GRU_NI(64, true, true); else LG_GRU_NI(64, true, false); }
        else { if (save) LG_GRU_NI(64, false, true); else LG_GRU_NI(64, false, false); }
    } else {
        if (ut) { if (save) LG_GRU_NI(32, true, true); else LG_GRU_NI(32, true, false); }
        else { if (save) LG_GRU_NI(32, false, true); else LG_GRU_NI(32, false, false); }
    }
#undef LG_GRU_NI
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int64_t lg_gru_node_init_bwd_workspace_bytes(int64_t B, int64_t S, int64_t I, int64_t H) {
    if (B < 0 || S < 0 || (I != 1 && I != 10) || (H != 32 && H != 64)) return LG_EINVAL;
    const int64_t slab = 3 * H * H + 3 * H * I + 6 * H + H * (H + 1) + H;
    return std::max<int64_t>(1, nblocks_seq2(B * S)) * slab * static_cast<int64_t>(sizeof(float));
}

extern "C" int lg_gru_node_init_bwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
                                    const float* h_seq, const float* gates, const float* dx0,
                                    const int64_t* sensor_idx, const float* live, const float* proj_w,
                                    const float* dbias_in, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh,
                                    float* dproj_w, float* dproj_b, int64_t B, int64_t L, int64_t S, int64_t I,
                                    int64_t H, int64_t N, void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    if (!dims_ok(B, L, S) || N <= 0) return LG_EINVAL;
    if ((H != 32 && H != 64) || (I != 1 && I != 10)) return LG_EUNSUPPORTED;
    if (!residual || !w_ih || !w_hh || !h_seq || !gates || !dx0 || !sensor_idx || !proj_w || !dw_ih || !dw_hh ||
        !db_ih || !db_hh || !dproj_w || !dproj_b || !workspace || (I == 10 && !tfeat))
        return LG_EINVAL;
    if (B * N >= kLgMaxRows) return LG_EUNSUPPORTED;
    hipStream_t s = lg_stream(stream);
    const int nb = static_cast<int>(std::max<int64_t>(1, nblocks_seq2(B * S)));
    const int64_t G3 = 3 * H, gl = G3 * H + G3 * I + 2 * G3, len = gl + H * (H + 1) + H;
    if (ws_bytes < nb * len * static_cast<int64_t>(sizeof(float))) return LG_EINVAL;
    float* slab = static_cast<float*>(workspace);
    // inside a reduce batch dbias_in may still be pending (the layer-0 backward's reduction not
    // yet launched): its partials are then summed into db by the batch instead (as
    // lg_sensor_proj_bwd does)
    LgSlabSeg dbseg{gl + H * (H + 1), H, dproj_b};
    if (lg_reduce_batch_pending(dbias_in, &dbseg.slab2, &dbseg.G2, &dbseg.stride2, &dbseg.off2)) dbias_in = nullptr;
    if (B == 0) {
        if (hipMemsetAsync(slab, 0, sizeof(float) * len, s) != hipSuccess) return LG_EHIP;
    } else {
        const uint32_t Nseq = static_cast<uint32_t>(B * S);
        const lg_fastdiv fdS = lg_make_fastdiv(static_cast<uint32_t>(S));
        const GruNiB ni{dx0, sensor_idx, live, proj_w, dbias_in, static_cast<uint32_t>(B)};
#define LG_GRU_NIB(HH, UT)                                                                                        \
    lg_launch(k_gru_bwd2<HH, UT, true, true, true>, static_cast<unsigned>(nb), GB2<HH>::NTH, 0, s, residual, tfeat,   \
              w_hh, h_seq, gates, nullptr, slab, Nseq, static_cast<int>(L), static_cast<int>(S), fdS, ni)
        if (H == 64) {
            if (I == 10) LG_GRU_NIB(64, true); else LG_GRU_NIB(64, false);
        } else {
            if (I == 10) LG_GRU_NIB(32, true); else LG_GRU_NIB(32, false);
        }
#undef LG_GRU_NIB
        LG_RET_IF_LAUNCH_FAILED();
    }
    const int64_t nWhh = G3 * H, nWih = G3 * I;
    const LgSlabSeg segs[6] = {{0, nWhh, dw_hh}, {nWhh, nWih, dw_ih}, {nWhh + nWih, G3, db_ih},
                               {nWhh + nWih + G3, G3, db_hh}, {gl, H * (H + 1), dproj_w}, dbseg};
    return lg_launch_slab_reduce_multi(slab, nb, len, segs, 6, nullptr, nullptr, s);
}
