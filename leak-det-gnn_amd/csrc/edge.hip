// K8 + K9: EdgeHead (reference detector.py:76-88, 206-211) fused end to end.
//
//   feat[b,p] = [h_u, h_v, |h_u - h_v|]            (3D)      u, v = pipe_ends[p]
//   hid       = dropout(relu(W1 feat + b1))          (128)
//   logit     = W2 hid + b2                          (1)
//
// The (B, P, 3D) feature tensor (150 MB at B=256) is never written to HBM.  Both kernels
// run every product on v_mfma_f32_16x16x32_bf16 with 3-way split fp32 operands
// (split_bf16.h: fp32-level accuracy at 6/16 of the f32-MFMA issue time).
//
// Forward: one 512-thread workgroup handles TR = 2048/D pipe rows per tile (32 at D=64):
// each thread gathers one float4 of h_u and of h_v, and writes the three bf16 parts of
// (h_u, h_v, |h_u - h_v|) into an LDS feature image.  Wave w (of 8) computes hidden units
// [16w, 16w+16) for all rows as hid^T = W1 feat^T (its split W1 rows live in registers),
// applies bias/ReLU/dropout, dots with W2; the eight partial logits are summed in wave order.
// The next tile's endpoint rows are loaded into registers during the MFMA phase (and the
// endpoint ids one tile further ahead).  In training the post-activation hidden layer is
// written out (hid, fp32 [B*P][128]) for the backward.
//
// Backward (no recompute): from hid, dlogit:
//   g     = dlogit * W2 * dropout_scale * [hid > 0]     (= d pre-activation)
//   dW2  += dlogit * hid     db1 += g     db2 += dlogit  (fp64)
//   dW1  += g^T feat         (MFMA, K = rows, both operands by ds_read_b64_tr_b16)
//   dfeat^T = W1^T g^T       (MFMA, K = hidden; wave = 16 features x {u,v,|u-v|} x half the
//                             hidden units; the two halves meet in LDS in a fixed order)
//   dpipe[b,p,0] = dfeat_u + sgn*dfeat_abs,  dpipe[b,p,1] = dfeat_v - sgn*dfeat_abs,
//   sgn = sign(h_u - h_v) from the fp32 difference (torch abs backward).
// dpipe is then summed per node over the incidence CSR by lg_pipe_scatter_bwd
// (deterministic, no atomics).  Weight grads: per-workgroup slabs + fixed-order reduce.
#include <algorithm>
#include <tuple>
#include <vector>
#include "common.h"
#include "reduce.h"
#include "split_bf16.h"

#ifndef LG_EDGE_DH_AUX
#define LG_EDGE_DH_AUX LG_ACT_AUX  // lab A/B of the streamed scatter's dh stores
#endif

namespace {

constexpr int HID = 128;
constexpr int NW = 8;        // waves per workgroup (= HID / 16)
constexpr int NT = 64 * NW;

template <int D>
struct EG {
    static constexpr int K3 = 3 * D;            // feature width
    static constexpr int TR = 2048 / D;         // pipe rows per tile: one float4 of h_u and h_v per thread
    static constexpr int RB = TR / 16;          // 16-row blocks per tile
    static constexpr int KS = K3 / 32;          // k-steps of the feature contraction
    static constexpr int F4 = D / 4;            // float4 per node row
    static constexpr int FSB = K3 + 8;          // fwd feature image row stride (bf16): row reads conflict-free
    static constexpr int FTB = K3 + 16;         // bwd feature image row stride: transposed reads conflict-free
    static constexpr int GSB = HID + 8;         // bwd d-hidden image row stride
    static constexpr int DT = D / 16;           // 16-feature tiles of one endpoint row
    static constexpr int RG = NW / (2 * DT);    // row groups of the dfeat product
    static constexpr int RBW = RB / RG;         // row blocks per wave in the dfeat product
    static constexpr int KT = K3 / 16;          // 16-feature tiles of dW1
    static constexpr int HPT = TR / 16;         // float4 of the hidden tile per thread
    static constexpr int FPL = TR * FSB, FTPL = TR * FTB, GPL = TR * GSB;  // image plane strides
    static constexpr int NROLE = DT * RG * RBW;  // dfeat output blocks (16 features x 16 rows) = NW
    static constexpr int NRED = 2 * NROLE * 3;   // dfeat partials of both hidden halves (f32x4 x 64 lanes)
    // forward workgroups resident per CU (VGPR-bound: 144 VGPRs of split W1 at D=64; the
    // bf16 tier keeps only the hi part, 48 VGPRs, and fits two)
    static constexpr int FWD_WG_PER_CU = 1, FWD_WG_PER_CU_BF = 2;
    static constexpr int64_t FWD_LDS = int64_t{2} * 2 * 3 * FPL + 4 * (2 * 4 * TR + 2 * HID + 2 * TR);  // images, partials, b1/W2, row scales
    static constexpr int64_t BWD_LDS = int64_t{2} * (3 * FTPL + 3 * GPL) + 2 * TR * D + 16 * 64 * NRED;
    // F16 (the f16x2 transform): two image planes instead of three, then the per-row g scale
    // exponents [2][TR] and the per-tile product scale exponents [2] (+ pad)
    static constexpr int64_t BWD_LDS_F16 = int64_t{2} * (2 * FTPL + 2 * GPL) + 2 * TR * D + 16 * 64 * NRED + 4 * (2 * TR + 4);
    static constexpr int64_t bwd_lds(bool f16) { return f16 ? BWD_LDS_F16 : BWD_LDS; }
};
static_assert(EG<64>::RBW == 2 && EG<32>::RBW == 2, "dfeat wave split");
static_assert(EG<64>::NROLE == NW && EG<32>::NROLE == NW, "one dfeat output block per wave");
static_assert(EG<64>::BWD_LDS <= 160 * 1024 && EG<32>::BWD_LDS <= 160 * 1024, "LDS budget");
static_assert(EG<64>::BWD_LDS_F16 % 16 == 0 && EG<32>::BWD_LDS_F16 % 16 == 0, "16-byte aligned tail");

// max of a non-negative float's bits over the lanes of one node row of the gather layout
// (D / 4 lanes: 16 at D = 64, 8 at D = 32), broadcast to them
template <int D>
__device__ __forceinline__ uint32_t lg_rowgroup_max_bits(uint32_t m) {
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0xB1, 0xF, 0xF, false)));  // xor 1
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x4E, 0xF, 0xF, false)));  // xor 2
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x141, 0xF, 0xF, false)));  // half-row mirror
    if constexpr (D == 64)
        m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x140, 0xF, 0xF, false)));  // row mirror
    return m;
}
__device__ __forceinline__ int lg_wave_min_i32(int v) {
    for (int off = 1; off < 64; off <<= 1) v = min(v, __shfl_xor(v, off));
    return v;
}

// row r = b*P + p of the (B, P) logit space -> element (b, p) of a buffer with row stride ldo
__device__ __forceinline__ int64_t lg_row_index(int64_t r, const lg_fastdiv& fdP, int64_t ldo) {
    const uint32_t b = lg_div(static_cast<uint32_t>(r), fdP);
    return static_cast<int64_t>(b) * ldo + (static_cast<uint32_t>(r) - b * fdP.d);
}

// Prefetch loads below are unconditional (a row past the end reads pipe row 0 of window 0,
// whose values are never stored and meet a zero dlogit in the backward) and land exactly in
// the registers that are used: a load under a divergent branch, or a 16-byte load of an
// int64 pair whose unused high words the register allocator recycles as temporaries, makes
// the compiler wait for every load in flight (vmcnt(0)) right after issuing the prefetch —
// measured, that exposed a full memory round trip per tile.
__device__ __forceinline__ uint32_t clamp_row(int64_t r, int64_t BP) { return r < BP ? static_cast<uint32_t>(r) : 0u; }
// endpoint node ids of pipe row r: the low words of the int64 ids (ids < 2^31)
__device__ __forceinline__ void load_ends(const int64_t* __restrict__ ends, int64_t r, int64_t BP,
                                          const lg_fastdiv& fdP, uint32_t& nu, uint32_t& nv) {
    const uint32_t rr = clamp_row(r, BP);
    const uint32_t p = rr - lg_div(rr, fdP) * fdP.d;
    const uint32_t* e32 = reinterpret_cast<const uint32_t*>(ends);
    nu = e32[4 * p];
    nv = e32[4 * p + 2];
}
// float4 f of the two endpoint rows of pipe row r; 32-bit element offsets (the API requires
// N*B*D < 2^32)
template <int D>
__device__ __forceinline__ void load_rows(const float* __restrict__ h, int64_t r, int64_t BP, const lg_fastdiv& fdP,
                                          uint32_t nu, uint32_t nv, uint32_t sb, uint32_t sn, int f, f32x4& u,
                                          f32x4& v) {
    const uint32_t b = lg_div(clamp_row(r, BP), fdP);
    u = ld4(h + ((b * sb + nu * sn) * D + 4 * f));
    v = ld4(h + ((b * sb + nv * sn) * D + 4 * f));
}
// three bf16 parts of 4 floats -> 8-byte slots at img[off], img[pl + off], img[2 pl + off]
// (BF: the hi part only; the other planes are never read)
template <bool BF = false>
__device__ __forceinline__ void st_split4(uint16_t* img, int pl, int off, const f32x4& x) {
    lg_u32x2 a, b, c;
    split3_x4(x, a, b, c);
    *reinterpret_cast<lg_u32x2*>(img + off) = a;
    if (BF) return;
    *reinterpret_cast<lg_u32x2*>(img + pl + off) = b;
    *reinterpret_cast<lg_u32x2*>(img + 2 * pl + off) = c;
}

// 2-way fp16 split of 4 floats scaled by 2^e into 8-byte slots at img[off], img[pl + off]
__device__ __forceinline__ void st_split2h(uint16_t* img, int pl, int off, const f32x4& x, float sc) {
    uint32_t a0, a1, b0, b1;
    split2_f16_pair(x[0] * sc, x[1] * sc, a0, a1);
    split2_f16_pair(x[2] * sc, x[3] * sc, b0, b1);
    *reinterpret_cast<lg_u32x2*>(img + off) = lg_u32x2{a0, b0};
    *reinterpret_cast<lg_u32x2*>(img + pl + off) = lg_u32x2{a1, b1};
}
// max of a non-negative float's bits over the 16 lanes of a DPP row (row_ror within the row)
__device__ __forceinline__ uint32_t lg_row16_max_bits(uint32_t m) {
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0xB1, 0xF, 0xF, false)));
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x4E, 0xF, 0xF, false)));
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x124, 0xF, 0xF, false)));
    return max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x128, 0xF, 0xF, false)));
}

// F16 (fp32 tier, D = 64): the MLP's products on the 2-way fp16 split (split_bf16.h f16x2: 3 f16
// MFMAs per product instead of 6 bf16 ones, dropped term <= 2^-22 of the product).  Scales
// are uniform along K as the MFMA needs: W1 per wave (its own rows), the features per pipe
// row (the B operand's columns; the row's 16 gather lanes take the max through DPP), so
// hid = acc 2^-(sW + s_row) + b1 exactly unscaled.
template <int D, bool BF, bool F16 = false>
__global__ void __launch_bounds__(NT)
__attribute__((amdgpu_waves_per_eu((BF ? EG<D>::FWD_WG_PER_CU_BF : EG<D>::FWD_WG_PER_CU) * 2, F16 ? 2 : 4)))
k_edge_fwd(const int64_t* __restrict__ ends, const float* __restrict__ h, const float* __restrict__ W1,
           const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
           float* __restrict__ logit, int64_t ldo, float* __restrict__ hid_out, uint32_t sb, uint32_t sn,
           lg_fastdiv fdP, int64_t BP, int64_t ntiles, int dropout, float p_drop, float dscale, uint64_t seed,
           uint32_t salt) {
    using G = EG<D>;
    constexpr int RBF = G::RB / 2;  // row blocks per wave
#ifdef LG_KERNEL_LAB
    // kernel-lab builds only (results WRONG when set): 1 skip MFMA, 2 skip row loads, 4 skip split
    const int lab = dropout >> 8;
    dropout &= 1;
#else
    constexpr int lab = 0;
#endif
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const bool hbuf = BP * HID * 4 < 0x7FFFFFFF;  // the hidden layer's stores (common.h lg_act_rsrc)
    const __amdgpu_buffer_rsrc_t hrs = lg_act_rsrc(hid_out, hid_out && hbuf ? BP * HID : 0);
    uint16_t* fimg = reinterpret_cast<uint16_t*>(smem);                                  // [2][3][TR][FSB]
    float(*part)[4][G::TR] = reinterpret_cast<float(*)[4][G::TR]>(fimg + 2 * 3 * G::FPL);  // [2][4][TR]
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    // wave = hidden units [32 nh, 32 nh + 32) (two 16-unit tiles: every feature fragment read
    // from LDS feeds two MFMA chains) x row blocks [RBF rh, RBF rh + RBF)
    const int nh = w & 3, rh = w >> 2;
    // A operand: W1[n = 32 nh + 16 i + c][k = 32 ks + 8q + j], split once
    static_assert(!F16 || (!BF && D == 64), "f16x2: fp32 tier, D = 64");
    lg_bf16x8 wa[2][G::KS][3];
    lg_f16x8 wh[2][G::KS][F16 ? 2 : 1];
    int sw = 0;  // F16: the wave's W1 scale exponent
    if constexpr (F16) {
        f32x4 wr[2][G::KS][2];
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int ks = 0; ks < G::KS; ++ks) {
                const float* src = W1 + (32 * nh + 16 * i + c) * G::K3 + 32 * ks + 8 * q;
                wr[i][ks][0] = ld4(src);
                wr[i][ks][1] = ld4(src + 4);
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
                    for (int e = 0; e < 4; ++e) m = max(m, __float_as_uint(fabsf(wr[i][ks][h2][e])));
            }
        sw = lg_f16_scale_exp_c(lg_wave_max_bits(m));
        const float sc = lg_pow2f(sw);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int ks = 0; ks < G::KS; ++ks) split2_f16_x8(wr[i][ks][0] * sc, wr[i][ks][1] * sc, wh[i][ks][0], wh[i][ks][1]);
    } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int ks = 0; ks < G::KS; ++ks) {
                const float* src = W1 + (32 * nh + 16 * i + c) * G::K3 + 32 * ks + 8 * q;
                split3_x8(ld4(src), ld4(src + 4), wa[i][ks][0], wa[i][ks][1], wa[i][ks][2]);
            }
    }
    // b1 / W2 of hidden units n = 32 nh + 16 i + 4q + reg (the accumulator rows) are re-read
    // from LDS per tile (VGPR budget)
    float* bw = reinterpret_cast<float*>(part + 2);  // [2][HID]: b1, W2
    int* rsc = reinterpret_cast<int*>(bw + 2 * HID);  // F16: [2][TR] feature-row scale exponents
    if (threadIdx.x < HID) {
        bw[threadIdx.x] = b1[threadIdx.x];
        bw[HID + threadIdx.x] = W2[threadIdx.x];
    }
    const float bias2 = b2[0];
    const uint32_t key = lg_dropout_key_dev(seed, salt), thr = lg_keep_threshold16(p_drop);
    const int arow = threadIdx.x / G::F4, af = threadIdx.x % G::F4;  // gather slot of this thread
    const int64_t step = gridDim.x;
    // Software pipeline, one barrier per tile: while tile i's MFMAs run on feature image
    // i&1, the wave splits tile i+1's endpoint rows into image (i+1)&1.  Rows are loaded
    // three tiles ahead into two alternating register sets, node ids two tiles before their
    // rows (one pair per set), so issuing a tile's row loads never waits on the id load
    // issued just before it.
    uint32_t nu, nv, nua, nva, nub = 0, nvb = 0;
    f32x4 pu0, pv0, pu1, pv1;
    auto rowof = [&](int64_t t) { return t * G::TR + arow; };
    int srow = 0;  // F16: the row scale of the tile being staged (set by its first third)
    auto stage = [&](uint16_t* img, int part3, const f32x4& pu, const f32x4& pv) {  // a third of the slot
        if (lab & 4) return;
        if constexpr (F16) {
            if (part3 == 0) {
                uint32_t m = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    m = max(m, max(__float_as_uint(fabsf(pu[i])),
                                   max(__float_as_uint(fabsf(pv[i])), __float_as_uint(fabsf(pu[i] - pv[i])))));
                srow = lg_f16_scale_exp_c(lg_row16_max_bits(m));
                if (af == 0) rsc[(img == fimg ? 0 : 1) * G::TR + arow] = srow;
            }
            const float sc = lg_pow2f(srow);
            if (part3 == 0) st_split2h(img, G::FPL, arow * G::FSB + 4 * af, pu, sc);
            if (part3 == 1) st_split2h(img, G::FPL, arow * G::FSB + D + 4 * af, pv, sc);
            if (part3 == 2) {
                f32x4 a;
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = fabsf(pu[i] - pv[i]);
                st_split2h(img, G::FPL, arow * G::FSB + 2 * D + 4 * af, a, sc);
            }
            return;
        }
        if (part3 == 0) st_split4<BF>(img, G::FPL, arow * G::FSB + 4 * af, pu);
        if (part3 == 1) st_split4<BF>(img, G::FPL, arow * G::FSB + D + 4 * af, pv);
        if (part3 == 2) {
            f32x4 a;
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = fabsf(pu[i] - pv[i]);
            st_split4<BF>(img, G::FPL, arow * G::FSB + 2 * D + 4 * af, a);
        }
    };
    const int64_t t0 = blockIdx.x;
    load_ends(ends, rowof(t0), BP, fdP, nu, nv);
    load_rows<D>(h, rowof(t0), BP, fdP, nu, nv, sb, sn, af, pu0, pv0);
    stage(fimg, 0, pu0, pv0);
    stage(fimg, 1, pu0, pv0);
    stage(fimg, 2, pu0, pv0);
    load_ends(ends, rowof(t0 + step), BP, fdP, nu, nv);
    load_rows<D>(h, rowof(t0 + step), BP, fdP, nu, nv, sb, sn, af, pu0, pv0);
    load_ends(ends, rowof(t0 + 2 * step), BP, fdP, nu, nv);
    load_rows<D>(h, rowof(t0 + 2 * step), BP, fdP, nu, nv, sb, sn, af, pu1, pv1);
    // BF (two workgroups per CU, 128 VGPRs): one shared id pair, a tile ahead of its rows
    constexpr int IDA = BF ? 4 : 5;  // the id pair refilled in a body is tile + IDA step's
    load_ends(ends, rowof(t0 + 3 * step), BP, fdP, nua, nva);
    if constexpr (!BF) load_ends(ends, rowof(t0 + 4 * step), BP, fdP, nub, nvb);
    __syncthreads();
    // tile: this iteration's tile; (pu, pv): tile + step's rows, refilled with tile + 3 step's
    // (ids (eu, ev), refilled with tile + 5 step's)
    auto body = [&](int64_t tile, int buf, f32x4& pu, f32x4& pv, uint32_t& eu, uint32_t& ev) {
        const int64_t row0 = tile * G::TR;
        const uint16_t* cur = fimg + buf * 3 * G::FPL;
        uint16_t* nxt = fimg + (buf ^ 1) * 3 * G::FPL;
        f32x4 acc[RBF][2];
#pragma unroll
        for (int rb = 0; rb < RBF; ++rb) {
            if constexpr (F16) {  // bias after the unscale
                acc[rb][0] = acc[rb][1] = f32x4{0.f, 0.f, 0.f, 0.f};
                continue;
            }
            acc[rb][0] = ld4(bw + 32 * nh + 4 * q);
            acc[rb][1] = ld4(bw + 32 * nh + 16 + 4 * q);
        }
#pragma unroll
        for (int ks = 0; ks < G::KS; ++ks) {
#pragma unroll
            for (int rb = 0; rb < RBF; ++rb) {
                const uint16_t* src = cur + (16 * (RBF * rh + rb) + c) * G::FSB + 32 * ks + 8 * q;
                if constexpr (F16) {
                    const lg_f16x8 bh[2] = {__builtin_bit_cast(lg_f16x8, lds_frag_row(src)),
                                            __builtin_bit_cast(lg_f16x8, lds_frag_row(src + G::FPL))};
                    acc[rb][0] = mfma_f16x2(wh[0][ks], bh, acc[rb][0]);
                    acc[rb][1] = mfma_f16x2(wh[1][ks], bh, acc[rb][1]);
                } else {
                    const lg_bf16x8 bf[3] = {lds_frag_row(src), lds_frag_row(src + G::FPL), lds_frag_row(src + 2 * G::FPL)};
                    if (lab & 1) {
                        acc[rb][0][0] += bf[0][0];
                        continue;
                    }
                    acc[rb][0] = mfma_prec<BF>(wa[0][ks], bf, acc[rb][0]);
                    acc[rb][1] = mfma_prec<BF>(wa[1][ks], bf, acc[rb][1]);
                }
            }
            // the next tile's split, spread over the MFMA stream
            if (ks * 3 / G::KS != (ks + 1) * 3 / G::KS) stage(nxt, ks * 3 / G::KS, pu, pv);
        }
        if (!(lab & 2)) {
            load_rows<D>(h, rowof(tile + 3 * step), BP, fdP, eu, ev, sb, sn, af, pu, pv);
            load_ends(ends, rowof(tile + IDA * step), BP, fdP, eu, ev);
        }
#pragma unroll
        for (int rb = 0; rb < RBF; ++rb) {
            const int row = 16 * (RBF * rh + rb) + c;
            const int64_t r = row0 + row;
            if constexpr (F16) {  // unscale (exact) and the bias in one rounding
                const float us = lg_pow2f(-(sw + rsc[buf * G::TR + row]));
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x4 bv = ld4(bw + 32 * nh + 16 * i + 4 * q);
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) acc[rb][i][reg] = fmaf(acc[rb][i][reg], us, bv[reg]);
                }
            }
            // row-stream dropout (oracle/dropout_ref.py edge_stream_mask): one stream per
            // (row, 4 nh + q), one xorshift step per pair of this lane's 8 units
            uint32_t st = dropout ? lg_row_stream_seed(key, static_cast<uint64_t>(r), 4 * nh + q) : 0u;
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                f32x4 hv;
                const f32x4 w2v = ld4(bw + HID + 32 * nh + 16 * i + 4 * q);
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) {
                    float v = fmaxf(acc[rb][i][reg], 0.f);
                    if (dropout) {
                        if ((reg & 1) == 0) st = lg_xorshift32(st);
                        const uint32_t u16 = (reg & 1) ? (st >> 16) : (st & 0xFFFFu);
                        v = u16 >= thr ? v * dscale : 0.f;
                    }
                    hv[reg] = v;
                    s = fmaf(v, w2v[reg], s);
                }
                if (hid_out && r < BP) {  // the activation cache policy when 32-bit offsets reach
                    const uint32_t e = static_cast<uint32_t>(r) * HID + 32 * nh + 16 * i + 4 * q;
                    if (hbuf) st4_act(hrs, e, hv);
                    else st4(hid_out + e, hv);
                }
            }
            s += __shfl_xor(s, 16);
            s += __shfl_xor(s, 32);
            if (q == 0) part[buf][nh][row] = s;
        }
        __syncthreads();  // image buf^1 complete, image buf free, partial logits of this tile posted
        if (threadIdx.x < G::TR) {
            const int64_t r = row0 + threadIdx.x;
            const float(&pp)[4][G::TR] = part[buf];
            const float tot = (pp[0][threadIdx.x] + pp[1][threadIdx.x]) + (pp[2][threadIdx.x] + pp[3][threadIdx.x]);
            if (r < BP) logit[lg_row_index(r, fdP, ldo)] = tot + bias2;
        }
    };
    // unconditional pairs (a conditional second body merges both paths' pending loads at the
    // loop head, and the compiler then waits for all of them), the odd tail after the loop
    int64_t tile = t0;
    for (; tile + step < ntiles; tile += 2 * step) {
        body(tile, 0, pu0, pv0, nua, nva);
        if constexpr (BF) body(tile + step, 1, pu1, pv1, nua, nva);
        else body(tile + step, 1, pu1, pv1, nub, nvb);
    }
    if (tile < ntiles) body(tile, 0, pu0, pv0, nua, nva);
}

// The pipe scatter fused into the backward (SCAT): each workgroup owns whole windows (its tiles
// are the window's pipe rows, 32 at a time from the window start) and, after a window's last
// tile, sums that window's node gradients dh[n] = dpool / N + sum over the incidences of n (item
// order) of dpipe[window][p][role] — the arithmetic of k_pipe_scatter — from the per-pipe rows
// it has just written (L2 / Infinity Cache, not HBM); the incidence CSR is staged in LDS.
struct EdgeScatter {
    const int32_t* inc_rowptr;
    const int32_t* inc_item;
    const float* dpool;  // [B][D] or null
    float* dh;
    uint32_t N, P, B;
    int nm;   // dh node-major ([N][B][D]) or window-major
    int tpw;  // tiles per window
    // STREAM (the pipe schedule of lg_pipe_schedule_build): pipe rows in schedule order, a
    // block of scatter events per tile, the nodes without pipes
    const int4* spipe;       // [P] {u, v, p, 0} in schedule order
    const uint32_t* sblk;    // [tpw][bw] {count, 0, events [maxev][2], incidence bytes [2 TR]}
    const int32_t* szero;    // [nzero]
    int nzero, nslots, bw, maxev;
    int lab;  // kernel-lab builds only (LG_KERNEL_LAB; results WRONG when set): 1 skip dW1 MFMA, 2 skip dfeat MFMA, 4 skip the streamed scatter
    // POOL (lg_heads_bwd_scatter, STREAM only): the NoLeakHead backward of the workgroup's windows
    // in its prologue (k_pool_head_bwd's arithmetic), dpool written to the `dpool` scratch above
    const float* pooled = nullptr;  // [B][D]
    const float* nhid = nullptr;    // [B][HID] the NoLeakHead's saved hidden layer
    const float* nW1 = nullptr;     // [HID][D]
    const float* nw2 = nullptr;     // [HID]
    float nscale = 1.f;             // its dropout scale
    float* nslab = nullptr;         // per workgroup: [dW1 HID * D][db1 HID][dw2 HID]
    double* ndslab = nullptr;       // per workgroup: db2
    lg_fastdiv fdT{};               // division by tpw (SCAT / STREAM tile -> window, slot)
};

// dh rows of window `win` (SCAT): node n = a slot of 16 (D = 64) lanes, kScatNodes nodes per lane
// group in flight, the first four incidences of each in one batch; the same sums, in the same
// order, as k_pipe_scatter (heads.hip).
// The scatter is latency-bound (each round: CSR from LDS, rows from L2, sum, store), so the
// number of nodes in flight sets its time; it is limited by the registers live beside it.
// Inside the tile loop (a window that is not the workgroup's last) the split W1 and the dW1
// accumulators are live: kScatNodesLoop.  The last window is scattered after the loop, once the
// weight-gradient slab is written and those registers are dead: kScatNodesTail.
constexpr int kScatNodesLoop = 2;  // 11 dependent rounds per window at L-TOWN-A
#ifndef LG_SCAT_NODES_TAIL
#define LG_SCAT_NODES_TAIL 8
#endif
constexpr int kScatNodesTail = LG_SCAT_NODES_TAIL;  // 3 rounds
template <int D, int kScatNodes>
__device__ __forceinline__ void edge_scatter_window(const EdgeScatter& sc, const int32_t* icsr, const float* dpipe,
                                                    uint32_t win) {
    constexpr int LPR = D / 4, SLOTS = NT / LPR;
    const int sr = threadIdx.x / LPR, sf = threadIdx.x % LPR;
    const float fN = static_cast<float>(sc.N);
    const int32_t* item = icsr + sc.N + 1;
    f32x4 g0 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (sc.dpool) {
        const f32x4 g = ld4(sc.dpool + static_cast<int64_t>(win) * D + 4 * sf);
#pragma unroll
        for (int c = 0; c < 4; ++c) g0[c] = g[c] / fN;
    }
    const float* dp = dpipe + static_cast<int64_t>(win) * sc.P * 2 * D + 4 * sf;
    for (uint32_t n0 = 0; n0 < sc.N; n0 += SLOTS * kScatNodes) {
        int e0[kScatNodes], e1[kScatNodes];
        f32x4 v[kScatNodes][4];
#pragma unroll
        for (int j = 0; j < kScatNodes; ++j) {
            const uint32_t n = n0 + SLOTS * j + sr;
            e0[j] = n < sc.N ? icsr[n] : 0;
            e1[j] = n < sc.N ? icsr[n + 1] : 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int it = e0[j] + u < e1[j] ? item[e0[j] + u] : 0;  // 2 p + role
                v[j][u] = e0[j] + u < e1[j] ? ld4(dp + static_cast<int64_t>(it) * D) : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int j = 0; j < kScatNodes; ++j) {
            const uint32_t n = n0 + SLOTS * j + sr;
            if (n >= sc.N) continue;
            f32x4 acc = g0;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (e0[j] + u < e1[j]) acc += v[j][u];
            for (int e = e0[j] + 4; e < e1[j]; ++e) acc += ld4(dp + static_cast<int64_t>(item[e]) * D);
            const int64_t row = sc.nm ? static_cast<int64_t>(n) * sc.B + win : static_cast<int64_t>(win) * sc.N + n;
            st4(sc.dh + row * D + 4 * sf, acc);
        }
    }
}

// STREAM: the node gradients summed tile by tile (lg_pipe_schedule_build).  Pipes are visited
// in a bandwidth-reducing order, so a node's incidences fall in a few consecutive tiles; after
// a tile's dfeat rows are in LDS (they never go to HBM), each node it touches adds them to its
// running sum — a slot of LDS between its first and last tile, the HBM row at its last tile.
// The running sum starts from dpool / N and adds the incidences in schedule order: the order
// of the schedule's incidence CSR, so the sums are those of lg_pipe_scatter_bwd over it.
// Event word 0: node | first << 24 | last << 25; word 1: slot | start << 16 | count << 24.
// An event per D / 8 lanes, 8 channels a lane (two float4, halves D / 2 apart): the 2 TR events
// a tile can have (NT / (D / 8) = 2 TR slots) in ONE round.  g0l: the window's dpool / N row.
template <int D>
__device__ __forceinline__ void edge_stream_scatter(const EdgeScatter& sc, const uint32_t* eb, const float* dpl,
                                                    float* lacc, const float* g0l, uint32_t win, int DPS) {
    constexpr int LPE = D / 8;
    static_assert(NT / LPE == 2 * EG<D>::TR, "one round of events");
    const int e = threadIdx.x / LPE, c0 = 4 * (threadIdx.x % LPE), c1 = c0 + D / 2;
    const int ne = static_cast<int>(eb[0]);
    const uint8_t* incl = reinterpret_cast<const uint8_t*>(eb + 2 + 2 * sc.maxev);
    if (e < ne) {
        const uint32_t w0 = eb[2 + 2 * e], w1 = eb[3 + 2 * e];
        const uint32_t node = w0 & 0xFFFFFFu, slot = w1 & 0xFFFFu, st = (w1 >> 16) & 0xFFu, cnt = w1 >> 24;
        const float* src = (w0 >> 24) & 1u ? g0l : lacc + slot * D;
        f32x4 a0 = ld4(src + c0), a1 = ld4(src + c1);
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t b = incl[st + i];  // 2 row + role
            const float* r = dpl + (b >> 1) * DPS + (b & 1u) * D;
            a0 += ld4(r + c0);
            a1 += ld4(r + c1);
        }
        if ((w0 >> 25) & 1u) {  // the node's last tile: its dh row (activation cache policy, common.h)
            const int64_t row = sc.nm ? static_cast<int64_t>(node) * sc.B + win : static_cast<int64_t>(win) * sc.N + node;
            if (static_cast<int64_t>(sc.B) * sc.N * D < (int64_t{1} << 29)) {
                const __amdgpu_buffer_rsrc_t dhr = lg_act_rsrc(sc.dh, static_cast<int64_t>(sc.B) * sc.N * D);
                st4_act<LG_EDGE_DH_AUX>(dhr, static_cast<uint32_t>(row * D) + c0, a0);
                st4_act<LG_EDGE_DH_AUX>(dhr, static_cast<uint32_t>(row * D) + c1, a1);
            } else {
                st4(sc.dh + row * D + c0, a0);
                st4(sc.dh + row * D + c1, a1);
            }
        } else {
            float* dst = lacc + slot * D;
            st4(dst + c0, a0);
            st4(dst + c1, a1);
        }
    }
}
// the window's nodes without pipes: dh = dpool / N
template <int D>
__device__ __forceinline__ void edge_stream_zero(const EdgeScatter& sc, const float* g0l, uint32_t win) {
    constexpr int LPE = D / 8, SLOTS = NT / LPE;
    const int e = threadIdx.x / LPE, c0 = 4 * (threadIdx.x % LPE), c1 = c0 + D / 2;
    for (int i = e; i < sc.nzero; i += SLOTS) {
        const uint32_t node = static_cast<uint32_t>(sc.szero[i]);
        const int64_t row = sc.nm ? static_cast<int64_t>(node) * sc.B + win : static_cast<int64_t>(win) * sc.N + node;
        st4(sc.dh + row * D + c0, ld4(g0l + c0));
        st4(sc.dh + row * D + c1, ld4(g0l + c1));
    }
}

// slab per workgroup: [dW1 128*K3][db1 128][dW2 128][db2 1]
// MODE 0: dpipe rows only; 1 (SCAT): + each window's node sums from its dpipe rows; 2
// (STREAM): the node sums streamed per tile, no dpipe rows
// F16 (the fp32 tier's default): both products on the 2-way f16 split (3 f16 MFMAs per product
// instead of 6 bf16 ones) with power-of-two scales that keep the dfeat rows independent of
// which rows share their tile (bit-identical results across MODEs):
//   g rows scaled per ROW by 2^sg(row), from |dlogit(row)| max|W2| dscale (a bound on the row's
//     |g|): dfeat^T = W1^T g^T contracts over hidden units, so a per-row (column) scale is
//     allowed; W1^T scaled per wave by 2^sW; each wave unscales its partial by 2^-(sW + sg);
//   dW1 = g^T feat contracts over rows: the feature rows are scaled by 2^(T - sg(row)), T per
//     tile = min over its rows of sf(row) + sg(row) (sf from the row's max |feature|), so every
//     row's products carry 2^T and the tile's dW1 block is added times 2^-T.  T is reduced
//     (LDS atomic min) from the tile's loaded rows before the previous tile's second barrier.
template <int D, bool BF, int MODE = 0, bool F16 = false>
__global__ void __launch_bounds__(NT)
k_edge_bwd(const int64_t* __restrict__ ends, const float* __restrict__ h, const float* __restrict__ W1,
           const float* __restrict__ W2, const float* __restrict__ hid, const float* __restrict__ dlogit, int64_t ldo,
           float* __restrict__ dpipe, float* __restrict__ slab, double* __restrict__ db2slab, uint32_t sb,
           uint32_t sn, lg_fastdiv fdP, int64_t BP, int64_t ntiles, float dscale, EdgeScatter sc) {
    using G = EG<D>;
    static_assert(!(F16 && BF), "one transform");
    constexpr bool SCAT = MODE == 1, STREAM = MODE == 2, WIN = MODE != 0;  // WIN: workgroups own windows
    constexpr int SL = (HID * G::K3 + 2 * HID + 1 + 3) & ~3;  // rows padded to 16 bytes (the reduce's vector loads)
    constexpr int NPL = F16 ? 2 : 3;  // image planes
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if constexpr (STREAM) {
        if (sc.nslab) {
            // NoLeakHead backward (k_pool_head_bwd, pool.hip: the same sums in the same order) for
            // the windows this workgroup owns, before the images take the LDS:
            //   dhid = dlogit[b][P] * w2 * scale * [hid > 0],  dpool[b] = dhid W1 (fixed kk order),
            //   the slab row: dW1 += dhid pooled[b]^T, db1 += dhid, dw2 += dlogit[b][P] hid, db2 (fp64)
            constexpr int WS = D + 1, DQ = D / 4;
            static_assert(NT == 4 * HID, "four column quarters per hidden unit");
            float* w1l = reinterpret_cast<float*>(smem);  // [HID][WS]
            float* dhl = w1l + HID * WS;                   // [HID]
            float* pl = dhl + HID;                         // [D]
            for (int i = threadIdx.x; i < HID * D; i += NT) w1l[(i / D) * WS + (i % D)] = sc.nW1[i];
            const int k = threadIdx.x % HID, dq = threadIdx.x / HID;
            const float w2k = sc.nw2[k];
            float dw1n[DQ];
#pragma unroll
            for (int d = 0; d < DQ; ++d) dw1n[d] = 0.f;
            float db1n = 0.f, dw2n = 0.f;
            double db2n = 0.0;
            for (int64_t b = blockIdx.x; b < sc.B; b += gridDim.x) {
                const float dout = dlogit[b * ldo + sc.P];
                const float hk = sc.nhid[b * HID + k];
                if (threadIdx.x < D) pl[threadIdx.x] = sc.pooled[b * D + threadIdx.x];
                const float dhk = hk > 0.f ? dout * w2k * sc.nscale : 0.f;
                if (dq == 0) {
                    dhl[k] = dhk;
                    db1n += dhk;
                    dw2n = fmaf(dout, hk, dw2n);
                    if (k == 0) db2n += static_cast<double>(dout);
                }
                __syncthreads();  // pl, dhl (and on the first pass w1l) visible
#pragma unroll
                for (int d = 0; d < DQ; ++d) dw1n[d] = fmaf(dhk, pl[dq * DQ + d], dw1n[d]);
                if (threadIdx.x < D) {
                    float sdp = 0.f;
#pragma unroll 16
                    for (int kk = 0; kk < HID; ++kk) sdp = fmaf(dhl[kk], w1l[kk * WS + threadIdx.x], sdp);
                    const_cast<float*>(sc.dpool)[b * D + threadIdx.x] = sdp;  // read back by this workgroup's tiles
                }
                __syncthreads();
            }
            float* out = sc.nslab + static_cast<int64_t>(blockIdx.x) * (HID * D + 2 * HID);
#pragma unroll
            for (int d = 0; d < DQ; ++d) out[k * D + dq * DQ + d] = dw1n[d];
            if (dq == 0) {
                out[HID * D + k] = db1n;
                out[HID * D + HID + k] = dw2n;
            }
            if (threadIdx.x == 0) sc.ndslab[blockIdx.x] = db2n;
            __syncthreads();  // the LDS goes to the images
        }
    }
    uint16_t* fimg = reinterpret_cast<uint16_t*>(smem);     // [NPL][TR][FTB]  feat parts
    uint16_t* gimg = fimg + NPL * G::FTPL;                   // [NPL][TR][GSB]  g parts
    int8_t* sgn = reinterpret_cast<int8_t*>(gimg + NPL * G::GPL);  // [2][TR][D]  sign(h_u - h_v), by tile parity
    f32x4* red = reinterpret_cast<f32x4*>(sgn + 2 * G::TR * D);  // [2][NROLE][3][64] dfeat partials
    int* rsg = reinterpret_cast<int*>(red + 2 * G::NROLE * 3 * 64);  // F16: [2][TR] row g scales, by tile parity
    int* tmn = rsg + 2 * G::TR;                                       // F16: [2] tile product scales T
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
    const int tq = (lane >> 2) & 3, tp = lane & 3;  // transposed-read address slot of this lane
    // dfeat roles: features 16 kt + [0,16) of u, v, |u-v|, hidden half hh, row group rg
    const int kt = w % G::DT, hh = (w / G::DT) & 1, rg = w / (2 * G::DT);
    // A operand of dfeat^T = W1^T g^T: A[k = 16(kt + DT s3) + c][n = 64hh + 32ks + 8q + j] = W1[n][k]
    lg_bf16x8 wt[3][2][3];
    lg_f16x8 wh[3][2][2];
    int sW = 0;  // F16: this wave's W1^T scale exponent
    {
        f32x4 wx[3][2][2];
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const float* src = W1 + (64 * hh + 32 * ks + 8 * q) * G::K3 + 16 * (kt + G::DT * s3) + c;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    wx[s3][ks][0][j] = src[j * G::K3];
                    wx[s3][ks][1][j] = src[(j + 4) * G::K3];
                }
            }
        if constexpr (F16) {
            uint32_t m = 0;
#pragma unroll
            for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
                        for (int j = 0; j < 4; ++j) m = max(m, __float_as_uint(fabsf(wx[s3][ks][h2][j])));
            sW = lg_f16_scale_exp_c(lg_wave_max_bits(m));
            const float sc = lg_pow2f(sW);
#pragma unroll
            for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
                    split2_f16_x8(wx[s3][ks][0] * sc, wx[s3][ks][1] * sc, wh[s3][ks][0], wh[s3][ks][1]);
        } else {
#pragma unroll
            for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
                    split3_x8(wx[s3][ks][0], wx[s3][ks][1], wt[s3][ks][0], wt[s3][ks][1], wt[s3][ks][2]);
        }
    }
    const int arow = threadIdx.x / G::F4, af = threadIdx.x % G::F4;  // feature gather slot
    const int n4 = threadIdx.x & 31, hrow = threadIdx.x >> 5;        // hidden slot: rows hrow + 16 i
    const f32x4 w2g = ld4(W2 + 4 * n4);
    // F16: max |W2| (each wave's lanes 0-31 hold all of W2) times the dropout scale: the row
    // g bound is |dlogit(row)| w2m
    float w2m = 0.f;
    if constexpr (F16) {
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) m = max(m, __float_as_uint(fabsf(w2g[j])));
        w2m = __uint_as_float(lg_wave_max_bits(m)) * dscale;
    }
    auto row_gscale = [&](float dlv) { return lg_f16_scale_exp_c(__float_as_uint(fabsf(dlv) * w2m)); };
    f32x4 dwa[G::KT];
#pragma unroll
    for (int i = 0; i < G::KT; ++i) dwa[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dw2a = f32x4{0.f, 0.f, 0.f, 0.f};
    // db1 / db2 are sums of dlogit-weighted terms that cancel heavily (the dlogits of one
    // window sum to ~0 under the CE gradient): kept in fp64 end to end
    double db1a[4] = {0.0, 0.0, 0.0, 0.0};
    double db2 = 0.0;
    int tcur = 0;  // F16: dwa is dW1 x 2^tcur

    // this workgroup's k-th tile: tile blockIdx.x + k gridDim.x of the (B, P) row space, or
    // (SCAT) tile k % tpw of window blockIdx.x + (k / tpw) gridDim.x; rows [rbase, rlim) count
    const int64_t gstep = gridDim.x;
    // WIN: tile k -> (its window's rank kq(k) among this workgroup's windows, its tile kr(k) within
    // the window), on 32-bit fastdiv (a 64-bit division by the runtime tpw was ~60 scalar
    // instructions, evaluated several times per tile: 6,565 SALU per wave, PMC r04 / r05)
    auto kq = [&](int64_t k) -> uint32_t { return lg_div(static_cast<uint32_t>(k), sc.fdT); };
    auto kr = [&](int64_t k) -> uint32_t { return static_cast<uint32_t>(k) - kq(k) * static_cast<uint32_t>(sc.tpw); };
    auto kwin = [&](int64_t k) -> uint32_t { return blockIdx.x + kq(k) * static_cast<uint32_t>(gstep); };
    auto rbase = [&](int64_t k) -> int64_t {
        if constexpr (WIN) return static_cast<int64_t>(kwin(k)) * sc.P + kr(k) * G::TR;
        return (blockIdx.x + k * gstep) * G::TR;
    };
    auto rlim = [&](int64_t k) -> int64_t {
        if constexpr (WIN) return std::min<int64_t>(BP, (static_cast<int64_t>(kwin(k)) + 1) * sc.P);
        return BP;
    };
    const int64_t nk = WIN ? (blockIdx.x < sc.B ? sc.tpw * ((sc.B - blockIdx.x + gstep - 1) / gstep) : 0)
                            : (blockIdx.x < ntiles ? (ntiles - blockIdx.x + gstep - 1) / gstep : 0);
    uint32_t nu, nv;
    f32x4 pu, pv, hp[G::HPT];
    float dl[G::HPT];
    // STREAM: rows are schedule slots; row off of tile k -> (window, slot), (0, 0) past the window
    const uint32_t* spw = reinterpret_cast<const uint32_t*>(sc.spipe);
    auto sslot = [&](int64_t k, int off, uint32_t& b, uint32_t& slot) {
        const int64_t r = rbase(k) + off;
        const bool ok = r < rlim(k);
        b = ok ? kwin(k) : 0u;
        slot = ok ? static_cast<uint32_t>(r - static_cast<int64_t>(b) * sc.P) : 0u;
    };
    uint32_t hpipe[G::HPT];  // STREAM: pipe ids of the hidden-slot rows, a tile ahead of their loads
    uint32_t apipe = 0;      // STREAM + F16: pipe id of the feature row
    float dla = 0.f;         // F16: dlogit of the feature row (its g scale)
    auto load_ids = [&](int64_t k) {
        if constexpr (STREAM) {
            uint32_t b, slot;
            sslot(k, arow, b, slot);
            nu = spw[4 * slot];
            nv = spw[4 * slot + 1];
            if constexpr (F16) apipe = spw[4 * slot + 2];
#pragma unroll
            for (int i = 0; i < G::HPT; ++i) {
                sslot(k, hrow + 16 * i, b, slot);
                hpipe[i] = spw[4 * slot + 2];
            }
        } else {
            load_ends(ends, rbase(k) + arow, BP, fdP, nu, nv);
        }
    };
    auto load_feat = [&](int64_t k) {
        if constexpr (STREAM) {
            uint32_t b, slot;
            sslot(k, arow, b, slot);
            pu = ld4(h + ((b * sb + nu * sn) * D + 4 * af));
            pv = ld4(h + ((b * sb + nv * sn) * D + 4 * af));
        } else {
            load_rows<D>(h, rbase(k) + arow, BP, fdP, nu, nv, sb, sn, af, pu, pv);
        }
    };
    auto load_hid = [&](int64_t k) {  // raw (see load_ends); a row past the end is zeroed at use
#pragma unroll
        for (int i = 0; i < G::HPT; ++i) {
            if constexpr (STREAM) {
                uint32_t b, slot;
                sslot(k, hrow + 16 * i, b, slot);
                hp[i] = ld4(hid + ((b * sc.P + hpipe[i]) * HID + 4 * n4));
                dl[i] = dlogit[static_cast<int64_t>(b) * ldo + hpipe[i]];
            } else {
                const uint32_t r = clamp_row(rbase(k) + hrow + 16 * i, BP);
                hp[i] = ld4(hid + (r * HID + 4 * n4));
                dl[i] = dlogit[lg_row_index(r, fdP, ldo)];
            }
        }
        if constexpr (F16) {
            if constexpr (STREAM) {
                uint32_t b, slot;
                sslot(k, arow, b, slot);
                dla = dlogit[static_cast<int64_t>(b) * ldo + apipe];
            } else {
                dla = dlogit[lg_row_index(clamp_row(rbase(k) + arow, BP), fdP, ldo)];
            }
        }
    };
    // F16: tile k's product scale candidate of this thread's feature row (pu, pv, dla hold
    // tile k's row), min-reduced over the workgroup into tmn[k & 1]
    auto post_tile_scale = [&](int64_t k) {
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            m = max(m, max(__float_as_uint(fabsf(pu[i])), max(__float_as_uint(fabsf(pv[i])),
                                                              __float_as_uint(fabsf(pu[i] - pv[i])))));
        // a row without gradient (past the end, or dlogit 0) contributes nothing to dW1 and must not
        // lower T (its zero g leaves its features free: they are staged as zeros)
        const float dlv = rbase(k) + arow < rlim(k) ? dla : 0.f;
        const int sfe = lg_f16_scale_exp_c(lg_rowgroup_max_bits<D>(m));
        const int cand = lg_wave_min_i32(dlv != 0.f ? sfe + row_gscale(dlv) : 0x7FFFFFFF);
        if (lane == 0) __hip_atomic_fetch_min(&tmn[k & 1], cand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // SCAT: the incidence CSR in LDS (after the kernel's images), staged before the first barrier
    constexpr int64_t BASE = G::bwd_lds(F16);
    int32_t* icsr = reinterpret_cast<int32_t*>(smem + BASE);
    if constexpr (SCAT) {
        for (uint32_t i = threadIdx.x; i <= sc.N; i += NT) icsr[i] = sc.inc_rowptr[i];
        for (uint32_t i = threadIdx.x; i < 2 * sc.P; i += NT) icsr[sc.N + 1 + i] = sc.inc_item[i];
    }
    // STREAM: after the images, the tile's dfeat rows [TR][DPS] (du | dv), the event blocks of
    // two tiles, the open nodes' running sums [nslots][D]
    constexpr int DPS = 2 * D + 4;  // row stride: the finishing waves' 16-row stores conflict-free
    float* dpl = reinterpret_cast<float*>(smem + BASE);
    uint32_t* evb = reinterpret_cast<uint32_t*>(dpl + G::TR * DPS);
    float* g0l = reinterpret_cast<float*>(evb + 2 * sc.bw);  // [D] dpool / N of the window scattered next
    float* lacc = g0l + D;
    const int sf = threadIdx.x % (D / 4);
    const float fN = static_cast<float>(sc.N);
    const float* gsrc = sc.dpool ? sc.dpool : h;  // h: any readable row when there is no pool gradient
    f32x4 graw = f32x4{0.f, 0.f, 0.f, 0.f};  // raw dpool row of the window of the tile scattered next
    uint2 evn = uint2{0u, 0u};  // the next tile's event block, a uint2 per thread
    auto load_evblock = [&](int64_t k) {
        const int t = min(static_cast<int>(threadIdx.x), sc.bw / 2 - 1);
        evn = reinterpret_cast<const uint2*>(sc.sblk + kr(k) * sc.bw)[t];
    };
    auto store_evblock = [&](int64_t k) {
        if (static_cast<int>(threadIdx.x) < sc.bw / 2) reinterpret_cast<uint2*>(evb + (k & 1) * sc.bw)[threadIdx.x] = evn;
    };
    auto scatter_tile = [&](int64_t kk) {
        const uint32_t win = kwin(kk);
        edge_stream_scatter<D>(sc, evb + (kk & 1) * sc.bw, dpl, lacc, g0l, win, DPS);
        if (sc.nzero > 0 && kr(kk) == static_cast<uint32_t>(sc.tpw - 1)) edge_stream_zero<D>(sc, g0l, win);
    };
    auto post_g0 = [&]() {  // graw (this thread's 4 channels, threads < D / 4) -> g0l
        if (threadIdx.x < D / 4) {
            f32x4 g0 = f32x4{0.f, 0.f, 0.f, 0.f};
            if (sc.dpool) {
#pragma unroll
                for (int c2 = 0; c2 < 4; ++c2) g0[c2] = graw[c2] / fN;
            }
            st4(g0l + 4 * threadIdx.x, g0);
        }
    };
    auto load_graw = [&](int64_t k) {
        const uint32_t win = min(kwin(k), sc.B - 1);
        graw = ld4(gsrc + (sc.dpool ? static_cast<int64_t>(win) * D : 0) + 4 * sf);
    };
    load_ids(0);
    load_feat(0);
    load_hid(0);
    load_ids(1);
    if constexpr (STREAM) {
        load_evblock(0);
        store_evblock(0);
        load_graw(0);
    }
    if constexpr (F16) {  // tile 0's product scale (later tiles': posted during the tile before)
        if (threadIdx.x == 0) tmn[0] = tmn[1] = 0x7FFFFFFF;
        __syncthreads();
        if (nk > 0) post_tile_scale(0);
        __syncthreads();
    }
    int buf = 0;
    for (int64_t k = 0; k < nk; ++k, buf ^= 1) {
        const int64_t row0 = rbase(k), rend = rlim(k);
        int8_t* sgnb = sgn + buf * G::TR * D;
        int tT = 0;  // F16: the tile's product scale exponent T
        if constexpr (STREAM) post_g0();  // the window of tile k - 1, scattered after the barrier
        {
            f32x4 a;
            uint32_t sw = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float d = pu[i] - pv[i];
                a[i] = fabsf(d);
                sw |= static_cast<uint32_t>(static_cast<uint8_t>(d > 0.f ? 1 : (d < 0.f ? -1 : 0))) << (8 * i);
            }
            if constexpr (F16) {
                tT = tmn[buf];
                const float dlv = row0 + arow < rend ? dla : 0.f;
                const float fs = dlv != 0.f ? lg_pow2f(tT - row_gscale(dlv)) : 0.f;
                st_split2h(fimg, G::FTPL, arow * G::FTB + 4 * af, pu, fs);
                st_split2h(fimg, G::FTPL, arow * G::FTB + D + 4 * af, pv, fs);
                st_split2h(fimg, G::FTPL, arow * G::FTB + 2 * D + 4 * af, a, fs);
            } else {
                st_split4<BF>(fimg, G::FTPL, arow * G::FTB + 4 * af, pu);
                st_split4<BF>(fimg, G::FTPL, arow * G::FTB + D + 4 * af, pv);
                st_split4<BF>(fimg, G::FTPL, arow * G::FTB + 2 * D + 4 * af, a);
            }
            *reinterpret_cast<uint32_t*>(sgnb + arow * D + 4 * af) = sw;
        }
#pragma unroll
        for (int i = 0; i < G::HPT; ++i) {
            f32x4 g;
            const float dli = row0 + hrow + 16 * i < rend ? dl[i] : 0.f;  // rows past the end: no gradient
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                g[j] = hp[i][j] > 0.f ? dli * w2g[j] * dscale : 0.f;
                dw2a[j] = fmaf(dli, hp[i][j], dw2a[j]);
                db1a[j] += static_cast<double>(g[j]);
            }
            if (n4 == 0) db2 += static_cast<double>(dli);
            if constexpr (F16) {
                const int sg = row_gscale(dli);
                st_split2h(gimg, G::GPL, (hrow + 16 * i) * G::GSB + 4 * n4, g, lg_pow2f(sg));
                if (n4 == 0) rsg[buf * G::TR + hrow + 16 * i] = sg;
            } else {
                st_split4<BF>(gimg, G::GPL, (hrow + 16 * i) * G::GSB + 4 * n4, g);
            }
        }
        __syncthreads();
        if constexpr (F16) {
            if (threadIdx.x == 0) tmn[buf] = 0x7FFFFFFF;  // read above by every thread; tile k + 2's next
        }
        load_feat(k + 1);
        load_hid(k + 1);
        load_ids(k + 2);
        if constexpr (STREAM) load_evblock(k + 1);

        // dW1[n][k] += sum_rows g[row][n] feat[row][k]: n-tile w, every k-tile; the k (= row)
        // order inside a step is 4q + (j & 3) + 16 (j >> 2) in both operands
        if constexpr (F16) {  // dwa holds dW1 x 2^tcur: rescaled (exactly) when the tile's T differs
            if (tT != tcur && tT != 0x7FFFFFFF) {  // 0x7FFFFFFF: no row of the tile has a gradient
                const float rs = lg_pow2f(tT - tcur);
#pragma unroll
                for (int t = 0; t < G::KT; ++t) dwa[t] *= rs;
                tcur = tT;
            }
#pragma unroll
            for (int ks = 0; ks < G::TR / 32; ++ks) {
                const int r0 = 32 * ks + 4 * q + tq;
                lg_f16x8 ga[2];
#pragma unroll
                for (int pp = 0; pp < 2; ++pp) {
                    const uint16_t* src = gimg + pp * G::GPL + r0 * G::GSB + 16 * w + 4 * tp;
                    ga[pp] = __builtin_bit_cast(lg_f16x8, lds_frag_tr16(src, src + 16 * G::GSB));
                }
#pragma unroll
                for (int t = 0; t < G::KT; ++t) {
                    lg_f16x8 fb[2];
#pragma unroll
                    for (int pp = 0; pp < 2; ++pp) {
                        const uint16_t* src = fimg + pp * G::FTPL + r0 * G::FTB + 16 * t + 4 * tp;
                        fb[pp] = __builtin_bit_cast(lg_f16x8, lds_frag_tr16(src, src + 16 * G::FTB));
                    }
#ifdef LG_KERNEL_LAB
                    if (sc.lab & 1) {
                        dwa[t][0] += static_cast<float>(fb[0][0]) + static_cast<float>(ga[0][0]);
                        continue;
                    }
#endif
                    dwa[t] = mfma_f16x2(ga, fb, dwa[t]);
                }
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < G::TR / 32; ++ks) {
                const int r0 = 32 * ks + 4 * q + tq;
                lg_bf16x8 ga[3];
#pragma unroll
                for (int pp = 0; pp < 3; ++pp) {
                    const uint16_t* src = gimg + pp * G::GPL + r0 * G::GSB + 16 * w + 4 * tp;
                    ga[pp] = lds_frag_tr16(src, src + 16 * G::GSB);
                }
#pragma unroll
                for (int t = 0; t < G::KT; ++t) {
                    lg_bf16x8 fb[3];
#pragma unroll
                    for (int pp = 0; pp < 3; ++pp) {
                        const uint16_t* src = fimg + pp * G::FTPL + r0 * G::FTB + 16 * t + 4 * tp;
                        fb[pp] = lds_frag_tr16(src, src + 16 * G::FTB);
                    }
#ifdef LG_KERNEL_LAB
                    if (sc.lab & 1) {
                        dwa[t][0] += static_cast<float>(fb[0][0]) + static_cast<float>(ga[0][0]);
                        continue;
                    }
#endif
                    dwa[t] = mfma_prec<BF>(ga, fb, dwa[t]);
                }
            }
        }
        // STREAM: the previous tile's node sums (LDS reads and stores between the two MFMA
        // blocks, overlapping the dW1 chains in flight)
        if constexpr (STREAM) {
#ifdef LG_KERNEL_LAB
            if (k > 0 && !(sc.lab & 4)) scatter_tile(k - 1);
#else
            if (k > 0) scatter_tile(k - 1);
#endif
            load_graw(k);  // for this tile's, at the next one
        }
        // dfeat^T[k][row] = sum_n W1[n][k] g[row][n] over this wave's hidden half; partial
        // blocks role = (rg, kt, rbw) of both halves go to LDS
#pragma unroll
        for (int rbw = 0; rbw < G::RBW; ++rbw) {
            const int rowb = 16 * (rg * G::RBW + rbw);
            f32x4 cacc[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const uint16_t* src = gimg + (rowb + c) * G::GSB + 64 * hh + 32 * ks + 8 * q;
                if constexpr (F16) {
                    const lg_f16x8 gb[2] = {__builtin_bit_cast(lg_f16x8, lds_frag_row(src)),
                                            __builtin_bit_cast(lg_f16x8, lds_frag_row(src + G::GPL))};
#ifdef LG_KERNEL_LAB
                    if (sc.lab & 2) {
                        cacc[0][0] += static_cast<float>(gb[0][0]);
                        continue;
                    }
#endif
#pragma unroll
                    for (int s3 = 0; s3 < 3; ++s3) cacc[s3] = mfma_f16x2(wh[s3][ks], gb, cacc[s3]);
                } else {
                    const lg_bf16x8 gb[3] = {lds_frag_row(src), lds_frag_row(src + G::GPL), lds_frag_row(src + 2 * G::GPL)};
#ifdef LG_KERNEL_LAB
                    if (sc.lab & 2) {
                        cacc[0][0] += static_cast<float>(gb[0][0]);
                        continue;
                    }
#endif
#pragma unroll
                    for (int s3 = 0; s3 < 3; ++s3) cacc[s3] = mfma_prec<BF>(wt[s3][ks], gb, cacc[s3]);
                }
            }
            if constexpr (F16) {  // this half's partial unscaled: 2^-(sW + sg(row)), row = column c
                const float us = lg_pow2f(-(sW + rsg[buf * G::TR + rowb + c]));
#pragma unroll
                for (int s3 = 0; s3 < 3; ++s3) cacc[s3] *= us;
            }
            const int role = (rg * G::DT + kt) * G::RBW + rbw;
#pragma unroll
            for (int s3 = 0; s3 < 3; ++s3) red[((hh * G::NROLE + role) * 3 + s3) * 64 + lane] = cacc[s3];
        }
        if constexpr (F16) {
            if (k + 1 < nk) post_tile_scale(k + 1);  // pu, pv, dla hold tile k + 1's rows
        }
        __syncthreads();
        {
            // wave w finishes output block role = w: halves added in a fixed order
            const int rbw = w % G::RBW, kt2 = (w / G::RBW) % G::DT, rg2 = w / (G::RBW * G::DT);
            const int row = 16 * (rg2 * G::RBW + rbw) + c;
            const int64_t r = row0 + row;
            const f32x4* r0p = red + (w * 3) * 64 + lane;
            const f32x4* r1p = red + ((G::NROLE + w) * 3) * 64 + lane;
            const f32x4 cu = r0p[0] + r1p[0], cv = r0p[64] + r1p[64], ca = r0p[128] + r1p[128];
            const int ku = 16 * kt2 + 4 * q;
            const uint32_t sw = *reinterpret_cast<const uint32_t*>(sgnb + row * D + ku);
            // rend, not BP: (SCAT) a window's last tile runs past its P rows into the next window's,
            // which another workgroup owns and may already have written (with the real gradient)
            if (r < rend) {
                f32x4 du, dv;
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) {
                    const float sg = static_cast<float>(static_cast<int8_t>(sw >> (8 * reg)));
                    du[reg] = cu[reg] + sg * ca[reg];
                    dv[reg] = cv[reg] - sg * ca[reg];
                }
                float* o = STREAM ? dpl + (row * DPS + ku) : dpipe + (static_cast<uint32_t>(r) * 2 * D + ku);
                st4(o, du);
                st4(o + D, dv);
            }
            if constexpr (STREAM) store_evblock(k + 1);
        }
        if constexpr (SCAT) {
            if (kr(k) == static_cast<uint32_t>(sc.tpw - 1) && k + 1 < nk) {  // a window's last tile (not the workgroup's last window)
                __syncthreads();                            // every wave's dpipe rows of the window are stored
                edge_scatter_window<D, kScatNodesLoop>(sc, icsr, dpipe,
                                                       kwin(k));
            }
        }
    }

    float* out = slab + static_cast<int64_t>(blockIdx.x) * SL;
    if constexpr (F16) {
        const float us = lg_pow2f(-tcur);
#pragma unroll
        for (int t = 0; t < G::KT; ++t) dwa[t] *= us;
    }
#pragma unroll
    for (int t = 0; t < G::KT; ++t)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) out[(16 * w + 4 * q + reg) * G::K3 + 16 * t + c] = dwa[t][reg];
    // db1 / dW2: lanes l and l + 32 share n4, then the eight waves in order; db2 likewise
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        dw2a[j] += __shfl_xor(dw2a[j], 32);
        db1a[j] += __shfl_xor(db1a[j], 32);
    }
    db2 += __shfl_xor(db2, 32);
    __syncthreads();  // the last tile's LDS readers are done: reuse the partials area
    float* fin = reinterpret_cast<float*>(red);                  // [NW][32][4] dW2
    double* find = reinterpret_cast<double*>(fin + NW * 32 * 4);  // [NW][32][4] db1, [NW] db2
    if (lane < 32) {
        st4(fin + (w * 32 + lane) * 4, dw2a);
#pragma unroll
        for (int j = 0; j < 4; ++j) find[(w * 32 + lane) * 4 + j] = db1a[j];
    }
    if (lane == 0) find[NW * 32 * 4 + w] = db2;
    __syncthreads();
    if (threadIdx.x < 32) {
        f32x4 b = ld4(fin + threadIdx.x * 4);
        double a[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = find[threadIdx.x * 4 + j];
#pragma unroll
        for (int i = 1; i < NW; ++i) {
            b += ld4(fin + (i * 32 + threadIdx.x) * 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] += find[(i * 32 + threadIdx.x) * 4 + j];
        }
        st4(out + HID * G::K3 + 4 * threadIdx.x,
            f32x4{static_cast<float>(a[0]), static_cast<float>(a[1]), static_cast<float>(a[2]), static_cast<float>(a[3])});
        st4(out + HID * G::K3 + HID + 4 * threadIdx.x, b);
    }
    if (threadIdx.x == 0) {
        double s = find[NW * 32 * 4];
        for (int i = 1; i < NW; ++i) s += find[NW * 32 * 4 + i];
        db2slab[blockIdx.x] = s;
    }
    if constexpr (SCAT) {
        if (nk > 0) {  // the last window's node gradients (its dpipe rows were stored before the barriers above)
            __syncthreads();
            edge_scatter_window<D, kScatNodesTail>(sc, icsr, dpipe,
                                                   kwin(nk - 1));
        }
    }
    if constexpr (STREAM) {
        if (nk > 0) {  // the last tile's rows and events were stored before the barriers above
            post_g0();
            __syncthreads();
            scatter_tile(nk - 1);
        }
    }
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

#ifdef LG_KERNEL_LAB
inline int kEdgeLab(int flags) { return (flags >> 28) & 7; }
#else
inline int kEdgeLab(int) { return 0; }
#endif

// STREAM dynamic LDS: the images, the dfeat rows, two event blocks, the open nodes' sums
// the backward's transform: the f16x2 split on the fp32 tier unless LG_F_BF16X3 asks for the
// 3-way bf16 split; LG_F_BF16: one bf16 product
bool edge_bwd_f16(int flags) { return !(flags & LG_F_BF16) && !(flags & LG_F_BF16X3); }
int64_t edge_bwd_base_lds(int64_t D, int flags) {
    const bool f16 = edge_bwd_f16(flags);
    return D == 64 ? EG<64>::bwd_lds(f16) : EG<32>::bwd_lds(f16);
}
int64_t edge_stream_lds(int64_t D, int flags, const EdgeScatter& sc) {
    const int64_t base = edge_bwd_base_lds(D, flags), TR = 2048 / D;
    return base + TR * (2 * D + 4) * 4 + 2 * int64_t{sc.bw} * 4 + D * 4 + int64_t{sc.nslots} * D * 4;
}

int64_t tile_rows(int64_t D) { return 2048 / D; }
int bwd_grid(int64_t ntiles) { return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ntiles, lg_num_cus()))); }

template <typename Kern>
bool allow_lds(Kern kernel, int64_t dyn) {
    return dyn <= 64 * 1024 || hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   static_cast<int>(dyn)) == hipSuccess;
}

}  // namespace

extern "C" int lg_edge_head_fwd(const int64_t* ends, const float* h, const float* w1, const float* b1,
                                const float* w2, const float* b2, float* logits, int64_t ldo, float* hid,
                                int64_t B, int64_t N, int64_t P, int64_t D, int64_t hidden, int flags,
                                float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream) {
    if (B < 0 || N <= 0 || P < 0) return LG_EINVAL;
    if (hidden != HID || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const int dropout = (flags & LG_F_DROPOUT) ? 1 : 0;
    if (dropout && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    const int64_t BP = B * P;
    if (BP == 0) return LG_OK;
    if (!ends || !h || !w1 || !b1 || !w2 || !b2 || !logits || ldo < P) return LG_EINVAL;
    if (BP * HID >= (int64_t{1} << 32) || N * B * D >= (int64_t{1} << 32)) return LG_EUNSUPPORTED;  // 32-bit offsets
    const lg_fastdiv fdP = lg_make_fastdiv(static_cast<uint32_t>(P));
    const bool nm = (flags & LG_F_NODE_MAJOR) != 0;  // h is [N][B][D] instead of [B][N][D]
    const int64_t sb = nm ? 1 : N, sn = nm ? B : 1;
    const int64_t ntiles = cdiv(BP, tile_rows(D));
    // persistent grid sized to residency (tiles are dealt statically)
    const bool bf = (flags & LG_F_BF16) != 0;
    const int64_t per_cu = bf ? (D == 64 ? EG<64>::FWD_WG_PER_CU_BF : EG<32>::FWD_WG_PER_CU_BF)
                              : (D == 64 ? EG<64>::FWD_WG_PER_CU : EG<32>::FWD_WG_PER_CU);
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ntiles, per_cu * lg_num_cus()));
    const float scale = dropout ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
#ifdef LG_KERNEL_LAB
    const int dropout_arg = dropout | (((flags >> 28) & 7) << 8);
#else
    const int dropout_arg = dropout;
#endif
#define LG_EDGE_FWD(DD, BFB, F16B)                                                                                \
    do {                                                                                                          \
        if (!allow_lds(k_edge_fwd<DD, BFB, F16B>, EG<DD>::FWD_LDS)) return LG_EHIP;                               \
        lg_launch(k_edge_fwd<DD, BFB, F16B>, grid, NT, EG<DD>::FWD_LDS, s, ends, h, w1, b1, w2, b2, logits, ldo, hid,  \
                  sb, sn, fdP, BP, ntiles, dropout_arg, dropout_p, scale, seed, salt);                            \
    } while (0)
    // fp32 tier at D = 64: the f16x2 transform unless LG_F_BF16X3 asks for the 3-way bf16 split
    const bool f16 = !bf && !(flags & LG_F_BF16X3);
    if (D == 64) {
        if (bf) LG_EDGE_FWD(64, true, false);
        else if (f16) LG_EDGE_FWD(64, false, true);
        else LG_EDGE_FWD(64, false, false);
    } else {
        if (bf) LG_EDGE_FWD(32, true, false); else LG_EDGE_FWD(32, false, false);
    }
#undef LG_EDGE_FWD
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int64_t lg_edge_head_bwd_workspace_bytes(int64_t B, int64_t P, int64_t D, int64_t hidden) {
    if (B < 0 || P < 0 || hidden != HID || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const int64_t SL = (HID * 3 * D + 2 * HID + 1 + 3) & ~int64_t(3);  // = k_edge_bwd's padded slab row
    // rows for the larger of the two grids: tile-strided (lg_edge_head_bwd) and one workgroup per
    // window (lg_edge_head_bwd_scatter), which is the larger when P < 2048 / D pipes
    const int64_t G = std::max<int64_t>(bwd_grid(cdiv(std::max<int64_t>(B * P, 1), tile_rows(D))),
                                        std::max<int64_t>(1, std::min<int64_t>(B, lg_num_cus())));
    return ((G * SL * 4 + 255) & ~int64_t(255)) + G * 8;
}

namespace {

struct PoolGrads {  // lg_heads_bwd_scatter: the NoLeakHead's weight gradients
    float *dw1, *db1, *dw2, *db2;
};

int edge_bwd_impl(const int64_t* ends, const float* h, const float* w1, const float* w2, const float* hid,
                  const float* dlogits, int64_t ldo, float* dpipe, float* dw1, float* db1, float* dw2, float* db2,
                  int64_t B, int64_t N, int64_t P, int64_t D, int64_t hidden, int flags, float dropout_p,
                  void* workspace, int64_t ws_bytes, lg_stream_t stream, const EdgeScatter* scat,
                  const PoolGrads* pool = nullptr) {
    if (B < 0 || N <= 0 || P < 0) return LG_EINVAL;
    if (hidden != HID || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const int dropout = (flags & LG_F_DROPOUT) ? 1 : 0;
    if (dropout && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (!h || !w1 || !w2 || !dw1 || !db1 || !dw2 || !db2 || !workspace) return LG_EINVAL;
    const int64_t BP = B * P;
    if (BP > 0 && (!ends || !hid || !dlogits || !dpipe || ldo < P)) return LG_EINVAL;
    if (BP * HID >= (int64_t{1} << 32) || N * B * D >= (int64_t{1} << 32)) return LG_EUNSUPPORTED;  // 32-bit offsets
    const lg_fastdiv fdP = lg_make_fastdiv(static_cast<uint32_t>(std::max<int64_t>(P, 1)));
    const bool nm = (flags & LG_F_NODE_MAJOR) != 0;  // h is [N][B][D] instead of [B][N][D]
    const int64_t sb = nm ? 1 : N, sn = nm ? B : 1;
    const int64_t ntiles = cdiv(std::max<int64_t>(BP, 1), tile_rows(D));
    // SCAT: one workgroup per window (at most one per CU, as the strided schedule); the slab
    // of lg_edge_head_bwd_workspace_bytes has a row for every one of them
    const int grid = scat ? static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(B, lg_num_cus()))) : bwd_grid(ntiles);
    const float scale = dropout ? 1.0f / (1.0f - dropout_p) : 1.0f;
    const int64_t SL = (HID * 3 * D + 2 * HID + 1 + 3) & ~int64_t(3);  // = k_edge_bwd's padded slab row
    // the slab the launch grid writes: a row per workgroup + one fp64 per workgroup
    if (ws_bytes < ((grid * SL * 4 + 255) & ~int64_t(255)) + grid * 8) return LG_EINVAL;
    float* slab = static_cast<float*>(workspace);
    double* dslab = reinterpret_cast<double*>(static_cast<char*>(workspace) + ((grid * SL * 4 + 255) & ~int64_t(255)));
    hipStream_t s = lg_stream(stream);
    const EdgeScatter none{};
    if (BP == 0) {
        if (hipMemsetAsync(slab, 0, SL * grid * sizeof(float), s) != hipSuccess) return LG_EHIP;
        if (hipMemsetAsync(dslab, 0, grid * sizeof(double), s) != hipSuccess) return LG_EHIP;
    } else {
        const bool bf = (flags & LG_F_BF16) != 0, f16 = edge_bwd_f16(flags);
        const bool stream = scat && scat->spipe;
        const int64_t base = edge_bwd_base_lds(D, flags);
        const int64_t lds = stream ? edge_stream_lds(D, flags, *scat) : scat ? base + 4 * (N + 1 + 2 * P) : base;
#define LG_EDGE_BWD(DD, BFB, F16B)                                                                                \
    do {                                                                                                          \
        if (stream) {                                                                                             \
            if (!allow_lds(k_edge_bwd<DD, BFB, 2, F16B>, lds)) return LG_EHIP;                                     \
            lg_launch(k_edge_bwd<DD, BFB, 2, F16B>, grid, NT, lds, s, ends, h, w1, w2, hid, dlogits, ldo, dpipe,    \
                      slab, dslab, sb, sn, fdP, BP, ntiles, scale, *scat);                                         \
        } else if (scat) {                                                                                        \
            if (!allow_lds(k_edge_bwd<DD, BFB, 1, F16B>, lds)) return LG_EHIP;                                     \
            lg_launch(k_edge_bwd<DD, BFB, 1, F16B>, grid, NT, lds, s, ends, h, w1, w2, hid, dlogits, ldo, dpipe,    \
                      slab, dslab, sb, sn, fdP, BP, ntiles, scale, *scat);                                         \
        } else {                                                                                                  \
            if (!allow_lds(k_edge_bwd<DD, BFB, 0, F16B>, lds)) return LG_EHIP;                                     \
            lg_launch(k_edge_bwd<DD, BFB, 0, F16B>, grid, NT, lds, s, ends, h, w1, w2, hid, dlogits, ldo, dpipe,    \
                      slab, dslab, sb, sn, fdP, BP, ntiles, scale, none);                                          \
        }                                                                                                         \
    } while (0)
        if (D == 64) {
            if (bf) LG_EDGE_BWD(64, true, false);
            else if (f16) LG_EDGE_BWD(64, false, true);
            else LG_EDGE_BWD(64, false, false);
        } else {
            if (bf) LG_EDGE_BWD(32, true, false);
            else if (f16) LG_EDGE_BWD(32, false, true);
            else LG_EDGE_BWD(32, false, false);
        }
#undef LG_EDGE_BWD
    }
    LG_RET_IF_LAUNCH_FAILED();
    const int64_t K3 = 3 * D;
    const LgSlabSeg segs[3] = {{0, HID * K3, dw1}, {HID * K3, HID, db1}, {HID * K3 + HID, HID, dw2}};
    const int rc = lg_launch_slab_reduce_multi(slab, grid, SL, segs, 3, dslab, db2, s);
    if (rc != LG_OK || !pool) return rc;
    // the NoLeakHead's slab rows (lg_heads_bwd_scatter: written by the same grid's prologue)
    const LgSlabSeg psegs[3] = {{0, HID * D, pool->dw1}, {HID * D, HID, pool->db1}, {HID * D + HID, HID, pool->dw2}};
    return lg_launch_slab_reduce_multi(scat->nslab, grid, HID * D + 2 * HID, psegs, 3, scat->ndslab, pool->db2, s);
}

}  // namespace

extern "C" int lg_edge_head_bwd(const int64_t* ends, const float* h, const float* w1, const float* w2,
                                const float* hid, const float* dlogits, int64_t ldo, float* dpipe, float* dw1,
                                float* db1, float* dw2, float* db2, int64_t B, int64_t N, int64_t P, int64_t D,
                                int64_t hidden, int flags, float dropout_p, void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    return edge_bwd_impl(ends, h, w1, w2, hid, dlogits, ldo, dpipe, dw1, db1, dw2, db2, B, N, P, D, hidden, flags,
                         dropout_p, workspace, ws_bytes, stream, nullptr);
}

namespace {
// lg_edge_head_bwd_scatter; with `pool` (lg_heads_bwd_scatter) the STREAM form runs the
// NoLeakHead backward in its prologue (its slab in pool_ws) and returns 1 when it did, 0 when
// it took another form (the caller then runs lg_pool_head_bwd first: dpool is an input there)
int edge_bwd_scatter_impl(const int64_t* ends, const float* h, const float* w1, const float* w2, const float* hid,
                          const float* dlogits, int64_t ldo, float* dpipe, float* dw1, float* db1, float* dw2,
                          float* db2, const int32_t* inc_rowptr, const int32_t* inc_item, const int32_t* sched,
                          const int32_t* sched_hdr, const float* dpool, float* dh, int64_t B, int64_t N, int64_t P,
                          int64_t D, int64_t hidden, int flags, float dropout_p, void* workspace, int64_t ws_bytes,
                          lg_stream_t stream, const EdgeScatter* pool_sc, const PoolGrads* pool, bool* fused) {
    if (fused) *fused = false;
    if (B < 0 || N <= 0 || P < 0) return LG_EINVAL;
    if (!dh || !inc_rowptr || (P > 0 && !inc_item)) return LG_EINVAL;
    if (!sched != !sched_hdr) return LG_EINVAL;
    if (sched_hdr && (sched_hdr[0] != LG_PIPE_SCHED_VERSION || sched_hdr[1] != P || sched_hdr[2] != N || sched_hdr[3] != D))
        return LG_EINVAL;  // a schedule built for another graph or width
    if (B == 0) return edge_bwd_impl(ends, h, w1, w2, hid, dlogits, ldo, dpipe, dw1, db1, dw2, db2, B, N, P, D,
                                     hidden, flags, dropout_p, workspace, ws_bytes, stream, nullptr);
    // the fused forms run one workgroup per window: with fewer windows than CUs most of the
    // GPU would idle through the windows' tiles (C4: 64 windows of 235 tiles, 2.0 vs 1.1 ms per
    // step), so the two launches take over there
    const bool per_window = B >= lg_num_cus();
    if (per_window && sched && P > 0 && B * N < kLgMaxRows) {
        EdgeScatter sc{inc_rowptr, inc_item, dpool, dh, static_cast<uint32_t>(N), static_cast<uint32_t>(P),
                       static_cast<uint32_t>(B), (flags & LG_F_NODE_MAJOR) ? 1 : 0, sched_hdr[5],
                       reinterpret_cast<const int4*>(sched + sched_hdr[10]),
                       reinterpret_cast<const uint32_t*>(sched + sched_hdr[11]), sched + sched_hdr[12],
                       sched_hdr[9], sched_hdr[6], sched_hdr[8], sched_hdr[7], kEdgeLab(flags)};
        sc.fdT = lg_make_fastdiv(static_cast<uint32_t>(std::max(1, sc.tpw)));
        // STREAM when the open nodes' sums fit beside the images (L-TOWN-A at D = 64: 23 of them)
        if (edge_stream_lds(D, flags, sc) <= 160 * 1024) {
            if (pool_sc) {
                sc.pooled = pool_sc->pooled;
                sc.nhid = pool_sc->nhid;
                sc.nW1 = pool_sc->nW1;
                sc.nw2 = pool_sc->nw2;
                sc.nscale = pool_sc->nscale;
                sc.nslab = pool_sc->nslab;
                sc.ndslab = pool_sc->ndslab;
                if (fused) *fused = true;
            }
            return edge_bwd_impl(ends, h, w1, w2, hid, dlogits, ldo, dpipe, dw1, db1, dw2, db2, B, N, P, D, hidden,
                                 flags, dropout_p, workspace, ws_bytes, stream, &sc, pool_sc ? pool : nullptr);
        }
    }
    if (pool_sc) return LG_OK;  // the caller runs the two-step form
    const int64_t base = edge_bwd_base_lds(D, flags);
    if (!per_window || P == 0 || base + 4 * (N + 1 + 2 * P) > 160 * 1024 || B * N >= kLgMaxRows) {
        // the incidence CSR does not fit beside the kernel's images: the separate scatter launch
        const int rc = edge_bwd_impl(ends, h, w1, w2, hid, dlogits, ldo, dpipe, dw1, db1, dw2, db2, B, N, P, D, hidden,
                                     flags, dropout_p, workspace, ws_bytes, stream, nullptr);
        if (rc != LG_OK) return rc;
        return lg_pipe_scatter_bwd(inc_rowptr, inc_item, dpipe, dpool, dh, B, N, P, D, flags & LG_F_NODE_MAJOR, stream);
    }
    EdgeScatter sc{inc_rowptr, inc_item, dpool, dh, static_cast<uint32_t>(N), static_cast<uint32_t>(P),
                   static_cast<uint32_t>(B), (flags & LG_F_NODE_MAJOR) ? 1 : 0,
                   static_cast<int>(cdiv(P, tile_rows(D))), nullptr, nullptr, nullptr, 0, 0, 0, 0, kEdgeLab(flags)};
    sc.fdT = lg_make_fastdiv(static_cast<uint32_t>(std::max(1, sc.tpw)));
    return edge_bwd_impl(ends, h, w1, w2, hid, dlogits, ldo, dpipe, dw1, db1, dw2, db2, B, N, P, D, hidden, flags,
                         dropout_p, workspace, ws_bytes, stream, &sc);
}
}  // namespace

extern "C" int lg_edge_head_bwd_scatter(const int64_t* ends, const float* h, const float* w1, const float* w2,
                                        const float* hid, const float* dlogits, int64_t ldo, float* dpipe,
                                        float* dw1, float* db1, float* dw2, float* db2, const int32_t* inc_rowptr,
                                        const int32_t* inc_item, const int32_t* sched, const int32_t* sched_hdr,
                                        const float* dpool, float* dh, int64_t B, int64_t N,
                                        int64_t P, int64_t D, int64_t hidden, int flags, float dropout_p,
                                        void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    return edge_bwd_scatter_impl(ends, h, w1, w2, hid, dlogits, ldo, dpipe, dw1, db1, dw2, db2, inc_rowptr, inc_item,
                                 sched, sched_hdr, dpool, dh, B, N, P, D, hidden, flags, dropout_p, workspace, ws_bytes,
                                 stream, nullptr, nullptr, nullptr);
}

extern "C" int lg_heads_bwd_scatter(const float* pooled, const float* nhid, const float* nw1, const float* nw2,
                                    float* ndw1, float* ndb1, float* ndw2, float* ndb2, int nflags, float n_dropout_p,
                                    void* nworkspace, int64_t nws_bytes, const int64_t* ends, const float* h,
                                    const float* w1, const float* w2, const float* hid, const float* dlogits,
                                    int64_t ldo, float* dpipe, float* dw1, float* db1, float* dw2, float* db2,
                                    const int32_t* inc_rowptr, const int32_t* inc_item, const int32_t* sched,
                                    const int32_t* sched_hdr, float* dpool, float* dh, int64_t B, int64_t N, int64_t P,
                                    int64_t D, int64_t hidden, int flags, float dropout_p, void* workspace,
                                    int64_t ws_bytes, lg_stream_t stream) {
    if (B < 0 || N <= 0 || P < 0 || ldo <= P) return LG_EINVAL;
    if (hidden != HID || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const bool ndrop = (nflags & LG_F_DROPOUT) != 0;
    if (ndrop && !(n_dropout_p >= 0.f && n_dropout_p < 1.f)) return LG_EINVAL;
    if (!nw1 || !nw2 || !ndw1 || !ndb1 || !ndw2 || !ndb2 || !nworkspace || !dpool) return LG_EINVAL;
    if (B > 0 && (!pooled || !nhid)) return LG_EINVAL;
    // the fused form writes one NoLeakHead slab row per workgroup of the edge grid (<= B, <= CUs),
    // which lg_pool_head_bwd_workspace_bytes covers
    const int64_t nwsb = lg_pool_head_bwd_workspace_bytes(B, D, hidden);
    if (nwsb < 0) return static_cast<int>(nwsb);
    if (nws_bytes < nwsb) return LG_EINVAL;
    const int64_t G = std::max<int64_t>(1, std::min<int64_t>(B, 2LL * lg_num_cus()));  // lg_pool_head_bwd's grid
    EdgeScatter psc{};
    psc.pooled = pooled;
    psc.nhid = nhid;
    psc.nW1 = nw1;
    psc.nw2 = nw2;
    psc.nscale = ndrop ? 1.0f / (1.0f - n_dropout_p) : 1.0f;
    psc.nslab = static_cast<float*>(nworkspace);
    psc.ndslab = reinterpret_cast<double*>(static_cast<char*>(nworkspace) + ((G * (HID * D + 2 * HID) * 4 + 255) & ~int64_t(255)));
    const PoolGrads pg{ndw1, ndb1, ndw2, ndb2};
    if (B > 0) {
        bool fused = false;
        const int rc = edge_bwd_scatter_impl(ends, h, w1, w2, hid, dlogits, ldo, dpipe, dw1, db1, dw2, db2, inc_rowptr,
                                             inc_item, sched, sched_hdr, dpool, dh, B, N, P, D, hidden, flags,
                                             dropout_p, workspace, ws_bytes, stream, &psc, &pg, &fused);
        if (rc != LG_OK || fused) return rc;
    }
    // another form: the NoLeakHead backward first (its dpool is the scatter's input)
    const int rc = lg_pool_head_bwd(pooled, nhid, nw1, nw2, dlogits, ldo, P, dpool, ndw1, ndb1, ndw2, ndb2, B, D, hidden,
                                    nflags, n_dropout_p, nworkspace, nws_bytes, stream);
    if (rc != LG_OK) return rc;
    return lg_edge_head_bwd_scatter(ends, h, w1, w2, hid, dlogits, ldo, dpipe, dw1, db1, dw2, db2, inc_rowptr, inc_item,
                                    sched, sched_hdr, dpool, dh, B, N, P, D, hidden, flags, dropout_p, workspace,
                                    ws_bytes, stream);
}

/* ---------------------------------------------------------------------------------------------
 * Pipe schedule (host).  Pipes ordered by their endpoints' positions in the RCM order of the
 * pipe graph (key: the later endpoint, then the earlier one, then the id), so each node's
 * incidences fall in a few consecutive tiles; per tile, one event per node it touches.  Layout
 * in int32 words: header [16] (the fields of sched_hdr), pipes [P][4] {u, v, p, 0}, tile blocks
 * [tpw][bw] {event count, 0, events [maxev][2], incidence bytes [2 TR] (2 row + role, grouped
 * by event, rows in order)}, nodes without pipes [nzero].
 * -------------------------------------------------------------------------------------------*/
extern "C" int64_t lg_pipe_schedule_words(int64_t P, int64_t N, int64_t D) {
    if (P < 0 || N <= 0 || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const int64_t TR = tile_rows(D), tpw = cdiv(P, TR);
    return 16 + 4 * P + tpw * (2 + 4 * TR + TR / 2) + N;
}

extern "C" int lg_pipe_schedule_build(const int64_t* ends, int64_t P, int64_t N, int64_t D, int32_t* sched,
                                      int64_t words, int32_t* inc_rowptr, int32_t* inc_item) {
    if (P < 0 || N <= 0 || (P > 0 && !ends) || !sched || !inc_rowptr || (P > 0 && !inc_item)) return LG_EINVAL;
    if (D != 32 && D != 64) return LG_EUNSUPPORTED;
    if (N >= (int64_t{1} << 24) || P >= (int64_t{1} << 30)) return LG_EUNSUPPORTED;
    for (int64_t i = 0; i < 2 * P; ++i)
        if (ends[i] < 0 || ends[i] >= N) return LG_EINVAL;
    const int64_t TR = tile_rows(D), tpw = cdiv(P, TR);
    // node positions in the RCM order of the pipe graph
    std::vector<int64_t> ei(2 * P);
    for (int64_t p = 0; p < P; ++p) {
        ei[p] = ends[2 * p];
        ei[P + p] = ends[2 * p + 1];
    }
    std::vector<int32_t> order(N), pos(N);
    if (P > 0) {
        const int rc = lg_rcm_order(ei.data(), P, N, order.data());
        if (rc != LG_OK) return rc;
    }
    for (int64_t i = 0; i < N; ++i) pos[order[i]] = static_cast<int32_t>(i);
    std::vector<int32_t> perm(P);
    for (int64_t p = 0; p < P; ++p) perm[p] = static_cast<int32_t>(p);
    auto key = [&](int32_t p) {
        const int32_t a = pos[ends[2 * p]], b = pos[ends[2 * p + 1]];
        return std::make_tuple(std::max(a, b), std::min(a, b), p);
    };
    std::sort(perm.begin(), perm.end(), [&](int32_t x, int32_t y) { return key(x) < key(y); });
    // the tile range of each node's incidences
    std::vector<int64_t> first(N, -1), last(N, -1);
    for (int64_t i = 0; i < P; ++i)
        for (int role = 0; role < 2; ++role) {
            const int64_t n = ends[2 * perm[i] + role], t = i / TR;
            if (first[n] < 0) first[n] = t;
            last[n] = t;
        }
    // events per tile: nodes in order of first touch, each with its incidences in row order
    struct Ev { int32_t node, slot; int cnt; std::vector<uint8_t> inc; };
    std::vector<std::vector<Ev>> tiles(tpw);
    int64_t maxev = 0;
    std::vector<int32_t> at(N, -1);  // event index of node n in the tile being built
    for (int64_t t = 0; t < tpw; ++t) {
        auto& ev = tiles[t];
        const int64_t i1 = std::min(P, (t + 1) * TR);
        for (int64_t i = t * TR; i < i1; ++i)
            for (int role = 0; role < 2; ++role) {
                const int32_t n = static_cast<int32_t>(ends[2 * perm[i] + role]);
                if (at[n] < 0) {
                    at[n] = static_cast<int32_t>(ev.size());
                    ev.push_back(Ev{n, 0, 0, {}});
                }
                ev[at[n]].inc.push_back(static_cast<uint8_t>(2 * (i - t * TR) + role));
            }
        for (auto& e : ev) at[e.node] = -1;
        maxev = std::max<int64_t>(maxev, static_cast<int64_t>(ev.size()));
    }
    // LDS slots of the nodes open across a tile boundary; a slot freed at tile t is reused from t + 1
    std::vector<char> used;
    std::vector<int32_t> slot_of(N, -1);
    for (int64_t t = 0; t < tpw; ++t) {
        std::vector<int32_t> freed;
        for (auto& e : tiles[t]) {
            const bool f = first[e.node] == t, l = last[e.node] == t;
            if (f && !l) {
                size_t sidx = 0;
                while (sidx < used.size() && used[sidx]) ++sidx;
                if (sidx == used.size()) used.push_back(0);
                used[sidx] = 1;
                slot_of[e.node] = static_cast<int32_t>(sidx);
            }
            e.slot = slot_of[e.node] < 0 ? 0 : slot_of[e.node];
            if (!f && l) freed.push_back(slot_of[e.node]);
        }
        for (int32_t x : freed) used[x] = 0;
    }
    const int64_t nslots = static_cast<int64_t>(used.size());
    if (nslots >= 65536) return LG_EUNSUPPORTED;
    std::vector<int32_t> zero;
    for (int64_t n = 0; n < N; ++n)
        if (first[n] < 0) zero.push_back(static_cast<int32_t>(n));
    const int64_t bw = 2 + 2 * maxev + TR / 2;
    const int64_t off_pipes = 16, off_blocks = off_pipes + 4 * P, off_zero = off_blocks + tpw * bw;
    const int64_t total = off_zero + static_cast<int64_t>(zero.size());
    if (total > words) return LG_EINVAL;
    std::fill(sched, sched + total, 0);
    const int32_t hdr[16] = {LG_PIPE_SCHED_VERSION, static_cast<int32_t>(P), static_cast<int32_t>(N),
                             static_cast<int32_t>(D), static_cast<int32_t>(TR), static_cast<int32_t>(tpw),
                             static_cast<int32_t>(nslots), static_cast<int32_t>(maxev), static_cast<int32_t>(bw),
                             static_cast<int32_t>(zero.size()), static_cast<int32_t>(off_pipes),
                             static_cast<int32_t>(off_blocks), static_cast<int32_t>(off_zero),
                             static_cast<int32_t>(total), 0, 0};
    std::copy(hdr, hdr + 16, sched);
    for (int64_t i = 0; i < P; ++i) {
        sched[off_pipes + 4 * i] = static_cast<int32_t>(ends[2 * perm[i]]);
        sched[off_pipes + 4 * i + 1] = static_cast<int32_t>(ends[2 * perm[i] + 1]);
        sched[off_pipes + 4 * i + 2] = perm[i];
    }
    for (int64_t t = 0; t < tpw; ++t) {
        int32_t* blk = sched + off_blocks + t * bw;
        uint8_t* incl = reinterpret_cast<uint8_t*>(blk + 2 + 2 * maxev);
        blk[0] = static_cast<int32_t>(tiles[t].size());
        int st = 0;
        for (size_t e = 0; e < tiles[t].size(); ++e) {
            const Ev& v = tiles[t][e];
            const uint32_t w0 = static_cast<uint32_t>(v.node) | (first[v.node] == t ? 1u << 24 : 0u) |
                                (last[v.node] == t ? 1u << 25 : 0u);
            const uint32_t w1 = static_cast<uint32_t>(v.slot) | (static_cast<uint32_t>(st) << 16) |
                                (static_cast<uint32_t>(v.inc.size()) << 24);
            blk[2 + 2 * e] = static_cast<int32_t>(w0);
            blk[3 + 2 * e] = static_cast<int32_t>(w1);
            for (uint8_t b : v.inc) incl[st++] = b;
        }
    }
    std::copy(zero.begin(), zero.end(), sched + off_zero);
    // the incidence CSR in schedule order (lg_pipe_scatter_bwd over it sums as the stream does)
    std::fill(inc_rowptr, inc_rowptr + N + 1, 0);
    for (int64_t i = 0; i < 2 * P; ++i) ++inc_rowptr[ends[i] + 1];
    for (int64_t n = 0; n < N; ++n) inc_rowptr[n + 1] += inc_rowptr[n];
    std::vector<int32_t> fill(inc_rowptr, inc_rowptr + N);
    for (int64_t i = 0; i < P; ++i)
        for (int role = 0; role < 2; ++role) inc_item[fill[ends[2 * perm[i] + role]]++] = 2 * perm[i] + role;
    return LG_OK;
}
