// 3-way bf16 split of fp32 operands for bf16 MFMA at fp32-level accuracy (gfx950).
//
// x = x0 + x1 + x2 with x_i = bf16_rne(x - x0 - ...): |x - (x0 + x1 + x2)| <= 2^-24 |x|.
// A product x w is then sum_{i+j<=2} x_i w_j (6 bf16 MFMAs, each product exact in fp32,
// fp32 accumulate); the dropped terms are <= 2^-24 |x w|: fp32-level accuracy at 6/16 of
// the f32-MFMA issue time (v_mfma_f32_16x16x32_bf16: 16 cyc per 16x16x32 vs 32 cyc per
// 16x16x4 for v_mfma_f32_16x16x4_f32, i.e. 96 vs 256 cycles per K = 32).
#pragma once
#include "common.h"

typedef __bf16 lg_bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 lg_bf16x8 __attribute__((ext_vector_type(8)));
typedef float lg_f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t lg_u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t lg_u32x4 __attribute__((ext_vector_type(4)));
typedef short lg_i16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    const lg_f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, lg_bf16x2));
}
__device__ __forceinline__ float bf_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf_hi(uint32_t p) { return __uint_as_float(p & 0xFFFF0000u); }

// one pair of floats -> (hi, mid, lo) packed bf16 pairs
__device__ __forceinline__ void split3_pair(float a, float b, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
    p0 = pk_bf16(a, b);
    const float ra = a - bf_lo(p0), rb = b - bf_hi(p0);
    p1 = pk_bf16(ra, rb);
    p2 = pk_bf16(ra - bf_lo(p1), rb - bf_hi(p1));
}
// 4 floats -> three 4 x bf16 parts (8 bytes each)
__device__ __forceinline__ void split3_x4(const f32x4& u, lg_u32x2& f0, lg_u32x2& f1, lg_u32x2& f2) {
    uint32_t a0, a1, a2, b0, b1, b2;
    split3_pair(u[0], u[1], a0, a1, a2);
    split3_pair(u[2], u[3], b0, b1, b2);
    f0 = lg_u32x2{a0, b0};
    f1 = lg_u32x2{a1, b1};
    f2 = lg_u32x2{a2, b2};
}
// 8 floats (two f32x4) -> three bf16x8 fragments (hi, mid, lo)
__device__ __forceinline__ void split3_x8(const f32x4& u, const f32x4& v, lg_bf16x8& f0, lg_bf16x8& f1,
                                          lg_bf16x8& f2) {
    lg_u32x4 p0, p1, p2;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const float a = h < 2 ? u[2 * h] : v[2 * h - 4], b = h < 2 ? u[2 * h + 1] : v[2 * h - 3];
        uint32_t x0, x1, x2;
        split3_pair(a, b, x0, x1, x2);
        p0[h] = x0;
        p1[h] = x1;
        p2[h] = x2;
    }
    f0 = __builtin_bit_cast(lg_bf16x8, p0);
    f1 = __builtin_bit_cast(lg_bf16x8, p1);
    f2 = __builtin_bit_cast(lg_bf16x8, p2);
}
__device__ __forceinline__ f32x4 mfma_bf(const lg_bf16x8& a, const lg_bf16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// acc += a * b on split operands: the six terms with i + j <= 2, smallest first
// BF (the bf16 node-MLP tier, LG_F_BF16): the single hi x hi product — operands rounded to
// bf16, fp32 accumulate.  Unused split parts and their LDS reads are dead code then.
template <bool BF>
__device__ __forceinline__ f32x4 mfma_prec(const lg_bf16x8 (&a)[3], const lg_bf16x8 (&b)[3], f32x4 c);

__device__ __forceinline__ f32x4 mfma_split(const lg_bf16x8 (&a)[3], const lg_bf16x8 (&b)[3], f32x4 c) {
    c = mfma_bf(a[2], b[0], c);
    c = mfma_bf(a[1], b[1], c);
    c = mfma_bf(a[0], b[2], c);
    c = mfma_bf(a[1], b[0], c);
    c = mfma_bf(a[0], b[1], c);
    return mfma_bf(a[0], b[0], c);
}

template <>
__device__ __forceinline__ f32x4 mfma_prec<false>(const lg_bf16x8 (&a)[3], const lg_bf16x8 (&b)[3], f32x4 c) {
    return mfma_split(a, b, c);
}
template <>
__device__ __forceinline__ f32x4 mfma_prec<true>(const lg_bf16x8 (&a)[3], const lg_bf16x8 (&b)[3], f32x4 c) {
    return mfma_bf(a[0], b[0], c);
}

// gfx950 ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, columns 4p..4p+3
// of a 4 x 16 block of 16-bit elements; lane i of the group receives column i (row q in
// element q).  EXEC must be all ones.  p must be 8-byte aligned.
__device__ __forceinline__ lg_u32x2 lds_read_tr16(const uint16_t* p) {
    typedef __attribute__((address_space(3))) lg_i16x4 lds_i16x4;
    const lg_i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p));
    return __builtin_bit_cast(lg_u32x2, v);
}
// two transposed 4-row reads -> one bf16x8 fragment (elements 0..3 from r0, 4..7 from r1)
__device__ __forceinline__ lg_bf16x8 lds_frag_tr16(const uint16_t* r0, const uint16_t* r1) {
    const lg_u32x2 a = lds_read_tr16(r0), b = lds_read_tr16(r1);
    const lg_u32x4 v = {a[0], a[1], b[0], b[1]};
    return __builtin_bit_cast(lg_bf16x8, v);
}
__device__ __forceinline__ lg_bf16x8 lds_frag_row(const uint16_t* p) {
    return *reinterpret_cast<const lg_bf16x8*>(p);
}

// ---- 2-way fp16 split with power-of-two scaling (the "f16x2" transform) -----------------
// x * 2^s = x0 + x1 + r with x0 = f16_rne(x 2^s), x1 = f16_rne(x 2^s - x0): |r| <= 2^-22 |x 2^s|
// while x 2^s stays in fp16's normal range.  A product a w is then a0 w0 + a1 w0 + a0 w1
// (3 f16 MFMAs, products exact in fp32, fp32 accumulate; the dropped a1 w1 is <= 2^-22 |a w|)
// — fp32-level accuracy at half the MFMAs of the 3-way bf16 split.  The scale exponent s
// puts the largest |x| of the block at [2^14, 2^15): everything down to 2^-17 of it keeps
// both parts normal, smaller values lose only absolute precision below 2^-38 of the block max.
typedef _Float16 lg_f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 lg_f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split2_f16_pair(float a, float b, uint32_t& p0, uint32_t& p1) {
    const lg_f32x2 v = {a, b};
    const lg_f16x2 h0 = __builtin_convertvector(v, lg_f16x2);
    const lg_f32x2 r = v - __builtin_convertvector(h0, lg_f32x2);
    p0 = __builtin_bit_cast(uint32_t, h0);
    p1 = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, lg_f16x2));
}
// 8 floats (two f32x4) -> two f16x8 fragments (hi, lo)
__device__ __forceinline__ void split2_f16_x8(const f32x4& u, const f32x4& v, lg_f16x8& f0, lg_f16x8& f1) {
    lg_u32x4 p0, p1;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const float a = h < 2 ? u[2 * h] : v[2 * h - 4], b = h < 2 ? u[2 * h + 1] : v[2 * h - 3];
        uint32_t x0, x1;
        split2_f16_pair(a, b, x0, x1);
        p0[h] = x0;
        p1[h] = x1;
    }
    f0 = __builtin_bit_cast(lg_f16x8, p0);
    f1 = __builtin_bit_cast(lg_f16x8, p1);
}
__device__ __forceinline__ f32x4 mfma_h(const lg_f16x8& a, const lg_f16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// a x b on the f16x2 split of both operands (hi, lo): the three products, smallest terms first
__device__ __forceinline__ f32x4 mfma_f16x2(const lg_f16x8 (&a)[2], const lg_f16x8 (&b)[2], f32x4 c) {
    c = mfma_h(a[1], b[0], c);
    c = mfma_h(a[0], b[1], c);
    return mfma_h(a[0], b[0], c);
}
// 2^e as a float for e in [-126, 127] (clamped)
__device__ __forceinline__ float lg_pow2f(int e) {
    e = e < -126 ? -126 : (e > 127 ? 127 : e);
    return __uint_as_float(static_cast<uint32_t>(e + 127) << 23);
}
// scale exponent for a block whose largest |value| has the float bits `mbits` (>= 0): puts that
// value at [2^14, 2^15); a zero block gets 0
__device__ __forceinline__ int lg_f16_scale_exp(uint32_t mbits) {
    if (mbits == 0) return 0;
    const int e = static_cast<int>((mbits >> 23) & 0xFF) - 127;  // floor(log2 max) (subnormals: -127)
    return 14 - e;
}
// max over the wave of a non-negative float's bits (integer order = float order), broadcast
// (DPP within rows of 16, then the four row results through readlane)
__device__ __forceinline__ uint32_t lg_wave_max_bits(uint32_t m) {
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0xB1, 0xF, 0xF, false)));  // xor 1
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x4E, 0xF, 0xF, false)));  // xor 2
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x124, 0xF, 0xF, false)));  // row_ror 4
    m = max(m, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(m), 0x128, 0xF, 0xF, false)));  // row_ror 8
    const uint32_t r0 = __builtin_amdgcn_readlane(m, 0), r1 = __builtin_amdgcn_readlane(m, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(m, 32), r3 = __builtin_amdgcn_readlane(m, 48);
    return max(max(r0, r1), max(r2, r3));
}

typedef _Float16 lg_f16x4 __attribute__((ext_vector_type(4)));
// 4 floats -> two f16x4 parts (hi, lo) of the f16x2 split
__device__ __forceinline__ void split2_f16_x4(const f32x4& u, lg_f16x4& f0, lg_f16x4& f1) {
    uint32_t a0, a1, b0, b1;
    split2_f16_pair(u[0], u[1], a0, a1);
    split2_f16_pair(u[2], u[3], b0, b1);
    f0 = __builtin_bit_cast(lg_f16x4, lg_u32x2{a0, b0});
    f1 = __builtin_bit_cast(lg_f16x4, lg_u32x2{a1, b1});
}
// the f16x2 scale exponent of a block clamped to [-63, 63], so that the sum of two block
// exponents (a product's unscale) stays a normal power of two.  Blocks with max |v| < 2^-49
// keep less relative precision, blocks above 2^79 would overflow f16: neither occurs in the
// GCN's activations or gradients.
__device__ __forceinline__ int lg_f16_scale_exp_c(uint32_t mbits) {
    const int e = lg_f16_scale_exp(mbits);
    return e < -63 ? -63 : (e > 63 ? 63 : e);
}
