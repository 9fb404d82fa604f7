// K8 + K9: EdgeHead (reference detector.py:76-88, 206-211) fused end to end.
//
//   feat[b,p] = [h_u, h_v, |h_u - h_v|]            (3D)      u, v = pipe_ends[p]
//   hid       = dropout(relu(W1 feat + b1))          (128)
//   logit     = W2 hid + b2                          (1)
//
// The (B, P, 3D) feature tensor (150 MB at B=256) and the (B, P, 128) hidden
// tensor are never written to HBM.  One 512-thread workgroup processes 16 pipe
// rows at a time: the rows' endpoint features are gathered into LDS once, then
// wave w (of 8) computes hidden units [16w, 16w+16) for all 16 rows as
// hid^T = W1 feat^T on v_mfma_f32_16x16x4_f32 (exact fp32; its W1 slice lives in
// registers), applies bias/ReLU/dropout, dots with W2 and the eight partial
// logits are added in wave order.
//
// Backward recomputes hid, then per row tile:
//   dhid  = dlogit * W2 * relu' * dropout mask                (lane-local)
//   dW1^T += feat^T dhid   (MFMA, K = rows)   dW2 += dlogit*hid   db1 += dhid   db2 += dlogit
//   dfeat^T = W1^T dhid^T  (MFMA, K = 128)     -> per-pipe endpoint grads
//   dpipe[b,p,0] = dfeat_u + sgn*dfeat_abs,  dpipe[b,p,1] = dfeat_v - sgn*dfeat_abs,
//   sgn = sign(h_u - h_v)  (torch abs backward).
// dpipe is then summed per node over the incidence CSR by lg_pipe_scatter_bwd
// (deterministic, no atomics).  Weight grads: per-workgroup slabs + fixed-order reduce.
#include <algorithm>
#include "common.h"
#include "reduce.h"

namespace {

constexpr int HID = 128;
constexpr int TR = 16;       // pipe rows per tile
constexpr int NW = 8;        // waves per workgroup (= HID / 16)

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int fk(int ks, int q) { return 16 * (ks >> 2) + 4 * q + (ks & 3); }
// row r = b*P + p of the (B, P) logit space -> element (b, p) of a buffer with row stride ldo
__device__ __forceinline__ int64_t lg_row_index(int64_t r, const lg_fastdiv& fdP, int64_t ldo) {
    const uint32_t b = lg_div(static_cast<uint32_t>(r), fdP);
    return static_cast<int64_t>(b) * ldo + (static_cast<uint32_t>(r) - b * fdP.d);
}

template <int D>
struct EG {
    static constexpr int K3 = 3 * D;       // feature width
    static constexpr int KS = K3 / 4;      // k-steps of the feat contraction
    static constexpr int FS = K3 + 4;      // LDS row stride of the feature tile
    static constexpr int MT = K3 / 16;     // 16-row tiles of K3
    static constexpr int DT = D / 16;      // 16-row tiles of D
    static constexpr int F4 = D / 4;       // float4 per node row
    static constexpr int NSPLIT = NW / DT; // waves sharing one k-triple of dfeat (split over hidden)
    static constexpr int KPER = 32 / NSPLIT;  // k-steps (of 32 over hidden=128) per wave
};

// Gather the two endpoint rows of 16 pipe rows into ft[16][FS] (u at [0,D), v at [D,2D)).
template <int D>
__device__ __forceinline__ void gather_tile(const int64_t* __restrict__ ends, const float* __restrict__ h,
                                            float* __restrict__ ft, int64_t row0, int64_t BP, const lg_fastdiv& fdP,
                                            int64_t sb, int64_t sn) {
    using G = EG<D>;
    const int t = threadIdx.x;
    if (t < TR * 2 * G::F4) {
        const int row = t / (2 * G::F4), rem = t % (2 * G::F4), side = rem / G::F4, f4 = rem % G::F4;
        const int64_t gr = row0 + row;
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (gr < BP) {
            const uint32_t b = lg_div(static_cast<uint32_t>(gr), fdP), p = static_cast<uint32_t>(gr) - b * fdP.d;
            const int64_t node = ends[2 * p + side];
            v = ld4(h + (static_cast<int64_t>(b) * sb + node * sn) * D + 4 * f4);  // row of (window b, node)
        }
        st4(ft + row * G::FS + side * D + 4 * f4, v);
    }
}

// feat[row][k] with the |u - v| third computed on the fly
template <int D>
__device__ __forceinline__ f32x4 feat4(const float* __restrict__ ft, int row, int k) {
    using G = EG<D>;
    if (k < 2 * D) return ld4(ft + row * G::FS + k);
    const f32x4 u = ld4(ft + row * G::FS + (k - 2 * D));
    const f32x4 v = ld4(ft + row * G::FS + (k - D));
    f32x4 a;
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = fabsf(u[i] - v[i]);
    return a;
}
template <int D>
__device__ __forceinline__ float feat1(const float* __restrict__ ft, int row, int k) {
    using G = EG<D>;
    if (k < 2 * D) return ft[row * G::FS + k];
    return fabsf(ft[row * G::FS + (k - 2 * D)] - ft[row * G::FS + (k - D)]);
}

// hid^T tile rows n = 16w + 4q + reg for feat row j, bias included
template <int D>
__device__ __forceinline__ f32x4 hidden_tile(const float* __restrict__ ft, const float (&aw)[EG<D>::KS], f32x4 acc,
                                             int j, int q) {
#pragma unroll
    for (int a = 0; a < EG<D>::KS / 4; ++a) {
        const f32x4 v = feat4<D>(ft, j, 16 * a + 4 * q);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc = mfma(aw[4 * a + i], v[i], acc);
    }
    return acc;
}

template <int D>
__global__ void __launch_bounds__(64 * NW)
k_edge_fwd(const int64_t* __restrict__ ends, const float* __restrict__ h, const float* __restrict__ W1,
           const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
           float* __restrict__ logit, int64_t ldo, int64_t sb, int64_t sn, lg_fastdiv fdP, int64_t BP, int64_t ntiles, int dropout,
           float p_drop, float dscale, uint64_t seed, uint32_t salt) {
    using G = EG<D>;
    __shared__ __attribute__((aligned(16))) float ft[TR * G::FS];
    __shared__ float part[NW][TR];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    float aw[G::KS];
#pragma unroll
    for (int ks = 0; ks < G::KS; ++ks) aw[ks] = W1[(16 * w + j) * G::K3 + fk(ks, q)];
    f32x4 b1v, w2v;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        b1v[reg] = b1[16 * w + 4 * q + reg];
        w2v[reg] = W2[16 * w + 4 * q + reg];
    }
    const float bias2 = b2[0];
    const uint32_t key = lg_dropout_key(seed, salt);
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row0 = tile * TR;
        gather_tile<D>(ends, h, ft, row0, BP, fdP, sb, sn);
        __syncthreads();
        const f32x4 acc = hidden_tile<D>(ft, aw, b1v, j, q);
        float s = 0.f;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            float v = fmaxf(acc[reg], 0.f);
            if (dropout) v = lg_dropout(v, p_drop, dscale, key, (row0 + j) * HID + 16 * w + 4 * q + reg);
            s = fmaf(v, w2v[reg], s);
        }
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        if (q == 0) part[w][j] = s;
        __syncthreads();
        if (threadIdx.x < TR) {
            const int64_t r = row0 + threadIdx.x;
            float tot = part[0][threadIdx.x];
#pragma unroll
            for (int i = 1; i < NW; ++i) tot += part[i][threadIdx.x];
            if (r < BP) logit[lg_row_index(r, fdP, ldo)] = tot + bias2;
        }
        __syncthreads();
    }
}

// slab per workgroup: [dW1 128*K3][db1 128][dW2 128][db2 1]
template <int D>
__global__ void __launch_bounds__(64 * NW)
k_edge_bwd(const int64_t* __restrict__ ends, const float* __restrict__ h, const float* __restrict__ W1,
           const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ dlogit, int64_t ldo,
           float* __restrict__ dpipe, float* __restrict__ slab, double* __restrict__ db2slab, int64_t sb, int64_t sn,
           lg_fastdiv fdP,
           int64_t BP, int64_t ntiles, int dropout, float p_drop, float dscale, uint64_t seed, uint32_t salt) {
    using G = EG<D>;
    constexpr int HS = HID + 4;
    constexpr int SL = HID * G::K3 + 2 * HID + 1;
    __shared__ __attribute__((aligned(16))) float ft[TR * G::FS];
    __shared__ __attribute__((aligned(16))) float dh[TR * HS];  // dhid[row][n]
    __shared__ __attribute__((aligned(16))) float red[(G::NSPLIT - 1) * G::DT][64][12];  // dfeat partials
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    // dfeat: wave w handles k-triple kt = w % DT (k-tiles kt, kt+DT, kt+2DT = the u, v, |u-v|
    // columns of the same node feature) over hidden slice hh = w / DT; partials meet in LDS.
    const int kt = w % G::DT, hh = w / G::DT;
    float aw[G::KS];
#pragma unroll
    for (int ks = 0; ks < G::KS; ++ks) aw[ks] = W1[(16 * w + j) * G::K3 + fk(ks, q)];
    float wt[3][G::KPER];  // W1^T fragments: A[k = 16*(kt + s3*DT) + j][n = fk(hh*KPER + ks, q)]
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
        for (int ks = 0; ks < G::KPER; ++ks)
            wt[s3][ks] = W1[fk(hh * G::KPER + ks, q) * G::K3 + 16 * (kt + s3 * G::DT) + j];
    f32x4 b1v, w2v;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        b1v[reg] = b1[16 * w + 4 * q + reg];
        w2v[reg] = W2[16 * w + 4 * q + reg];
    }
    f32x4 dwt[G::MT];
#pragma unroll
    for (int mt = 0; mt < G::MT; ++mt) dwt[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dw2 = f32x4{0.f, 0.f, 0.f, 0.f}, db1 = f32x4{0.f, 0.f, 0.f, 0.f};
    double db2 = 0.0;  // sum of all dlogits: heavy cancellation, kept in fp64 end to end
    const uint32_t key = lg_dropout_key(seed, salt);

    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row0 = tile * TR;
        gather_tile<D>(ends, h, ft, row0, BP, fdP, sb, sn);
        const bool rv = row0 + j < BP;
        const float dl = rv ? dlogit[lg_row_index(row0 + j, fdP, ldo)] : 0.f;
        __syncthreads();
        const f32x4 acc = hidden_tile<D>(ft, aw, b1v, j, q);
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int n = 16 * w + 4 * q + reg;
            const float pre = acc[reg];
            float m = pre > 0.f ? 1.f : 0.f;
            if (dropout) m = lg_keep(key, (row0 + j) * HID + n, p_drop) ? m * dscale : 0.f;
            dw2[reg] = fmaf(dl, pre * m, dw2[reg]);
            const float g = dl * w2v[reg] * m;
            db1[reg] += g;
            dh[j * HS + n] = g;
        }
        if (w == 0 && q == 0) db2 += static_cast<double>(dl);
        __syncthreads();
        // dW1^T[k][n] += sum_rows feat[row][k] * dhid[row][n]   (rows = 4q + kk)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int row = 4 * q + kk;
            const float bv = dh[row * HS + 16 * w + j];
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt) dwt[mt] = mfma(feat1<D>(ft, row, 16 * mt + j), bv, dwt[mt]);
        }
        {
            // dfeat^T[k][row] = sum_n W1[n][k] dhid[row][n] over this wave's hidden slice
            f32x4 cu = f32x4{0.f, 0.f, 0.f, 0.f}, cv = cu, ca = cu;
#pragma unroll
            for (int a = 0; a < G::KPER / 4; ++a) {
                const f32x4 g4 = ld4(dh + j * HS + 16 * (hh * G::KPER / 4 + a) + 4 * q);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    cu = mfma(wt[0][4 * a + i], g4[i], cu);
                    cv = mfma(wt[1][4 * a + i], g4[i], cv);
                    ca = mfma(wt[2][4 * a + i], g4[i], ca);
                }
            }
            if (hh > 0) {
                float* rp = &red[(hh - 1) * G::DT + kt][lane][0];
                st4(rp, cu);
                st4(rp + 4, cv);
                st4(rp + 8, ca);
            }
            __syncthreads();
            if (hh == 0) {
#pragma unroll
                for (int o = 1; o < G::NSPLIT; ++o) {  // fixed order -> deterministic
                    const float* rp = &red[(o - 1) * G::DT + kt][lane][0];
                    cu += ld4(rp);
                    cv += ld4(rp + 4);
                    ca += ld4(rp + 8);
                }
                if (rv) {
                    const int ku = 16 * kt + 4 * q;
                    const f32x4 u = ld4(ft + j * G::FS + ku), v = ld4(ft + j * G::FS + D + ku);
                    f32x4 du, dv;
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) {
                        const float d = u[reg] - v[reg];
                        const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
                        du[reg] = cu[reg] + sg * ca[reg];
                        dv[reg] = cv[reg] - sg * ca[reg];
                    }
                    float* o = dpipe + (row0 + j) * 2 * D + ku;
                    st4(o, du);
                    st4(o + D, dv);
                }
            }
        }
        __syncthreads();
    }

    float* out = slab + static_cast<int64_t>(blockIdx.x) * SL;
#pragma unroll
    for (int mt = 0; mt < G::MT; ++mt)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) out[(16 * w + j) * G::K3 + 16 * mt + 4 * q + reg] = dwt[mt][reg];
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            dw2[reg] += __shfl_xor(dw2[reg], off);
            db1[reg] += __shfl_xor(db1[reg], off);
        }
        db2 += __shfl_xor(db2, off);
    }
    if (j == 0) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            out[HID * G::K3 + 16 * w + 4 * q + reg] = db1[reg];
            out[HID * G::K3 + HID + 16 * w + 4 * q + reg] = dw2[reg];
        }
    }
    if (w == 0 && lane == 0) db2slab[blockIdx.x] = db2;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

int bwd_grid(int64_t ntiles) { return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ntiles, lg_num_cus()))); }

}  // namespace

extern "C" int lg_edge_head_fwd(const int64_t* ends, const float* h, const float* w1, const float* b1,
                                const float* w2, const float* b2, float* logits, int64_t ldo, int64_t B, int64_t N,
                                int64_t P,
                                int64_t D, int64_t hidden, int flags, float dropout_p, uint64_t seed, uint32_t salt,
                                lg_stream_t stream) {
    if (B < 0 || N <= 0 || P < 0) return LG_EINVAL;
    if (hidden != HID || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const int dropout = (flags & LG_F_DROPOUT) ? 1 : 0;
    if (dropout && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    const int64_t BP = B * P;
    if (BP == 0) return LG_OK;
    if (!ends || !h || !w1 || !b1 || !w2 || !b2 || !logits || ldo < P) return LG_EINVAL;
    if (BP >= kLgMaxRows) return LG_EUNSUPPORTED;
    const lg_fastdiv fdP = lg_make_fastdiv(static_cast<uint32_t>(P));
    const bool nm = (flags & LG_F_NODE_MAJOR) != 0;  // h is [N][B][D] instead of [B][N][D]
    const int64_t sb = nm ? 1 : N, sn = nm ? B : 1;
    const int64_t ntiles = cdiv(BP, TR);
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ntiles, 4LL * lg_num_cus()));
    const float scale = dropout ? 1.0f / (1.0f - dropout_p) : 1.0f;
    hipStream_t s = lg_stream(stream);
    if (D == 64)
        k_edge_fwd<64><<<grid, 64 * NW, 0, s>>>(ends, h, w1, b1, w2, b2, logits, ldo, sb, sn, fdP, BP, ntiles, dropout, dropout_p,
                                                scale, seed, salt);
    else
        k_edge_fwd<32><<<grid, 64 * NW, 0, s>>>(ends, h, w1, b1, w2, b2, logits, ldo, sb, sn, fdP, BP, ntiles, dropout, dropout_p,
                                                scale, seed, salt);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int64_t lg_edge_head_bwd_workspace_bytes(int64_t B, int64_t P, int64_t D, int64_t hidden) {
    if (B < 0 || P < 0 || hidden != HID || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const int64_t SL = HID * 3 * D + 2 * HID + 1;
    const int64_t G = bwd_grid(cdiv(std::max<int64_t>(B * P, 1), TR));
    return ((G * SL * 4 + 255) & ~int64_t(255)) + G * 8;
}

extern "C" int lg_edge_head_bwd(const int64_t* ends, const float* h, const float* w1, const float* b1,
                                const float* w2, const float* dlogits, int64_t ldo, float* dpipe, float* dw1,
                                float* db1,
                                float* dw2, float* db2, int64_t B, int64_t N, int64_t P, int64_t D, int64_t hidden,
                                int flags, float dropout_p, uint64_t seed, uint32_t salt, void* workspace,
                                lg_stream_t stream) {
    if (B < 0 || N <= 0 || P < 0) return LG_EINVAL;
    if (hidden != HID || (D != 32 && D != 64)) return LG_EUNSUPPORTED;
    const int dropout = (flags & LG_F_DROPOUT) ? 1 : 0;
    if (dropout && !(dropout_p >= 0.f && dropout_p < 1.f)) return LG_EINVAL;
    if (!h || !w1 || !b1 || !w2 || !dw1 || !db1 || !dw2 || !db2 || !workspace) return LG_EINVAL;
    const int64_t BP = B * P;
    if (BP > 0 && (!ends || !dlogits || !dpipe || ldo < P)) return LG_EINVAL;
    if (BP >= kLgMaxRows) return LG_EUNSUPPORTED;
    const lg_fastdiv fdP = lg_make_fastdiv(static_cast<uint32_t>(std::max<int64_t>(P, 1)));
    const bool nm = (flags & LG_F_NODE_MAJOR) != 0;  // h is [N][B][D] instead of [B][N][D]
    const int64_t sb = nm ? 1 : N, sn = nm ? B : 1;
    const int64_t ntiles = cdiv(std::max<int64_t>(BP, 1), TR);
    const int grid = bwd_grid(ntiles);
    const float scale = dropout ? 1.0f / (1.0f - dropout_p) : 1.0f;
    const int64_t SL = HID * 3 * D + 2 * HID + 1;
    float* slab = static_cast<float*>(workspace);
    double* dslab = reinterpret_cast<double*>(static_cast<char*>(workspace) + ((grid * SL * 4 + 255) & ~int64_t(255)));
    hipStream_t s = lg_stream(stream);
    if (BP == 0) {
        if (hipMemsetAsync(slab, 0, SL * grid * sizeof(float), s) != hipSuccess) return LG_EHIP;
        if (hipMemsetAsync(dslab, 0, grid * sizeof(double), s) != hipSuccess) return LG_EHIP;
    } else if (D == 64) {
        k_edge_bwd<64><<<grid, 64 * NW, 0, s>>>(ends, h, w1, b1, w2, dlogits, ldo, dpipe, slab, dslab, sb, sn, fdP, BP, ntiles, dropout,
                                                dropout_p, scale, seed, salt);
    } else {
        k_edge_bwd<32><<<grid, 64 * NW, 0, s>>>(ends, h, w1, b1, w2, dlogits, ldo, dpipe, slab, dslab, sb, sn, fdP, BP, ntiles, dropout,
                                                dropout_p, scale, seed, salt);
    }
    LG_RET_IF_LAUNCH_FAILED();
    const int64_t K3 = 3 * D;
    const LgSlabSeg segs[3] = {{0, HID * K3, dw1}, {HID * K3, HID, db1}, {HID * K3 + HID, HID, dw2}};
    return lg_launch_slab_reduce_multi(slab, grid, SL, segs, 3, dslab, db2, s);
}
