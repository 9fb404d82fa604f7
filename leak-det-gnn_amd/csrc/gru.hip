// SharedSensorGRUEncoder (reference detector.py:28-73) as two fused HIP kernels.
//
// One nn.GRU(input 1 [+9 time features], hidden 64, 1 layer) runs over B*S
// independent sequences (sequence q = b*S + s) of L steps; the encoder keeps h_L.
// PyTorch gate order / formulas:
//   r = sig(W_ir x + b_ir + W_hr h + b_hr)     z = sig(W_iz x + b_iz + W_hz h + b_hz)
//   n = tanh(W_in x + b_in + r * (W_hn h + b_hn))     h' = (1 - z) * n + z * h
//
// Work split: one 256-thread workgroup = 16 sequences; wave w owns hidden units
// [16w, 16w+16), i.e. gate rows {w, 4+w, 8+w} of the 12 16-row tiles.  Gates are
// computed transposed, G^T (192 x 16 seq) = W (192 x K) * [h;x]^T, with
// v_mfma_f32_16x16x4_f32 (exact fp32).  With the K index permuted as
// k = f(ks, q) = 16*(ks>>2) + 4q + (ks&3), the accumulator layout of the new h IS
// the B-operand layout of the next step's h, so the recurrence stays in registers;
// the four waves swap their quarters of h through a 4 KiB LDS slot once per step.
// The input projection is folded into the same accumulators (K = 10 padded to 12),
// so x = [residual, tfeat] is read straight from (B, L, S) / (B, L, 9) — the
// (B*S, L, 10) concatenation of the reference (detector.py:62-67) is never built.
//
// Backward (BPTT) recomputes the gates from the saved h_{t-1}, exchanges dG^T
// through LDS, and accumulates dW_hh / dW_ih / db in registers per wave (each wave
// owns disjoint gate rows), written once per workgroup to a slab and reduced in
// fixed order -> deterministic.
#include <algorithm>
#include "common.h"
#include "reduce.h"

namespace {

constexpr int H = 64;
constexpr int G3 = 3 * H;
constexpr int TS = 16;  // sequences per workgroup

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int fk(int ks, int q) { return 16 * (ks >> 2) + 4 * q + (ks & 3); }
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

template <bool USE_TIME>
__device__ __forceinline__ float load_x(const float* __restrict__ resid, const float* __restrict__ tfeat, int64_t b,
                                        int64_t s, int t, int k, int L, int S, bool valid) {
    if (!valid) return 0.f;
    if (k == 0) return resid[(b * L + t) * S + s];
    if (USE_TIME && k <= 9) return tfeat[(b * L + t) * 9 + (k - 1)];
    return 0.f;
}

template <bool USE_TIME>
__global__ void __launch_bounds__(256)
k_gru_fwd(const float* __restrict__ resid, const float* __restrict__ tfeat, const float* __restrict__ Wih,
          const float* __restrict__ Whh, const float* __restrict__ bih, const float* __restrict__ bhh,
          float* __restrict__ hs, float* __restrict__ hout, int B, int L, int S) {
    constexpr int I = USE_TIME ? 10 : 1;
    __shared__ __attribute__((aligned(16))) float hx[2][64][16];
    const int64_t Nseq = static_cast<int64_t>(B) * S;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const int64_t seq = static_cast<int64_t>(blockIdx.x) * TS + j;
    const bool valid = seq < Nseq;
    const int64_t b = valid ? seq / S : 0, s = valid ? seq - b * S : 0;

    float ah[3][16], ax[3][3];
#pragma unroll
    for (int gi = 0; gi < 3; ++gi) {
        const int row = gi * H + 16 * w + j;  // A-operand row of this lane
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) ah[gi][ks] = Whh[row * H + fk(ks, q)];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int k = 4 * kx + q;
            ax[gi][kx] = k < I ? Wih[row * I + k] : 0.f;
        }
    }
    f32x4 br, bz, bhn, bin;  // D-layout rows 4q+reg of each gate tile
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int c = 16 * w + 4 * q + reg;
        br[reg] = bih[c] + bhh[c];
        bz[reg] = bih[H + c] + bhh[H + c];
        bhn[reg] = bhh[2 * H + c];
        bin[reg] = bih[2 * H + c];
    }
    float hf[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) hf[i] = 0.f;

    float xv[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) xv[kx] = load_x<USE_TIME>(resid, tfeat, b, s, 0, 4 * kx + q, L, S, valid);

    for (int t = 0; t < L; ++t) {
        f32x4 ar = br, az = bz, ahn = bhn, ain = bin;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            ar = mfma(ax[0][kx], xv[kx], ar);
            az = mfma(ax[1][kx], xv[kx], az);
            ain = mfma(ax[2][kx], xv[kx], ain);
        }
        if (t + 1 < L) {  // prefetch next step's inputs under the MFMA chain
#pragma unroll
            for (int kx = 0; kx < 3; ++kx)
                xv[kx] = load_x<USE_TIME>(resid, tfeat, b, s, t + 1, 4 * kx + q, L, S, valid);
        }
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
            ar = mfma(ah[0][ks], hf[ks], ar);
            az = mfma(ah[1][ks], hf[ks], az);
            ahn = mfma(ah[2][ks], hf[ks], ahn);
        }
        f32x4 hn;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const float r = sigm(ar[reg]);
            const float z = sigm(az[reg]);
            const float n = tanhf(ain[reg] + r * ahn[reg]);
            hn[reg] = (1.f - z) * n + z * hf[4 * w + reg];
        }
        st4(&hx[t & 1][lane][4 * w], hn);
        if (hs && valid) st4(hs + ((static_cast<int64_t>(t) * Nseq + seq) * H + 16 * w + 4 * q), hn);
        __syncthreads();
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const f32x4 v = ld4(&hx[t & 1][lane][4 * a]);
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) hf[4 * a + reg] = v[reg];
        }
    }
    if (valid) {
        f32x4 v;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) v[reg] = hf[4 * w + reg];
        st4(hout + seq * H + 16 * w + 4 * q, v);
    }
}

// slab layout per workgroup: [dWhh 192*64][dWih 192*I][dbih 192][dbhh 192]
template <bool USE_TIME, bool NEED_DX>
__global__ void __launch_bounds__(256)
k_gru_bwd(const float* __restrict__ resid, const float* __restrict__ tfeat, const float* __restrict__ Wih,
          const float* __restrict__ Whh, const float* __restrict__ bih, const float* __restrict__ bhh,
          const float* __restrict__ hs, const float* __restrict__ dhL, float* __restrict__ dx,
          float* __restrict__ slab, int B, int L, int S) {
    constexpr int I = USE_TIME ? 10 : 1;
    constexpr int SWH = H + 1;
    constexpr int SLAB = G3 * H + G3 * I + 2 * G3;
    __shared__ __attribute__((aligned(16))) float whh[G3 * SWH];
    __shared__ __attribute__((aligned(16))) float wih[G3 * 16];
    __shared__ __attribute__((aligned(16))) float dg[64][64 + 4];
    const int64_t Nseq = static_cast<int64_t>(B) * S;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
    const int64_t seq0 = static_cast<int64_t>(blockIdx.x) * TS;
    const int64_t seq = seq0 + j;
    const bool valid = seq < Nseq;
    const int64_t b = valid ? seq / S : 0, s = valid ? seq - b * S : 0;

    for (int i = threadIdx.x; i < G3 * H; i += 256) whh[(i / H) * SWH + (i % H)] = Whh[i];
    for (int i = threadIdx.x; i < G3 * 16; i += 256) wih[i] = (i % 16) < I ? Wih[(i / 16) * I + (i % 16)] : 0.f;
    __syncthreads();

    float ah[3][16], ax[3][3];
#pragma unroll
    for (int gi = 0; gi < 3; ++gi) {
        const int row = gi * H + 16 * w + j;
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) ah[gi][ks] = whh[row * SWH + fk(ks, q)];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) ax[gi][kx] = wih[row * 16 + 4 * kx + q];
    }
    f32x4 br, bz, bhn, bin;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int c = 16 * w + 4 * q + reg;
        br[reg] = bih[c] + bhh[c];
        bz[reg] = bih[H + c] + bhh[H + c];
        bhn[reg] = bhh[2 * H + c];
        bin[reg] = bih[2 * H + c];
    }

    f32x4 dh = f32x4{0.f, 0.f, 0.f, 0.f};
    if (valid) dh = ld4(dhL + seq * H + 16 * w + 4 * q);

    f32x4 dwh[3][4], dwi[3], dbg[3], dbin;
#pragma unroll
    for (int gi = 0; gi < 3; ++gi) {
        dwi[gi] = f32x4{0.f, 0.f, 0.f, 0.f};
        dbg[gi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) dwh[gi][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    dbin = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int t = L - 1; t >= 0; --t) {
        // h_{t-1} in B layout (lane-local) and x_t
        float hf[16];
        if (t > 0 && valid) {
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const f32x4 v = ld4(hs + ((static_cast<int64_t>(t - 1) * Nseq + seq) * H + 16 * a + 4 * q));
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) hf[4 * a + reg] = v[reg];
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) hf[i] = 0.f;
        }
        float xv[3];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) xv[kx] = load_x<USE_TIME>(resid, tfeat, b, s, t, 4 * kx + q, L, S, valid);

        f32x4 ar = br, az = bz, ahn = bhn, ain = bin;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            ar = mfma(ax[0][kx], xv[kx], ar);
            az = mfma(ax[1][kx], xv[kx], az);
            ain = mfma(ax[2][kx], xv[kx], ain);
        }
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
            ar = mfma(ah[0][ks], hf[ks], ar);
            az = mfma(ah[1][ks], hf[ks], az);
            ahn = mfma(ah[2][ks], hf[ks], ahn);
        }
        f32x4 gr, gz, ghn, gin, dhp;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const float r = sigm(ar[reg]);
            const float z = sigm(az[reg]);
            const float n = tanhf(ain[reg] + r * ahn[reg]);
            const float hp = hf[4 * w + reg];
            const float d = dh[reg];
            const float dn = d * (1.f - z);
            const float dz = d * (hp - n);
            dhp[reg] = d * z;
            const float dnp = dn * (1.f - n * n);
            gin[reg] = dnp;
            ghn[reg] = dnp * r;
            const float drr = dnp * ahn[reg];
            gr[reg] = drr * r * (1.f - r);
            gz[reg] = dz * z * (1.f - z);
        }
        dbg[0] += gr;
        dbg[1] += gz;
        dbg[2] += ghn;
        dbin += gin;
        __syncthreads();  // previous step's readers of dg are done
        st4(&dg[lane][4 * w], gr);
        st4(&dg[lane][16 + 4 * w], gz);
        st4(&dg[lane][32 + 4 * w], ghn);
        st4(&dg[lane][48 + 4 * w], gin);
        __syncthreads();

        // dh_{t-1}[c'] = dh*z + sum_g W_hh[g][c'] dgh[g]   (rows c' = 16w + 4q + reg)
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 48; ++ks) acc = mfma(whh[fk(ks, q) * SWH + 16 * w + j], dg[lane][ks], acc);
        dh = dhp + acc;

        // dW_hh[g][c] += sum_seq dgh[g][seq] h_{t-1}[seq][c],  dW_ih likewise with dgi, x
        // A[g_local = j][k = seq 4q+kk] was written by lane (seq) + 16*(j>>2) at entry 16gi + 4w + (j&3)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int src = (4 * q + kk) + 16 * (j >> 2);
            const float a0 = dg[src][4 * w + (j & 3)];
            const float a1 = dg[src][16 + 4 * w + (j & 3)];
            const float a2 = dg[src][32 + 4 * w + (j & 3)];
            const float a2i = dg[src][48 + 4 * w + (j & 3)];
            const int64_t sq = seq0 + 4 * q + kk;
            const bool v2 = sq < Nseq && t > 0;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float hb = v2 ? hs[(static_cast<int64_t>(t - 1) * Nseq + sq) * H + 16 * nt + j] : 0.f;
                dwh[0][nt] = mfma(a0, hb, dwh[0][nt]);
                dwh[1][nt] = mfma(a1, hb, dwh[1][nt]);
                dwh[2][nt] = mfma(a2, hb, dwh[2][nt]);
            }
            const bool vx = sq < Nseq;
            const int64_t bb = vx ? sq / S : 0, ss = vx ? sq - bb * S : 0;
            const float xb = j < I ? load_x<USE_TIME>(resid, tfeat, bb, ss, t, j, L, S, vx) : 0.f;
            dwi[0] = mfma(a0, xb, dwi[0]);
            dwi[1] = mfma(a1, xb, dwi[1]);
            dwi[2] = mfma(a2i, xb, dwi[2]);
        }
        if (NEED_DX && w == 0) {
            // dx^T[k][seq] = sum_g W_ih[g][k] dgi[g][seq]   (k = 4q + reg < I)
            f32x4 dxa = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 48; ++ks) {
                const float bv = ks < 32 ? dg[lane][ks] : dg[lane][ks + 16];
                dxa = mfma(wih[fk(ks, q) * 16 + j], bv, dxa);
            }
            if (valid) {
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) {
                    const int k = 4 * q + reg;
                    if (k < I) dx[(seq * L + t) * I + k] = dxa[reg];
                }
            }
        }
    }

    // per-workgroup slab: waves own disjoint gate rows, no cross-wave reduction needed
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
            for (int nt = 0; nt < 4; ++nt) oWhh[g * H + 16 * nt + j] = dwh[gi][nt][reg];
            if (j < I) oWih[g * I + j] = dwi[gi][reg];
        }
    // biases: sum the 16 sequence lanes (same q) of each lane-local row
#pragma unroll
    for (int off = 1; off < 16; off <<= 1)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
#pragma unroll
            for (int gi = 0; gi < 3; ++gi) dbg[gi][reg] += __shfl_xor(dbg[gi][reg], off);
            dbin[reg] += __shfl_xor(dbin[reg], off);
        }
    if (j == 0) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int c = 16 * w + 4 * q + reg;
            obhh[c] = dbg[0][reg];
            obhh[H + c] = dbg[1][reg];
            obhh[2 * H + c] = dbg[2][reg];
            obih[c] = dbg[0][reg];
            obih[H + c] = dbg[1][reg];
            obih[2 * H + c] = dbin[reg];
        }
    }
}

inline int64_t nblocks_seq(int64_t nseq) { return (nseq + TS - 1) / TS; }

}  // namespace

extern "C" int64_t lg_gru_bwd_workspace_bytes(int64_t B, int64_t S, int64_t I) {
    if (B < 0 || S < 0 || (I != 1 && I != 10)) return LG_EINVAL;
    const int64_t slab = G3 * H + G3 * I + 2 * G3;
    return std::max<int64_t>(1, nblocks_seq(B * S)) * slab * static_cast<int64_t>(sizeof(float));
}

extern "C" int lg_gru_fwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
                          const float* b_ih, const float* b_hh, float* h_seq, float* h_last, int64_t B, int64_t L,
                          int64_t S, int64_t I, int64_t Hd, lg_stream_t stream) {
    if (B < 0 || L <= 0 || S <= 0 || L > INT32_MAX || S > INT32_MAX || B * S > INT32_MAX / 2) return LG_EINVAL;
    if (Hd != H || (I != 1 && I != 10)) return LG_EUNSUPPORTED;
    if (!residual || !w_ih || !w_hh || !b_ih || !b_hh || !h_last || (I == 10 && !tfeat)) return LG_EINVAL;
    if (B == 0) return LG_OK;
    const unsigned grid = static_cast<unsigned>(nblocks_seq(B * S));
    hipStream_t s = lg_stream(stream);
    if (I == 10)
        k_gru_fwd<true><<<grid, 256, 0, s>>>(residual, tfeat, w_ih, w_hh, b_ih, b_hh, h_seq, h_last, (int)B, (int)L,
                                              (int)S);
    else
        k_gru_fwd<false><<<grid, 256, 0, s>>>(residual, tfeat, w_ih, w_hh, b_ih, b_hh, h_seq, h_last, (int)B, (int)L,
                                               (int)S);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_gru_bwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
                          const float* b_ih, const float* b_hh, const float* h_seq, const float* dh_last, float* dx,
                          float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, int64_t B, int64_t L, int64_t S,
                          int64_t I, int64_t Hd, void* workspace, lg_stream_t stream) {
    if (B < 0 || L <= 0 || S <= 0 || L > INT32_MAX || S > INT32_MAX || B * S > INT32_MAX / 2) return LG_EINVAL;
    if (Hd != H || (I != 1 && I != 10)) return LG_EUNSUPPORTED;
    if (!residual || !w_ih || !w_hh || !b_ih || !b_hh || !h_seq || !dh_last || !dw_ih || !dw_hh || !db_ih ||
        !db_hh || !workspace || (I == 10 && !tfeat))
        return LG_EINVAL;
    hipStream_t s = lg_stream(stream);
    const int nb = static_cast<int>(std::max<int64_t>(1, nblocks_seq(B * S)));
    float* slab = static_cast<float*>(workspace);
    const int len = static_cast<int>(G3 * H + G3 * I + 2 * G3);
    if (B == 0) {
        if (hipMemsetAsync(slab, 0, sizeof(float) * len, s) != hipSuccess) return LG_EHIP;
    } else {
        const unsigned grid = static_cast<unsigned>(nblocks_seq(B * S));
#define LG_GRU_BWD(UT, DX)                                                                                        \
    k_gru_bwd<UT, DX><<<grid, 256, 0, s>>>(residual, tfeat, w_ih, w_hh, b_ih, b_hh, h_seq, dh_last, dx, slab,     \
                                           (int)B, (int)L, (int)S)
        if (I == 10) {
            if (dx) LG_GRU_BWD(true, true); else LG_GRU_BWD(true, false);
        } else {
            if (dx) LG_GRU_BWD(false, true); else LG_GRU_BWD(false, false);
        }
#undef LG_GRU_BWD
        LG_RET_IF_LAUNCH_FAILED();
    }
    const int G = B == 0 ? 1 : nb;
    const int64_t nWhh = G3 * H, nWih = G3 * I;
    int rc = lg_launch_slab_reduce(slab, G, len, nWhh, dw_hh, s);
    if (rc == LG_OK) rc = lg_launch_slab_reduce(slab + nWhh, G, len, nWih, dw_ih, s);
    if (rc == LG_OK) rc = lg_launch_slab_reduce(slab + nWhh + nWih, G, len, G3, db_ih, s);
    if (rc == LG_OK) rc = lg_launch_slab_reduce(slab + nWhh + nWih + G3, G, len, G3, db_hh, s);
    return rc;
}
