// K4 (gcn_norm + CSR), pipe-incidence CSR and K3 (batchified edge index).
//
// These run once per graph / per model, so they favour determinism over speed:
// counts by integer atomics (order-free), one-block exclusive scan, slot fill by
// atomics, then a per-row insertion sort that restores ascending edge order so the
// CSR is bit-identical from run to run and visits each row's entries in the order
// PyG's scatter_add does (edges ascending, appended self loop last).
#include <algorithm>
#include <utility>
#include <vector>

#include "common.h"

namespace {

constexpr int kThreads = 256;

__global__ void k_count_edges(const int64_t* __restrict__ ei, int64_t E, int64_t N, int drop_loops,
                              int32_t* __restrict__ cnt, int32_t* __restrict__ cnt_t) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int64_t s = ei[e], d = ei[E + e];
    if (s < 0 || s >= N || d < 0 || d >= N) return;  // host validates; never write out of range
    if (drop_loops && s == d) return;
    atomicAdd(&cnt[d], 1);
    atomicAdd(&cnt_t[s], 1);
}

// rowptr[n] = sum_{m<n} (cnt[m] + extra); rowptr[N] = total.  One block.
__global__ void __launch_bounds__(1024) k_scan_rows(const int32_t* __restrict__ cnt, int64_t N, int extra,
                                                    int32_t* __restrict__ rowptr) {
    __shared__ int32_t part[1024];
    const int t = threadIdx.x;
    const int64_t chunk = (N + 1023) / 1024;
    const int64_t lo = t * chunk, hi = min<int64_t>(N, lo + chunk);
    int32_t sum = 0;
    for (int64_t n = lo; n < hi; ++n) sum += cnt[n] + extra;
    part[t] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
        const int32_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int32_t run = part[t] - sum;  // exclusive prefix of this chunk
    for (int64_t n = lo; n < hi; ++n) {
        rowptr[n] = run;
        run += cnt[n] + extra;
    }
    if (t == 1023) rowptr[N] = part[1023];
}

__global__ void k_fill_edges(const int64_t* __restrict__ ei, int64_t E, int64_t N, int drop_loops,
                             const int32_t* __restrict__ rowptr, const int32_t* __restrict__ rowptr_t,
                             int32_t* __restrict__ cur, int32_t* __restrict__ cur_t, int32_t* __restrict__ item,
                             int32_t* __restrict__ item_t) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int64_t s = ei[e], d = ei[E + e];
    if (s < 0 || s >= N || d < 0 || d >= N) return;
    if (drop_loops && s == d) return;
    item[rowptr[d] + atomicAdd(&cur[d], 1)] = static_cast<int32_t>(e);
    item_t[rowptr_t[s] + atomicAdd(&cur_t[s], 1)] = static_cast<int32_t>(e);
}

__device__ __forceinline__ void insertion_sort(int32_t* a, int n) {
    for (int i = 1; i < n; ++i) {
        const int32_t v = a[i];
        int j = i - 1;
        while (j >= 0 && a[j] > v) {
            a[j + 1] = a[j];
            --j;
        }
        a[j + 1] = v;
    }
}

// Per row: restore ascending edge order, then write col / w (and the self loop).
__global__ void k_finalize(const int64_t* __restrict__ ei, int64_t E, int64_t N, int add_loops, int normalize,
                           float fill, const int32_t* __restrict__ cnt, const int32_t* __restrict__ cnt_t,
                           const int32_t* __restrict__ rowptr, const int32_t* __restrict__ rowptr_t,
                           int32_t* __restrict__ item, int32_t* __restrict__ item_t, float* __restrict__ dis,
                           int32_t* __restrict__ col, float* __restrict__ w, int32_t* __restrict__ col_t,
                           float* __restrict__ w_t, int phase) {
    const int64_t n = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (n >= N) return;
    if (phase == 0) {
        insertion_sort(item + rowptr[n], cnt[n]);
        insertion_sort(item_t + rowptr_t[n], cnt_t[n]);
        // deg = scatter_add(edge_weight, dst): unit weights plus the loop's fill value.
        const float deg = static_cast<float>(cnt[n]) + (add_loops ? fill : 0.0f);
        // deg.pow(-0.5) as torch evaluates it in fp32: sqrt rounded to fp32, then 1/x rounded
        // to fp32.  Each step is done in fp64 and rounded once, which is exact for fp32
        // sqrt and division (53 >= 2*24 + 2), so dis is bit-identical to the CPU reference.
        const float sq = static_cast<float>(sqrt(static_cast<double>(deg)));
        dis[n] = deg > 0.0f ? static_cast<float>(1.0 / static_cast<double>(sq)) : 0.0f;  // inf -> 0
        return;
    }
    // phase 1: all dis[] are final.
    const int32_t b = rowptr[n], c = cnt[n];
    const float dn = dis[n];
    for (int i = 0; i < c; ++i) {
        const int32_t e = item[b + i];
        const int32_t s = static_cast<int32_t>(ei[e]);
        col[b + i] = s;
        w[b + i] = normalize ? (dis[s] * 1.0f) * dn : 1.0f;
    }
    if (add_loops) {
        col[b + c] = static_cast<int32_t>(n);
        w[b + c] = normalize ? (dn * fill) * dn : fill;
    }
    const int32_t bt = rowptr_t[n], ct = cnt_t[n];
    for (int i = 0; i < ct; ++i) {
        const int32_t e = item_t[bt + i];
        const int32_t d = static_cast<int32_t>(ei[E + e]);
        col_t[bt + i] = d;
        w_t[bt + i] = normalize ? (dn * 1.0f) * dis[d] : 1.0f;
    }
    if (add_loops) {
        col_t[bt + ct] = static_cast<int32_t>(n);
        w_t[bt + ct] = normalize ? (dn * fill) * dn : fill;
    }
}

__global__ void k_count_inc(const int64_t* __restrict__ ends, int64_t P2, int64_t N, int32_t* __restrict__ cnt) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= P2) return;
    const int64_t n = ends[i];
    if (n < 0 || n >= N) return;
    atomicAdd(&cnt[n], 1);
}

__global__ void k_fill_inc(const int64_t* __restrict__ ends, int64_t P2, int64_t N,
                           const int32_t* __restrict__ rowptr, int32_t* __restrict__ cur,
                           int32_t* __restrict__ item) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= P2) return;
    const int64_t n = ends[i];
    if (n < 0 || n >= N) return;
    item[rowptr[n] + atomicAdd(&cur[n], 1)] = static_cast<int32_t>(i);
}

__global__ void k_sort_inc(int64_t N, const int32_t* __restrict__ rowptr, int32_t* __restrict__ item) {
    const int64_t n = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (n >= N) return;
    insertion_sort(item + rowptr[n], rowptr[n + 1] - rowptr[n]);
}

__global__ void k_batchify(const int64_t* __restrict__ ei, int64_t E, int64_t N, int64_t B,
                           int64_t* __restrict__ out) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= B * E) return;
    const int64_t b = i / E, e = i - b * E;
    const int64_t off = b * N;
    out[i] = ei[e] + off;
    out[B * E + i] = ei[E + e] + off;
}

// Node table of the node-major kernels: one 64-byte record per node, read by ONE scalar
// load (s_load_dwordx16) per tile: {e0, e1, (col, w bits) x kLgNmInline, self, 0}.
// self = position k < kLgNmInline of the entry whose col is the node itself (-1: none
// inline); the backward reads that entry's block as the tile's own dz rows.
// thread i writes record i (node i) and record N + i (node order[i], the schedule section)
__global__ void k_nm_table(const int32_t* __restrict__ rowptr, const int2* __restrict__ pairs, int64_t N,
                           const int32_t* __restrict__ order, int32_t* __restrict__ tab) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= 2 * N) return;
    const int64_t n = i < N ? i : (order ? order[i - N] : i - N);
    const int e0 = rowptr[n], e1 = rowptr[n + 1];
    int v[16];
    v[0] = e0;
    v[1] = e1;
    int self = -1;
#pragma unroll
    for (int k = 0; k < kLgNmInline; ++k) {
        const bool have = e0 + k < e1;
        const int2 p = have ? pairs[e0 + k] : int2{0, 0};
        v[2 + 2 * k] = p.x;
        v[3 + 2 * k] = p.y;
        if (have && self < 0 && p.x == static_cast<int>(n)) self = k;
    }
    v[2 + 2 * kLgNmInline] = self;
    v[3 + 2 * kLgNmInline] = static_cast<int>(n);
    int4* o = reinterpret_cast<int4*>(tab + 16 * i);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = int4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
}

// Sensor marks of a node table for the compressed layer-0 input (lg_gcn_fwd_nm_x0): every
// (col, w) entry whose col has a sensor slot gets col = kLgSensorCol | slot; pos_slot[i] =
// node_slot of the schedule section's record N + i.
__global__ void k_nm_mark(const int32_t* __restrict__ tab, const int2* __restrict__ pairs, int64_t N, int64_t nnz,
                          const int32_t* __restrict__ node_slot, int32_t* __restrict__ tab_out,
                          int2* __restrict__ pairs_out, int32_t* __restrict__ pos_slot) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    auto mark = [&](int32_t c) { return (c >= 0 && c < N && node_slot[c] >= 0) ? (kLgSensorCol | node_slot[c]) : c; };
    if (i < 2 * N) {
        const int4* t = reinterpret_cast<const int4*>(tab + 16 * i);
        int v[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int4 q = t[k];
            v[4 * k] = q.x;
            v[4 * k + 1] = q.y;
            v[4 * k + 2] = q.z;
            v[4 * k + 3] = q.w;
        }
#pragma unroll
        for (int k = 0; k < kLgNmInline; ++k)
            if (v[0] + k < v[1]) v[2 + 2 * k] = mark(v[2 + 2 * k]);
        int4* o = reinterpret_cast<int4*>(tab_out + 16 * i);
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = int4{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
        if (i >= N) pos_slot[i - N] = node_slot[v[15]];
    }
    if (i < nnz) {
        const int2 p = pairs[i];
        pairs_out[i] = int2{mark(p.x), p.y};
    }
}

inline unsigned nblocks(int64_t n) { return static_cast<unsigned>((n + kThreads - 1) / kThreads); }
inline int64_t align256(int64_t b) { return (b + 255) & ~int64_t(255); }

}  // namespace

extern "C" int64_t lg_graph_workspace_bytes(int64_t E, int64_t N) {
    if (E < 0 || N < 0) return LG_EINVAL;
    // cnt, cnt_t, cur, cur_t, dis : N each; item, item_t : E + N each (indexed by CSR
    // position, which includes the self-loop slot of every row)
    return align256(4 * (5 * N + 2 * (E + N)) + 64);
}

extern "C" int lg_graph_build(const int64_t* edge_index, int64_t E, int64_t N, int add_self_loops, int normalize,
                              float fill_value, int32_t* rowptr, int32_t* col, float* w, int32_t* rowptr_t,
                              int32_t* col_t, float* w_t, void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    if (E < 0 || N <= 0 || N > INT32_MAX / 2 || E > INT32_MAX / 2) return LG_EINVAL;
    if ((E > 0 && !edge_index) || !rowptr || !col || !w || !rowptr_t || !col_t || !w_t || !workspace)
        return LG_EINVAL;
    if (ws_bytes < lg_graph_workspace_bytes(E, N)) return LG_EINVAL;
    hipStream_t s = lg_stream(stream);
    int32_t* cnt = static_cast<int32_t*>(workspace);
    int32_t* cnt_t = cnt + N;
    int32_t* cur = cnt_t + N;
    int32_t* cur_t = cur + N;
    float* dis = reinterpret_cast<float*>(cur_t + N);
    int32_t* item = reinterpret_cast<int32_t*>(dis + N);
    int32_t* item_t = item + (E + N);
    if (hipMemsetAsync(cnt, 0, sizeof(int32_t) * 4 * N, s) != hipSuccess) return LG_EHIP;
    const int drop = add_self_loops ? 1 : 0;
    if (E > 0) {
        k_count_edges<<<nblocks(E), kThreads, 0, s>>>(edge_index, E, N, drop, cnt, cnt_t);
        LG_RET_IF_LAUNCH_FAILED();
    }
    k_scan_rows<<<1, 1024, 0, s>>>(cnt, N, drop, rowptr);
    k_scan_rows<<<1, 1024, 0, s>>>(cnt_t, N, drop, rowptr_t);
    LG_RET_IF_LAUNCH_FAILED();
    if (E > 0) {
        k_fill_edges<<<nblocks(E), kThreads, 0, s>>>(edge_index, E, N, drop, rowptr, rowptr_t, cur, cur_t, item,
                                                     item_t);
        LG_RET_IF_LAUNCH_FAILED();
    }
    for (int phase = 0; phase < 2; ++phase) {
        k_finalize<<<nblocks(N), kThreads, 0, s>>>(edge_index, E, N, drop, normalize ? 1 : 0, fill_value, cnt,
                                                   cnt_t, rowptr, rowptr_t, item, item_t, dis, col, w, col_t, w_t,
                                                   phase);
        LG_RET_IF_LAUNCH_FAILED();
    }
    return LG_OK;
}

extern "C" int64_t lg_incidence_workspace_bytes(int64_t P, int64_t N) {
    if (P < 0 || N < 0) return LG_EINVAL;
    return align256(4 * (2 * N) + 64);
}

extern "C" int lg_incidence_build(const int64_t* ends, int64_t P, int64_t N, int32_t* inc_rowptr,
                                  int32_t* inc_item, void* workspace, int64_t ws_bytes, lg_stream_t stream) {
    if (P < 0 || N <= 0 || 2 * P > INT32_MAX / 2 || N > INT32_MAX / 2) return LG_EINVAL;
    if ((P > 0 && (!ends || !inc_item)) || !inc_rowptr || !workspace) return LG_EINVAL;
    if (ws_bytes < lg_incidence_workspace_bytes(P, N)) return LG_EINVAL;
    hipStream_t s = lg_stream(stream);
    int32_t* cnt = static_cast<int32_t*>(workspace);
    int32_t* cur = cnt + N;
    if (hipMemsetAsync(cnt, 0, sizeof(int32_t) * 2 * N, s) != hipSuccess) return LG_EHIP;
    const int64_t P2 = 2 * P;
    if (P2 > 0) {
        k_count_inc<<<nblocks(P2), kThreads, 0, s>>>(ends, P2, N, cnt);
        LG_RET_IF_LAUNCH_FAILED();
    }
    k_scan_rows<<<1, 1024, 0, s>>>(cnt, N, 0, inc_rowptr);
    LG_RET_IF_LAUNCH_FAILED();
    if (P2 > 0) {
        k_fill_inc<<<nblocks(P2), kThreads, 0, s>>>(ends, P2, N, inc_rowptr, cur, inc_item);
        k_sort_inc<<<nblocks(N), kThreads, 0, s>>>(N, inc_rowptr, inc_item);
        LG_RET_IF_LAUNCH_FAILED();
    }
    return LG_OK;
}

extern "C" int lg_batchify_edge_index(const int64_t* edge_index, int64_t E, int64_t N, int64_t B, int64_t* out,
                                      lg_stream_t stream) {
    if (E < 0 || N < 0 || B < 0) return LG_EINVAL;
    if (E == 0 || B == 0) return LG_OK;
    if (!edge_index || !out) return LG_EINVAL;
    k_batchify<<<nblocks(B * E), kThreads, 0, lg_stream(stream)>>>(edge_index, E, N, B, out);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_nm_table_build(const int32_t* rowptr, const int32_t* pairs, int64_t N, const int32_t* order,
                                 int32_t* nodetab, lg_stream_t stream) {
    if (N <= 0 || N > INT32_MAX / 32 || !rowptr || !pairs || !nodetab) return LG_EINVAL;
    k_nm_table<<<nblocks(2 * N), kThreads, 0, lg_stream(stream)>>>(rowptr, reinterpret_cast<const int2*>(pairs), N,
                                                                   order, nodetab);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_nm_table_sensor_mark(const int32_t* nodetab, const int32_t* pairs, int64_t N, int64_t nnz,
                                       const int32_t* node_slot, int32_t* nodetab_out, int32_t* pairs_out,
                                       int32_t* pos_slot, lg_stream_t stream) {
    if (N <= 0 || N > INT32_MAX / 32 || nnz < 0 || nnz > INT32_MAX / 2 || !nodetab || !node_slot || !nodetab_out ||
        !pos_slot || (nnz > 0 && (!pairs || !pairs_out)))
        return LG_EINVAL;
    const int64_t n = std::max<int64_t>(2 * N, nnz);
    k_nm_mark<<<nblocks(n), kThreads, 0, lg_stream(stream)>>>(nodetab, reinterpret_cast<const int2*>(pairs), N, nnz,
                                                              node_slot, nodetab_out, reinterpret_cast<int2*>(pairs_out),
                                                              pos_slot);
    LG_RET_IF_LAUNCH_FAILED();
    return LG_OK;
}

extern "C" int lg_rcm_order(const int64_t* edge_index, int64_t E, int64_t N, int32_t* order) {
    if (N <= 0 || N > INT32_MAX / 2 || E < 0 || !order || (E > 0 && !edge_index)) return LG_EINVAL;
    // undirected adjacency without self loops / duplicates, CSR sorted by neighbour id
    std::vector<std::pair<int32_t, int32_t>> und;
    und.reserve(2 * static_cast<size_t>(E));
    for (int64_t e = 0; e < E; ++e) {
        const int64_t u = edge_index[e], v = edge_index[E + e];
        if (u < 0 || u >= N || v < 0 || v >= N) return LG_EINVAL;
        if (u == v) continue;
        und.emplace_back(static_cast<int32_t>(u), static_cast<int32_t>(v));
        und.emplace_back(static_cast<int32_t>(v), static_cast<int32_t>(u));
    }
    std::sort(und.begin(), und.end());
    und.erase(std::unique(und.begin(), und.end()), und.end());
    std::vector<int64_t> rp(N + 1, 0);
    for (const auto& uv : und) ++rp[uv.first + 1];
    for (int64_t n = 0; n < N; ++n) rp[n + 1] += rp[n];
    std::vector<int32_t> deg(N);
    for (int64_t n = 0; n < N; ++n) deg[n] = static_cast<int32_t>(rp[n + 1] - rp[n]);
    // component starts: nodes by (degree, id)
    std::vector<int32_t> by_deg(N);
    for (int64_t n = 0; n < N; ++n) by_deg[n] = static_cast<int32_t>(n);
    std::stable_sort(by_deg.begin(), by_deg.end(), [&](int32_t a, int32_t b) { return deg[a] < deg[b]; });
    std::vector<char> seen(N, 0);
    std::vector<int32_t> seq;
    seq.reserve(N);
    std::vector<int32_t> nb;
    for (int32_t s : by_deg) {
        if (seen[s]) continue;
        seen[s] = 1;
        size_t head = seq.size();
        seq.push_back(s);
        while (head < seq.size()) {
            const int32_t u = seq[head++];
            nb.clear();
            for (int64_t k = rp[u]; k < rp[u + 1]; ++k)
                if (!seen[und[k].second]) nb.push_back(und[k].second);
            std::stable_sort(nb.begin(), nb.end(), [&](int32_t a, int32_t b) { return deg[a] < deg[b]; });
            for (int32_t v : nb) {
                seen[v] = 1;
                seq.push_back(v);
            }
        }
    }
    for (int64_t i = 0; i < N; ++i) order[i] = seq[N - 1 - i];
    return LG_OK;
}
