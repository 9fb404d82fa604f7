// Cycle breakdown of k_gcn_fwd (lab tool): builds gcn.hip with -DGCN_PROF, runs one
// train-mode forward on an L-TOWN-A-shaped synthetic graph (N = 661, degrees 2..5 incl.
// the self loop) and prints per-wave s_memtime cycle averages per phase.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGCN_PROF -I include tools/gcn_prof.cpp \
//     leak-det-gnn_amd/csrc/reduce.hip -o tools/gcn_prof.bin && tools/gcn_prof.bin 256
#include "../leak-det-gnn_amd/csrc/gcn.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? atoll(argv[1]) : 256, N = 661, D = 64;
    std::vector<int32_t> rp(N + 1), col;
    std::vector<float> w;
    for (int64_t n = 0; n < N; ++n) {
        rp[n] = int32_t(col.size());
        for (int64_t d : {-7, -1, 1, 7})
            if (n + d >= 0 && n + d < N && (n * 13 + d) % 5 != 0) {
                col.push_back(int32_t(n + d));
                w.push_back(0.25f);
            }
        col.push_back(int32_t(n));
        w.push_back(0.25f);
    }
    rp[N] = int32_t(col.size());
    const int64_t nnz = col.size();
    int32_t *drp, *dcol;
    float *dw, *x, *y, *W, *bias;
    hipMalloc(&drp, (N + 1) * 4);
    hipMalloc(&dcol, nnz * 4);
    hipMalloc(&dw, nnz * 4);
    hipMalloc(&x, B * N * D * 4);
    hipMalloc(&y, B * N * D * 4);
    hipMalloc(&W, D * D * 4);
    hipMalloc(&bias, D * 4);
    hipMemcpy(drp, rp.data(), (N + 1) * 4, hipMemcpyHostToDevice);
    hipMemcpy(dcol, col.data(), nnz * 4, hipMemcpyHostToDevice);
    hipMemcpy(dw, w.data(), nnz * 4, hipMemcpyHostToDevice);
    hipMemset(x, 0, B * N * D * 4);
    hipMemset(W, 0, D * D * 4);
    hipMemset(bias, 0, D * 4);
    const int flags = LG_F_BIAS | LG_F_RELU | LG_F_DROPOUT;
    for (int it = 0; it < 3; ++it) lg_gcn_fwd(drp, dcol, dw, x, W, bias, y, B, N, D, nnz, flags, 0.1f, 1, 2, nullptr);
#ifdef GCN_PROF
    std::vector<unsigned long long> zero(65536 * 8, 0);
    hipMemcpyToSymbol(HIP_SYMBOL(g_gcn_prof), zero.data(), zero.size() * 8);
#endif
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    const int rc = lg_gcn_fwd(drp, dcol, dw, x, W, bias, y, B, N, D, nnz, flags, 0.1f, 1, 2, nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
#ifndef GCN_PROF
    for (int it = 0; it < 20; ++it) lg_gcn_fwd(drp, dcol, dw, x, W, bias, y, B, N, D, nnz, flags, 0.1f, 1, 2, nullptr);
    hipEventRecord(e0);
    for (int it = 0; it < 50; ++it) lg_gcn_fwd(drp, dcol, dw, x, W, bias, y, B, N, D, nnz, flags, 0.1f, 1, 2, nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("rc %d  %.2f us per launch (50 launches, no instrumentation)\n", rc, ms * 1e3 / 50);
    return 0;
#else
    std::vector<unsigned long long> prof(65536 * 8);
    hipMemcpyFromSymbol(prof.data(), HIP_SYMBOL(g_gcn_prof), prof.size() * 8);
    double sum[8] = {0};
    int waves = 0;
    for (int i = 0; i < 65536; ++i) {
        if (prof[8 * i + 6] == 0) continue;
        ++waves;
        for (int k = 0; k < 8; ++k) sum[k] += prof[8 * i + k];
    }
    const double tiles = sum[6], rounds = sum[7];
    printf("rc %d  %.1f us  waves %d  tiles %.0f  rounds %.0f (%.2f per tile)\n", rc, ms * 1e3, waves, tiles, rounds,
           rounds / tiles);
    printf("per round: csr+issue %.0f  hook(MFMA) %.0f  wait+fma %.0f | per tile: tail MFMA %.0f  epilogue+stores %.0f"
           " cycles\n",
           sum[1] / rounds, sum[2] / rounds, sum[3] / rounds, sum[4] / tiles, sum[5] / tiles);
    return 0;
#endif
}
