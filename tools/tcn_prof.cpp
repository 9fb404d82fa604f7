// Cycle breakdown of k_tcn_conv (lab tool): builds the kernel with -DTCN_PROF, runs one
// conv layer on synthetic rows and prints, per workgroup averages, the s_memtime cycles
// spent in K loops, between K loops (LayerNorm partials, barrier, DMA issue) and in the
// prologue.  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DTCN_PROF -I include \
//   tools/tcn_prof.cpp leak-det-gnn_amd/csrc/reduce.hip -o /tmp/tcn_prof && /tmp/tcn_prof 256 252
#include "../leak-det-gnn_amd/csrc/tcn.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    const int64_t nseg = argc > 1 ? atoll(argv[1]) : 256, rows_out = argc > 2 ? atoll(argv[2]) : 252;
    const int64_t rows_in = rows_out, rows_blk = rows_out, C = 128;
    std::vector<int32_t> plan(rows_out * 4);
    for (int64_t r = 0; r < rows_out; ++r) {
        plan[4 * r] = int32_t(r);
        plan[4 * r + 1] = int32_t(r >= 4 ? r - 4 : -1);
        plan[4 * r + 2] = int32_t(r >= 8 ? r - 8 : -1);
        plan[4 * r + 3] = int32_t(r);
    }
    float *in, *blk, *out, *wpk, *w, *par;
    int32_t* dplan;
    hipMalloc(&in, nseg * rows_in * C * 4);
    hipMalloc(&blk, nseg * rows_blk * C * 4);
    hipMalloc(&out, nseg * rows_out * C * 4);
    hipMalloc(&wpk, C * 3 * C * 4);
    hipMalloc(&w, C * 3 * C * 4);
    hipMalloc(&par, 3 * C * 4);
    hipMalloc(&dplan, plan.size() * 4);
    hipMemset(in, 0, nseg * rows_in * C * 4);
    hipMemset(blk, 0, nseg * rows_blk * C * 4);
    hipMemset(w, 0, C * 3 * C * 4);
    hipMemset(par, 0, 3 * C * 4);
    hipMemcpy(dplan, plan.data(), plan.size() * 4, hipMemcpyHostToDevice);
    lg_tcn_pack_weight(w, wpk, C, nullptr);
    for (int it = 0; it < 3; ++it)
        lg_tcn_conv_fwd(in, blk, dplan, wpk, par, par + C, par + 2 * C, 1e-5f, out, nseg, rows_in, rows_blk, rows_out,
                        C, nullptr);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    int rc = lg_tcn_conv_fwd(in, blk, dplan, wpk, par, par + C, par + 2 * C, 1e-5f, out, nseg, rows_in, rows_blk,
                             rows_out, C, nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> prof(4096 * 8);
    hipMemcpyFromSymbol(prof.data(), HIP_SYMBOL(g_tcn_prof), prof.size() * 8);
    const int grid = std::min<int64_t>((nseg * rows_out + 15) / 16, 256);
    double k = 0, b = 0, p = 0, n = 0, pa = 0, wa = 0;
    for (int i = 0; i < grid; ++i) {
        k += prof[8 * i];
        b += prof[8 * i + 1];
        p += prof[8 * i + 2];
        n += prof[8 * i + 3];
        pa += prof[8 * i + 4];
        wa += prof[8 * i + 5];
    }
    printf("rc %d  %.1f us  grid %d  tiles/wg %.2f\n", rc, ms * 1e3, grid, n / grid);
    printf("per tile: K loop %.0f  between %.0f (partials %.0f, wait+barrier %.0f, dma %.0f) cycles; prologue %.0f per wg\n",
           k / n, b / n, pa / n, wa / n, (b - pa - wa) / n, p / grid);
    return 0;
}
