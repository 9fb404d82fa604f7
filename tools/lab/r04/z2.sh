#!/bin/bash
# r04z2: counter summaries (rocprofv3 --pmc passes, one group per pass) of the hot kernels,
# then the pc kernel's per-wave timeline (stamps lab build)
set -o pipefail
OUT=gpurun_out/r04z2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/pmc_kernels.py --out $OUT --tag r04 --targets gcn_fwd_nm_train:k_gcn_fwd_pc,gcn_bwd_nm:k_gcn_bwd_nm3,gcn_fwd_x0:k_gcn_fwd_pc,node_init_bits:k_node_init_bits,edge_fwd:k_edge_fwd,edge_bwd_stream:k_edge_bwd,gru_bwd:k_gru_bwd > $OUT/pmc.log 2>&1 \
 && LEAKGNN_LIB=leak-det-gnn_amd/lib/stamps/libleakgnn.so timeout -k 10 120 python -u tools/kbench.py --which none --nmlab dflt --stamps --iters 10 > $OUT/stamps.txt 2>&1
rc=$?; echo "rc=$rc"; tail -5 $OUT/pmc.log; cut -c1-3000 $OUT/stamps.txt 2>/dev/null | tail -5; exit $rc
