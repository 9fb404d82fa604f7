#!/bin/bash
# r03v: full GPU suite + backward variant check + timings (store guard in every tile-store kernel)
set -o pipefail
OUT=gpurun_out/r03v; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -3 $OUT/gpu_tests.txt; grep FAILED $OUT/gpu_tests.txt
timeout -k 10 200 python -u tools/lab/diag/bpc_check.py > $OUT/bpc_check.txt 2>&1; tail -1 $OUT/bpc_check.txt
timeout -k 10 200 python -u tools/kbench.py --which gcn_fwd_nm_train,gcn_bwd_nm,gcn_bwd_nm_nm3f16,gcn_bwd_nm_pc,gcn_bwd_nm_l0,gcn_bwd_nm_l0_nm3f16,gcn_bwd_nm_l0_pc --iters 50 > $OUT/kb.txt 2>&1; grep -E "bwd|fwd" $OUT/kb.txt
exit $rc
