#!/bin/bash
# r03p: producer/consumer backward (k_gcn_bwd_pc) + f16x2 nm3 backward: parity + timing
set -o pipefail
OUT=gpurun_out/r03p; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_library.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $OUT/tests.txt | tail -15
W=gcn_bwd_nm,gcn_bwd_nm_nm3f16,gcn_bwd_nm_bf3,gcn_bwd_nm_l0,gcn_bwd_nm_l0_nm3f16,gcn_bwd_nm_l0_bf3
for i in 1 2; do
timeout -k 10 200 python -u tools/kbench.py --which $W --iters 50 > $OUT/kb$i.txt 2>&1 || { tail -5 $OUT/kb$i.txt; exit 1; }
grep bwd $OUT/kb$i.txt
done
exit $rc
