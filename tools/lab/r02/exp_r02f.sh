#!/bin/bash
# r02f: full GPU suite with the new config tests, then a quick graph-timed fwd check
set -o pipefail
OUT=gpurun_out/r02f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { grep -E "PASS|FAIL|ERROR" $OUT/tests.log | tail -5; tail -40 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -2
grep -E "test_gpu_configs|test_gpu_harness" $OUT/tests.log | grep -E "PASSED|FAILED" | sed 's/.*:://' | head -30
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 300 python tools/kbench.py --which gcn_fwd_nm,gcn_fwd_nm_train,copy --B 256 --iters 100 --nmlab bpc3,nm2+bpc3,nomfma+bpc3 > $OUT/kblab.txt 2>&1 || { cat $OUT/kblab.txt; exit 1; }
grep -v amdgpu.ids $OUT/kblab.txt
