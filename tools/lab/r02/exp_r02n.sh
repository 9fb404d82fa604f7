#!/bin/bash
# r02n: GRU forward fast-math A/B (12-wave and per-unit kernels) + parity of the fast-math build
set -o pipefail
OUT=gpurun_out/r02n; mkdir -p $OUT
L1=leak-det-gnn_amd/lib/lab/libleakgnn.so; L2=leak-det-gnn_amd/lib/lab2/libleakgnn.so
LEAKGNN_LIB=$L1 timeout -k 10 120 python tools/kbench.py --which gru_fwd > $OUT/kb_12w.txt 2>&1 || exit 1
LEAKGNN_LIB=$L2 timeout -k 10 120 python tools/kbench.py --which gru_fwd > $OUT/kb_12w_fast.txt 2>&1 || exit 1
LG_GRU_FWD_UNIT=1 LEAKGNN_LIB=$L2 timeout -k 10 120 python tools/kbench.py --which gru_fwd > $OUT/kb_unit_fast.txt 2>&1 || exit 1
for f in kb_12w kb_12w_fast kb_unit_fast; do echo $f; grep -v amdgpu $OUT/$f.txt; done
LEAKGNN_LIB=$L2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k gru > $OUT/t_fast.log 2>&1; echo "fast parity rc $?"
grep -E "PASSED|FAILED|^E  " $OUT/t_fast.log | head
