#!/bin/bash
# r02m: GRU forward per-unit-group kernel (parity + A/B vs the 12-wave kernel), kernel-timer
# test, bench with hipExtLaunchKernelGGL kernel timing, PMC counter summaries
set -o pipefail
OUT=gpurun_out/r02m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_library.py -v --timeout 120 --timeout-method thread -k timer > $OUT/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|^E  " $OUT/tests.log | tail -25
[ $rc -eq 0 ] || exit 1
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 120 python tools/kbench.py --which gru_fwd,gru_bwd > $OUT/kb_new.txt 2>&1 || exit 1
LG_GRU_FWD_UNIT=1 LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 120 python tools/kbench.py --which gru_fwd > $OUT/kb_old.txt 2>&1 || exit 1
echo 12w; cat $OUT/kb_new.txt; echo unit; cat $OUT/kb_old.txt
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 900 python -u tools/pmc_kernels.py --out $OUT --tag r02m > $OUT/pmc.log 2>&1; echo "pmc rc $?"
tail -150 $OUT/pmc.log
LG_GRU_FWD_UNIT=1 LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 300 python -u tools/pmc_kernels.py --out $OUT --tag r02m_gru_unit --targets gru_fwd:k_gru_fwd_u > $OUT/pmc_unit.log 2>&1; echo "pmc unit rc $?"
tail -40 $OUT/pmc_unit.log
