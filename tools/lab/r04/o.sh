#!/bin/bash
# r04o: counters of the f16x2 GRU training backward (k_gru_bwd2), then the 3-way split's (lab)
set -o pipefail
OUT=gpurun_out/r04o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/pmc_kernels.py --out $OUT --tag gru_f16 --targets gru_bwd:k_gru_bwd > $OUT/pmc.log 2>&1 \
 && LG_LAB_GRU_BF16X3=1 LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 400 python -u tools/pmc_kernels.py --out $OUT --tag gru_x3 --targets gru_bwd:k_gru_bwd > $OUT/pmc_x3.log 2>&1
rc=$?; echo "rc=$rc"; tail -20 $OUT/pmc_gru_f16.txt; exit $rc
