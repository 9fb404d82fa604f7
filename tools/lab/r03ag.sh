#!/bin/bash
# r03ag: GRU backward counters, new row mapping vs previous layout
set -o pipefail
OUT=gpurun_out/r03ag; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/pmc_kernels.py --out $OUT --tag gru_new --targets gru_bwd:k_gru_bwd2 > $OUT/new.txt 2>&1 || { tail -5 $OUT/new.txt; exit 1; }
LEAKGNN_LIB=leak-det-gnn_amd/lib/v_gruold/libleakgnn.so timeout -k 10 300 python tools/pmc_kernels.py --out $OUT --tag gru_old --targets gru_bwd:k_gru_bwd2 > $OUT/old.txt 2>&1 || { tail -5 $OUT/old.txt; exit 1; }
grep -E "LDS|WAIT|VALU/wave|MFMA_busy" $OUT/new.txt $OUT/old.txt
