#!/bin/bash
# r03a: forward OPT variants (bitwise check + isolated timing) and the per-wave timeline
set -o pipefail
OUT=gpurun_out/r03a; mkdir -p $OUT
export TMPDIR=/tmp
LAB=leak-det-gnn_amd/lib/lab/libleakgnn.so
STP=leak-det-gnn_amd/lib/lab_stamps/libleakgnn.so
LEAKGNN_LIB=$LAB timeout -k 10 300 python -u tools/lab/diag/nm3_opt_check.py > $OUT/check.txt 2>&1 || { tail -30 $OUT/check.txt; exit 1; }
tail -3 $OUT/check.txt
LEAKGNN_LIB=$LAB timeout -k 10 400 python -u tools/kbench.py --which copy --nmlab opt0+mask,opt1+mask,opt2+mask,opt4+mask,opt8+mask,opt3+mask,opt7+mask,opt15+mask,opt15+mask+bpc4,opt15+mask+bpc2,opt0+mask+bf16,opt15,opt0,opt0+mask --iters 50 > $OUT/kb.txt 2>&1 || { tail -30 $OUT/kb.txt; exit 1; }
cat $OUT/kb.txt
LEAKGNN_LIB=$STP timeout -k 10 300 python -u tools/kbench.py --which none --nmlab opt0+mask,opt15+mask,opt15+mask+bpc4 --stamps --iters 5 > $OUT/stamps.txt 2>&1 || { tail -30 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
