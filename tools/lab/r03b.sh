#!/bin/bash
# r03b: W-in-registers forward (nm5): bitwise vs nm3, isolated timing, timeline
set -o pipefail
OUT=gpurun_out/r03b; mkdir -p $OUT
export TMPDIR=/tmp
LAB=leak-det-gnn_amd/lib/lab/libleakgnn.so
STP=leak-det-gnn_amd/lib/lab_stamps/libleakgnn.so
timeout -k 10 300 python -u tools/lab/diag/nm3_opt_check.py --nm5 --opts "" > $OUT/check.txt 2>&1 || { tail -30 $OUT/check.txt; exit 1; }
cat $OUT/check.txt
LEAKGNN_LIB=$LAB timeout -k 10 400 python -u tools/kbench.py --which copy --nmlab opt0+mask,nm5+mask,opt7+mask,nm5,opt0,nm5+mask+bpc1,opt0+mask+bf16,nm5+mask+bf16,nm5+mask+bf16+bpc3,nm5+mask,opt0+mask --iters 50 > $OUT/kb.txt 2>&1 || { tail -30 $OUT/kb.txt; exit 1; }
cat $OUT/kb.txt
LEAKGNN_LIB=$STP timeout -k 10 300 python -u tools/kbench.py --which none --nmlab nm5+mask,opt0+mask+bpc3 --stamps --iters 5 > $OUT/stamps.txt 2>&1 || { tail -30 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
