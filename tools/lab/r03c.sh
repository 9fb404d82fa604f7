#!/bin/bash
# r03c: nm3 W-first staging, nm5 with LDS-staged W, -fno-slp-vectorize builds
set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT
export TMPDIR=/tmp
LAB=leak-det-gnn_amd/lib/lab/libleakgnn.so
NOS=leak-det-gnn_amd/lib/lab_noslp/libleakgnn.so
STP=leak-det-gnn_amd/lib/lab_stamps/libleakgnn.so
timeout -k 10 300 python -u tools/lab/diag/nm3_opt_check.py --nm5 --opts "" > $OUT/check.txt 2>&1; tail -4 $OUT/check.txt
LEAKGNN_LIB=$LAB timeout -k 10 300 python -u tools/lab/diag/nm3_opt_check.py --opts 16,20,28,30,31 > $OUT/check_lab.txt 2>&1; tail -4 $OUT/check_lab.txt
L="opt0+mask,opt16+mask,opt20+mask,opt28+mask,opt30+mask,opt31+mask,nm5+mask,opt4+mask,opt20,nm5,opt0+mask"
LEAKGNN_LIB=$LAB timeout -k 10 400 python -u tools/kbench.py --which none --nmlab $L --iters 50 > $OUT/kb.txt 2>&1 || { tail -30 $OUT/kb.txt; exit 1; }
cat $OUT/kb.txt
LEAKGNN_LIB=$NOS timeout -k 10 400 python -u tools/kbench.py --which none --nmlab $L --iters 50 > $OUT/kb_noslp.txt 2>&1 || { tail -30 $OUT/kb_noslp.txt; exit 1; }
cat $OUT/kb_noslp.txt
LEAKGNN_LIB=$STP timeout -k 10 300 python -u tools/kbench.py --which none --nmlab opt20+mask,nm5+mask --stamps --iters 5 > $OUT/stamps.txt 2>&1 || { tail -30 $OUT/stamps.txt; exit 1; }
grep stamps $OUT/stamps.txt
