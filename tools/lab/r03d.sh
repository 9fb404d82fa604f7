#!/bin/bash
# r03d: nm5 prefetch depth (NPF 3/4/5), bitwise check vs nm3
set -o pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/diag/nm3_opt_check.py --nm5 --opts "" > $OUT/check.txt 2>&1; tail -2 $OUT/check.txt
L="opt0+mask,nm5+mask,nm5,opt0,nm5+mask+bf16,opt0+mask+bf16"
for v in lab lab_n3 lab_n5 lab; do
  echo "== $v"
  LEAKGNN_LIB=leak-det-gnn_amd/lib/$v/libleakgnn.so timeout -k 10 300 python -u tools/kbench.py --which none --nmlab $L --iters 50 > $OUT/kb_$v.txt 2>&1 || { tail -30 $OUT/kb_$v.txt; exit 1; }
  grep gcn $OUT/kb_$v.txt
done
