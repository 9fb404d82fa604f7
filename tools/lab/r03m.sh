#!/bin/bash
# r03m: pc producer with the next tile's 4th neighbour in flight one tile ahead (X4) vs without
set -o pipefail
OUT=gpurun_out/r03m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/lab/diag/nm3_opt_check.py --nm5 --opts "" > $OUT/check.txt 2>&1; tail -3 $OUT/check.txt
L="mask,nm3+mask,x,mask"
for v in libleakgnn v_nox4 v_x4n2 v_x4n4 libleakgnn v_nox4; do
  lib=leak-det-gnn_amd/lib/libleakgnn.so; [ $v = libleakgnn ] || lib=leak-det-gnn_amd/lib/$v/libleakgnn.so
  echo "== $v"
  LEAKGNN_LIB=$lib timeout -k 10 200 python -u tools/kbench.py --which none --nmlab $L --iters 50 > $OUT/kb_$v.txt 2>&1 || { tail -5 $OUT/kb_$v.txt; exit 1; }
  grep gcn $OUT/kb_$v.txt | grep train
done
