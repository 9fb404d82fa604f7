#!/bin/bash
# r03l: producer/consumer ring depth (4 / 6 / 8) and producer prefetch depth (2 / 3)
set -o pipefail
OUT=gpurun_out/r03l; mkdir -p $OUT
export TMPDIR=/tmp
L="mask,nm3+mask,x,mask"
for v in libleakgnn v_r6 v_r8 v_pn2 libleakgnn; do
  lib=leak-det-gnn_amd/lib/libleakgnn.so; [ $v = libleakgnn ] || lib=leak-det-gnn_amd/lib/$v/libleakgnn.so
  echo "== $v"
  LEAKGNN_LIB=$lib timeout -k 10 200 python -u tools/kbench.py --which none --nmlab $L --iters 50 > $OUT/kb_$v.txt 2>&1 || { tail -5 $OUT/kb_$v.txt; continue; }
  grep gcn $OUT/kb_$v.txt | grep train
done
