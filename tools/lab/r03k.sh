#!/bin/bash
# r03k: producer/consumer geometry (4x2, 6x1, 4x1), producer prefetch depth, ring depth
set -o pipefail
OUT=gpurun_out/r03k; mkdir -p $OUT
export TMPDIR=/tmp
L="mask,pc6+f16+mask,nm3+mask,nm5+f16+mask,pc1+f16+mask,mask,pc6+f16+mask,x,pc6+f16,nm3"
for v in libleakgnn v_pn4 v_r6; do
  lib=leak-det-gnn_amd/lib/libleakgnn.so; [ $v = libleakgnn ] || lib=leak-det-gnn_amd/lib/$v/libleakgnn.so
  echo "== $v"
  LEAKGNN_LIB=$lib timeout -k 10 200 python -u tools/kbench.py --which none --nmlab $L --iters 50 > $OUT/kb_$v.txt 2>&1 || { tail -30 $OUT/kb_$v.txt; exit 1; }
  grep gcn $OUT/kb_$v.txt | grep train
done
