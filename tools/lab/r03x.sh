#!/bin/bash
# r03x: row-tile kernels, gather batch size 2 / 3 / 6 at C5
set -o pipefail
OUT=gpurun_out/r03x; mkdir -p $OUT
export TMPDIR=/tmp
for v in libleakgnn v_nb6 v_nb2 libleakgnn; do
  lib=leak-det-gnn_amd/lib/libleakgnn.so; [ $v = libleakgnn ] || lib=leak-det-gnn_amd/lib/$v/libleakgnn.so
  echo "== $v"
  LEAKGNN_LIB=$lib timeout -k 10 300 python -u tools/kbench.py --which c5_fwd,c5_bwd --iters 30 > $OUT/kb_$v.txt 2>&1 || { tail -5 $OUT/kb_$v.txt; exit 1; }
  grep c5 $OUT/kb_$v.txt
done
