#!/bin/bash
# r03ad: row-tile kernels (no waterfall) at C5: gather batch 2 / 3 (default) / 4 / 6, and the
# forward timeline (stamps)
set -o pipefail
OUT=gpurun_out/r03ad; mkdir -p $OUT
export TMPDIR=/tmp
for v in libleakgnn v_fnb2 v_fnb4 v_fnb6; do
  lib=leak-det-gnn_amd/lib/libleakgnn.so; [ $v = libleakgnn ] || lib=leak-det-gnn_amd/lib/$v/libleakgnn.so
  LEAKGNN_LIB=$lib timeout -k 10 200 python -u tools/kbench.py --which c5_fwd,c5_bwd --iters 30 > $OUT/kb_$v.txt 2>&1 || { tail -5 $OUT/kb_$v.txt; exit 1; }
  echo "== $v"; grep -E "c5_(fwd|bwd) " $OUT/kb_$v.txt
done
LEAKGNN_LIB=leak-det-gnn_amd/lib/v_stamps/libleakgnn.so timeout -k 10 200 python -u tools/kbench.py --which c5_fwd --stamps --iters 30 > $OUT/kb_stamps.txt 2>&1 || { tail -5 $OUT/kb_stamps.txt; exit 1; }
grep stamps $OUT/kb_stamps.txt
