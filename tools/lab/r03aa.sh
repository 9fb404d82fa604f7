#!/bin/bash
# r03aa: pc forward with the first tile's blocks touched before the W staging barrier (product
# lib) against the previous pc forward (lib/v_old), isolated train-mode launches, alternating
set -o pipefail
OUT=gpurun_out/r03aa; mkdir -p $OUT
export TMPDIR=/tmp
for v in libleakgnn v_old libleakgnn v_old; do
  lib=leak-det-gnn_amd/lib/libleakgnn.so; [ $v = libleakgnn ] || lib=leak-det-gnn_amd/lib/$v/libleakgnn.so
  LEAKGNN_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --which gcn_fwd_nm_train --nmlab mask --iters 50 > $OUT/kb_$v.txt 2>&1 || { tail -5 $OUT/kb_$v.txt; exit 1; }
  echo "== $v"; grep -E "gcn_fwd" $OUT/kb_$v.txt
done
