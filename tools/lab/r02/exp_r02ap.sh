#!/bin/bash
# r02ap: prefetch depth of the node-major backward (3 / 4 current / 5), graph-timed
# isolated launches of the layer-2 (mask bits) and layer-1 backward, three interleaved reps
set -o pipefail
OUT=gpurun_out/r02ap; mkdir -p $OUT
for rep in 1 2 3; do
for v in b3 b4 b5; do
  export LEAKGNN_LIB=$PWD/leak-det-gnn_amd/lib/ab/$v.so
  timeout -k 10 180 python tools/kbench.py --which gcn_bwd_nm,gcn_bwd_nm_l0 --iters 40 > $OUT/kb_${v}_$rep.txt 2>&1 || { tail -5 $OUT/kb_${v}_$rep.txt; exit 1; }
  echo "== $v rep $rep"; grep -v amdgpu $OUT/kb_${v}_$rep.txt | grep gcn_bwd
done
done
