#!/bin/bash
# r02an: prefetch depth of the node-major forward (neighbour blocks in flight per tile):
# NPF 2 / 3 / 4 (current) / 5 (r02an first pass), graph-timed isolated launches, twice each
set -o pipefail
OUT=gpurun_out/${TAG:-r02an}; mkdir -p $OUT
for rep in 1 2 3; do
for v in npf3 npf4 npf2; do
  export LEAKGNN_LIB=$PWD/leak-det-gnn_amd/lib/ab/$v.so
  timeout -k 10 180 python tools/kbench.py --which gcn_fwd_nm_train,gcn_fwd_nm --iters 40 > $OUT/kb_${v}_$rep.txt 2>&1 || { tail -5 $OUT/kb_${v}_$rep.txt; exit 1; }
  echo "== $v rep $rep"; grep -v amdgpu $OUT/kb_${v}_$rep.txt | grep gcn_fwd
done
done
