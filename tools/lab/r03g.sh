#!/bin/bash
# r03g: what the split transform costs: nm5 with 1 / 3 / 6 MFMA products, and 6 products without
# the residual VALU (lab builds; results wrong by design)
set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT
export TMPDIR=/tmp
for v in lab lab_p1 lab_p3 lab_nosplit lab lab_p1; do
  echo "== $v"
  LEAKGNN_LIB=leak-det-gnn_amd/lib/$v/libleakgnn.so timeout -k 10 200 python -u tools/kbench.py --which none --nmlab nm5+mask,nm5+mask+bf16 --iters 50 > $OUT/kb_$v.txt 2>&1 || { tail -30 $OUT/kb_$v.txt; exit 1; }
  grep gcn $OUT/kb_$v.txt
done
