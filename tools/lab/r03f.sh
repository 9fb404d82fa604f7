#!/bin/bash
# r03f: is the 3.3x neighbour re-read the limit?  nm3 / nm5 / pc on lab graphs
set -o pipefail
OUT=gpurun_out/r03f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/lab/diag/nm3_opt_check.py --nm5 --opts "" > $OUT/check.txt 2>&1; tail -1 $OUT/check.txt
for g in selfonly ring ltown; do
  echo "== $g"
  timeout -k 10 200 python -u tools/kbench.py --graph $g --which copy,spmm --nmlab mask,nm5+mask,pc+mask,mask+bf16,mask+nomfma --iters 50 > $OUT/kb_$g.txt 2>&1 || { tail -30 $OUT/kb_$g.txt; exit 1; }
  grep -v amdgpu.ids $OUT/kb_$g.txt
done
