#!/bin/bash
# r03h: nm5 with the 2-way fp16 transform (f16x2): accuracy vs nm3, timing; C5 kernels
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/lab/diag/nm3_opt_check.py --nm5 --opts "" > $OUT/check.txt 2>&1; grep -v amdgpu.ids $OUT/check.txt | grep -E "f16x2|OK|MISM"
L="mask,nm5+f16+mask,nm5+mask,mask+bf16,mask,nm5+f16+mask,nm5+f16,x"
timeout -k 10 200 python -u tools/kbench.py --which copy,c5_fwd,c5_bwd --nmlab $L --iters 50 > $OUT/kb.txt 2>&1 || { tail -30 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
