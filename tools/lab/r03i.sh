#!/bin/bash
# r03i: producer / consumer forward with two consumers per producer (pc), fp16x2 transform
set -o pipefail
OUT=gpurun_out/r03i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/lab/diag/nm3_opt_check.py --nm5 --opts "" > $OUT/check.txt 2>&1; grep -v amdgpu.ids $OUT/check.txt | grep -E "pc|f16x2|OK|MISM"
L="mask,pc+mask,pc+f16+mask,nm5+f16+mask,pc1+mask,pc+mask+bf16,mask,pc+f16+mask,pc+f16,pc"
timeout -k 10 200 python -u tools/kbench.py --which copy --nmlab $L --iters 50 > $OUT/kb.txt 2>&1 || { tail -30 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
