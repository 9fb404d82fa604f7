#!/bin/bash
# r03e: producer/consumer forward (pc): bitwise vs nm3, timing vs nm3 / nm5
set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/lab/diag/nm3_opt_check.py --nm5 --opts "" > $OUT/check.txt 2>&1; rc=$?; cat $OUT/check.txt | grep -v amdgpu.ids; [ $rc -le 1 ] || exit 1
L="mask,pc+mask,nm5+mask,mask,pc+mask,nm5+mask,x,pc,nm5,pc+mask+bf16,mask+bf16"
timeout -k 10 200 python -u tools/kbench.py --which copy --nmlab $L --iters 50 > $OUT/kb.txt 2>&1 || { tail -30 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
