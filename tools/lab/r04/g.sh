#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/diag/diag_edge16.py > $OUT/diag.txt 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids $OUT/diag.txt | tail -40
