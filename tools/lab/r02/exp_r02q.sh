#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02q; mkdir -p $OUT
timeout -k 10 300 python -u tools/diag_bf16.py > $OUT/diag.log 2>&1; echo "rc $?"; grep -v amdgpu $OUT/diag.log | tail -30
