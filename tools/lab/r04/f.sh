#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/diag/diag_x0.py > $OUT/diag.txt 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids $OUT/diag.txt | tail -40
timeout -k 10 300 python -u -m pytest tests/test_gpu_x0.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/x0.log 2>&1; echo "x0 rc=$?"; tail -30 $OUT/x0.log
