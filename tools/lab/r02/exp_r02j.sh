#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -v --timeout 300 --timeout-method thread -m gpu -k b256 > $OUT/t.log 2>&1; echo "exit $?"; grep -E "PASSED|FAILED|^E  " $OUT/t.log | head
