#!/bin/bash
# r02i: ReLU-kink diagnostic of the B=256 gradient errors, then the three r02h failures
set -o pipefail
OUT=gpurun_out/r02i; mkdir -p $OUT
export TMPDIR=/tmp
#timeout -k 10 400 python -u tools/diag_kink.py > $OUT/diag.log 2>&1; echo "diag exit $?"
#cat $OUT/diag.log | tail -60
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_library.py -v --timeout 300 --timeout-method thread -m gpu -k "b256 or compile" > $OUT/tests.log 2>&1
grep -E "FAILED|PASSED|passed|failed" $OUT/tests.log | tail -12
grep -E "^E  " $OUT/tests.log | head -30
