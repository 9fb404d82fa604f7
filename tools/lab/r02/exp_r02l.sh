#!/bin/bash
# r02l: kernel-timer test, bench with hipExtLaunchKernelGGL kernel timing, PMC counter summaries
set -o pipefail
OUT=gpurun_out/r02l; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_library.py tests/test_host.py -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|^E  " $OUT/tests.log | tail -15
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 900 python -u tools/pmc_kernels.py --out $OUT --tag r02l > $OUT/pmc.log 2>&1; echo "pmc rc $?"
tail -120 $OUT/pmc.log
