#!/bin/bash
# r03o: full GPU suite (new: C4 B=64, C5 node-major vs fp64, captured CLI, overlapped DP step) + bench
set -o pipefail
OUT=gpurun_out/r03o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?; tail -5 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && tail -c 3000 $OUT/bench.json
