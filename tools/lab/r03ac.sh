#!/bin/bash
# r03ac: row-tile kernels without the per-lane descriptor / soffset waterfall (C5) + their parity test
set -o pipefail
OUT=gpurun_out/r03ac; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_library.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rows or c5" > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u tools/kbench.py --which c5_fwd,c5_bwd --iters 30 > $OUT/kb.txt 2>&1 || { tail -5 $OUT/kb.txt; exit 1; }
grep c5 $OUT/kb.txt
