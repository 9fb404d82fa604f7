#!/bin/bash
# r03w: single-graph row-tile kernels (lg_gcn_fwd_rows / lg_gcn_bwd_rows): parity + C5 timing
set -o pipefail
OUT=gpurun_out/r03w; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_library.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread -k "rows or c5 or opcheck or timer" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt; grep -E "FAILED|Error" $OUT/tests.txt | head
timeout -k 10 300 python -u tools/kbench.py --which c5_fwd,c5_bwd --iters 30 > $OUT/kb.txt 2>&1; grep c5 $OUT/kb.txt
exit $rc
