#!/bin/bash
# r03ae: row-tile kernels with the lazy record decode, the first tile's gather over the W
# staging and the next tile's gather issued at the end of each forward tile (C5) + parity
set -o pipefail
OUT=gpurun_out/r03ae; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_library.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rows or c5" > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u tools/kbench.py --which c5_fwd,c5_bwd --iters 30 > $OUT/kb.txt 2>&1 || { tail -5 $OUT/kb.txt; exit 1; }
grep c5 $OUT/kb.txt
LEAKGNN_LIB=leak-det-gnn_amd/lib/v_stamps/libleakgnn.so timeout -k 10 200 python -u tools/kbench.py --which c5_fwd --stamps --iters 30 > $OUT/kb_stamps.txt 2>&1 || { tail -5 $OUT/kb_stamps.txt; exit 1; }
grep stamps $OUT/kb_stamps.txt
