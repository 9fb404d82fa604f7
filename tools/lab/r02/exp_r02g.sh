#!/bin/bash
# r02g: new backward kernel: parity (node-major tests) + timing vs the round-1 kernel; then full suite
set -o pipefail
OUT=gpurun_out/r02g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "node_major or high_degree or detector_vs_reference or c4_graph or replay or b64" > $OUT/tests_nm.log 2>&1 || { tail -40 $OUT/tests_nm.log; exit 1; }
tail -2 $OUT/tests_nm.log
timeout -k 10 200 python tools/kbench.py --which gcn_bwd_nm,gcn_bwd_nm_old,gcn_bwd_nm_l0,gcn_bwd_nm_l0_old,gcn_fwd_nm_train --B 256 --iters 100 > $OUT/kb.txt 2>&1 || { cat $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head -5; tail -40 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -2
