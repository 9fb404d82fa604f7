#!/bin/bash
# r04h: the whole GPU suite on the committed state
set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q --timeout 120 --timeout-method thread -m gpu > $OUT/tests.log 2>&1; echo "suite rc=$?"; grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -20; true
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 300 python -u tools/kbench.py --which edge_bwd --edgebwdlab 1,2,3,4,7 --iters 50 > $OUT/kb_lab.txt 2>&1 || { tail -20 $OUT/kb_lab.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb_lab.txt
