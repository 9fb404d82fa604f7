#!/bin/bash
# r04i: where the streamed EdgeHead backward's time goes (lab build: MFMAs / scatter skipped)
set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
export TMPDIR=/tmp
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 300 python -u tools/kbench.py --which edge_bwd --edgebwdlab 1,2,3,4,7 --iters 50 > $OUT/kb.txt 2>&1 || { tail -20 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
