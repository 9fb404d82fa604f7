#!/bin/bash
# r03y: C5 (100k nodes, B = 1) forward timeline (row-tile kernel, per-wave stamps) and floors
set -o pipefail
OUT=gpurun_out/r03y; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/kbench.py --which c5_fwd,c5_copy,c5_spmm --iters 30 > $OUT/kb.txt 2>&1 || { tail -5 $OUT/kb.txt; exit 1; }
grep c5 $OUT/kb.txt
LEAKGNN_LIB=leak-det-gnn_amd/lib/v_stamps/libleakgnn.so timeout -k 10 300 python -u tools/kbench.py --which c5_fwd --stamps --iters 30 > $OUT/kb_stamps.txt 2>&1 || { tail -5 $OUT/kb_stamps.txt; exit 1; }
cat $OUT/kb_stamps.txt
