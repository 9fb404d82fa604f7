#!/bin/bash
# r04r: per-step timeline of the GRU training backward (stamps lab build)
set -o pipefail
OUT=gpurun_out/r04r2; mkdir -p $OUT
LEAKGNN_LIB=leak-det-gnn_amd/lib/stamps/libleakgnn.so timeout -k 10 150 python -u tools/kbench.py --which gru_bwd --stamps --iters 10 > $OUT/kb_stamps.txt 2>&1
rc=$?; echo "rc=$rc"; grep -v "amdgpu.ids" $OUT/kb_stamps.txt | cut -c1-1500 | tail -8; exit $rc
