#!/bin/bash
# r02d: nm3 v2 (packed fma, one-add addressing) parity + graph-timed floors
set -o pipefail
OUT=gpurun_out/r02d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "node_major or high_degree or detector_vs_reference or c4_graph or replay" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 300 python tools/kbench.py --which copy,spmm --B 256 --iters 100 \
  --nmlab bpc1,bpc2,bpc3,bpc4,nm2+bpc3,nomfma+bpc3,noload+bpc3,nostore+bpc3,nomfma+noload+bpc3,nomfma+noload+nostore+bpc3,dst+bpc3,dst+bpc2,w8+bpc1,w8+bpc2,f32+bpc3 > $OUT/kblab.txt 2>&1 || { cat $OUT/kblab.txt; exit 1; }
grep -v amdgpu.ids $OUT/kblab.txt
