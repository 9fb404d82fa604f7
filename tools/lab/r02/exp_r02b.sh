#!/bin/bash
# r02b: node-table forward (nm3) parity + timing sweep against the round-1 pipeline (nm2)
set -o pipefail
OUT=gpurun_out/r02b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "node_major or high_degree or detector_vs_reference or c4_graph or replay" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python tools/kbench.py --which gcn_fwd_nm,gcn_fwd_nm_train,spmm,copy,gcn_bwd_nm --B 256 --iters 100 > $OUT/kb.txt 2>&1 || { cat $OUT/kb.txt; exit 1; }
cat $OUT/kb.txt
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 300 python tools/kbench.py --which none --B 256 --iters 100 \
  --nmlab nm2,nm2+nomfma,nm2+noload,nomfma,noload,w8,f32,bpc2,bpc3,w8+bpc1,nm2+bpc3 > $OUT/kblab.txt 2>&1 || { cat $OUT/kblab.txt; exit 1; }
cat $OUT/kblab.txt
timeout -k 10 200 python tools/kbench.py --which gcn_fwd_nm_train,copy --B 1024 --iters 50 > $OUT/kb1024.txt 2>&1 && cat $OUT/kb1024.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/kbench.py --which gcn_fwd_nm_train,spmm,copy,gcn_bwd_nm --B 256 --iters 50 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | cut -c1-150
