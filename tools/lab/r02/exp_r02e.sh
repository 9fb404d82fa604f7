#!/bin/bash
# r02e: nm3 tile queue: parity + graph-timed sweep (queue vs static schedule)
set -o pipefail
OUT=gpurun_out/r02e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "node_major or high_degree or detector_vs_reference or c4_graph or replay" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 300 python tools/kbench.py --which gcn_fwd_nm,gcn_fwd_nm_train,copy --B 256 --iters 100 \
  --nmlab bpc2,bpc3,bpc4,static+bpc3,nomfma+bpc3,nomfma+static+bpc3,w8+bpc1,w8+bpc2,nostore+bpc3 > $OUT/kblab.txt 2>&1 || { cat $OUT/kblab.txt; exit 1; }
grep -v amdgpu.ids $OUT/kblab.txt
timeout -k 10 200 python tools/kbench.py --which gcn_fwd_nm_train,copy --B 1024 --iters 50 > $OUT/kb1024.txt 2>&1 && grep -v amdgpu.ids $OUT/kb1024.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/kbench.py --which gcn_fwd_nm_train,spmm,copy --B 256 --iters 50 --eager > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 - <<'P'
import csv
for r in csv.DictReader(open('gpurun_out/r02e/kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
P
