#!/bin/bash
# r03af: GRU backward with the transposed reads' rows remapped (no 2-way bank conflicts) vs the
# previous layout (lib/v_gruold), + the GRU and row-tile / C5 parity tests
set -o pipefail
OUT=gpurun_out/r03af; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_library.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -m gpu -k "gru or rows or c5" > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc = 0 ] || exit 1
for v in libleakgnn v_gruold libleakgnn v_gruold; do
  lib=leak-det-gnn_amd/lib/libleakgnn.so; [ $v = libleakgnn ] || lib=leak-det-gnn_amd/lib/$v/libleakgnn.so
  LEAKGNN_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --which gru_bwd --iters 30 > $OUT/kb_$v.txt 2>&1 || { tail -5 $OUT/kb_$v.txt; exit 1; }
  echo "== $v"; grep -E "gru" $OUT/kb_$v.txt
done
timeout -k 10 300 python -u tools/kbench.py --which c5_fwd,c5_bwd --iters 30 > $OUT/kb_c5.txt 2>&1 || { tail -5 $OUT/kb_c5.txt; exit 1; }
grep c5 $OUT/kb_c5.txt
