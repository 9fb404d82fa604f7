#!/bin/bash
# r04n2: is the +-1-weight GRU gradient mismatch the f16x2 split or the conditioning?  the same
# test on the lab build's 3-way split and f16x2, then the kernel A/B and a short bench
set -o pipefail
OUT=gpurun_out/r04n2; mkdir -p $OUT
T="tests/test_gpu_parity.py::test_gru_bwd_f16x2_scales"
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so LG_LAB_GRU_BF16X3=1 timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu "$T" > $OUT/tests_x3.log 2>&1
echo "x3 rc=$?"
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu "$T" > $OUT/tests_f16.log 2>&1
echo "f16 rc=$?"
timeout -k 10 120 python -u tools/kbench.py --which gru_fwd,gru_bwd --iters 50 > $OUT/kb.txt 2>&1 \
 && LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 120 python -u tools/kbench.py --which gru_bwd --iters 50 > $OUT/kb_lab_f16.txt 2>&1 \
 && LG_LAB_GRU_BF16X3=1 LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 120 python -u tools/kbench.py --which gru_bwd --iters 50 > $OUT/kb_lab_x3.txt 2>&1 \
 && timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "rc=$rc"; grep -h "PASSED\|FAILED\|Error:" $OUT/tests_x3.log $OUT/tests_f16.log | cut -c1-200; cat $OUT/kb.txt $OUT/kb_lab_f16.txt $OUT/kb_lab_x3.txt 2>/dev/null | grep -v "^#" | cut -c1-300; python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us'])" 2>/dev/null; exit $rc
