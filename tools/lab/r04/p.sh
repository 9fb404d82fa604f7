#!/bin/bash
# r04p: GRU backward f16x2 with each step's dW deferred behind the next step's elementwise part,
# buffer loads: GRU parity tests (product build), kernel A/B (lab build, LG_LAB_GRU_BF16X3=1 is
# the 3-way split), short bench
set -o pipefail
OUT=gpurun_out/r04p; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "gru" > $OUT/tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 120 python -u tools/kbench.py --which gru_fwd,gru_bwd --iters 50 > $OUT/kb.txt 2>&1 \
 && LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 120 python -u tools/kbench.py --which gru_bwd --iters 50 > $OUT/kb_lab_f16.txt 2>&1 \
 && LG_LAB_GRU_NODEFER=1 LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 120 python -u tools/kbench.py --which gru_bwd --iters 50 > $OUT/kb_lab_nodefer.txt 2>&1 \
 && timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "rc=$rc"; grep -h "PASSED\|FAILED\|Error:\|passed\|failed" $OUT/tests.log | cut -c1-200 | tail -20; cat $OUT/kb.txt $OUT/kb_lab_f16.txt $OUT/kb_lab_nodefer.txt 2>/dev/null | grep -v "^#\|amdgpu.ids" | cut -c1-300; python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us'])" 2>/dev/null; exit $rc
