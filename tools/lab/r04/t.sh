#!/bin/bash
# r04t: GRU backward with the deferred dW moved ahead of the image writes: GRU
# parity tests, kernel time, short bench
set -o pipefail
OUT=gpurun_out/r04t; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "gru" > $OUT/tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 120 python -u tools/kbench.py --which gru_fwd,gru_bwd --iters 50 > $OUT/kb.txt 2>&1 \
 && timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "rc=$rc"; grep -h "FAILED\|Error:\|passed\|failed" $OUT/tests.log | cut -c1-200 | tail -6; grep -v "^#\|amdgpu.ids" $OUT/kb.txt | cut -c1-300; python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us'])" 2>/dev/null; exit $rc
