#!/bin/bash
# r02al: GRU forward stores h and the gates non-temporally: GRU tests, bench in-step kernels
set -o pipefail
OUT=gpurun_out/r02al; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gru or detector or b256" > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $OUT/gpu_tests.txt | head -20; exit 1; }
for i in 1 2; do
timeout -k 10 400 python bench.py --no-pmc --no-cpu-baseline --no-c4 --no-tier-leg > $OUT/bench$i.json 2> $OUT/bench$i.err || { tail -20 $OUT/bench$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench$i.json')); print(d['value'], d['ms_per_step'], d['kernels_us'], d['e2e_training']['value'])"
done
