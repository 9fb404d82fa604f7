#!/bin/bash
# r02r: sensor projection folded into node init (+ one fused backward kernel): full GPU suite, bench
set -o pipefail
OUT=gpurun_out/r02r; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1
grep -E "FAILED|passed|failed" $OUT/tests.log | tail -12
grep -E "^E  " $OUT/tests.log | head -20
timeout -k 10 600 python bench.py --no-pmc --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us']); print(d['mlp_tier']['value'], d['mlp_tier']['kernels_us'])"
