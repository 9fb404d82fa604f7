#!/bin/bash
# r02t: fused clip+AdamW (ClipAdamW): parity vs torch, captured step, bench
set -o pipefail
OUT=gpurun_out/r02t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_library.py tests/test_graph_step.py -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $OUT/tests.log | tail -16
grep -E "^E  " $OUT/tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --no-pmc --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us']); print(d['mlp_tier']['value'], d['c4']['value'], d['e2e_training']['value'])"
