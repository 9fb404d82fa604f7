#!/bin/bash
# r02p: bf16 node-MLP tier (configs[2]): parity bar, library op schemas, bench with the tier leg
set -o pipefail
OUT=gpurun_out/r02p; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_library.py tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -k "bf16" > $OUT/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|^E  |bf16 tier|rel 2-norm" $OUT/tests.log | head -60
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --no-pmc --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us']); print(d['mlp_tier'])"
