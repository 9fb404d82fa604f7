#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_library.py tests/test_gpu_parity.py tests/test_gpu_configs.py -v --timeout 300 --timeout-method thread -k "opcheck or b64 or b256 or bf16 or fixture or c4_graph or replay or node_major_matches" > $OUT/tests.log 2>&1
grep -E "PASSED|FAILED|passed|failed" $OUT/tests.log | tail -14
grep -E "^E  " $OUT/tests.log | head -10
timeout -k 10 600 python bench.py --no-pmc --no-cpu-baseline --no-c4 --no-tier-leg > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us'])"
