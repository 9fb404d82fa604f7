#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02v; mkdir -p $OUT
timeout -k 10 300 python -u tools/diag_layers.py > $OUT/diag.log 2>&1; echo "rc $?"; grep -v amdgpu $OUT/diag.log; timeout -k 10 600 python bench.py --no-pmc --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1; python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us']); print(d['mlp_tier']['value'], d['c4']['value'], d['e2e_training']['value'])"
