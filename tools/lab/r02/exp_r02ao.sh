#!/bin/bash
# r02ao: node-major forward with 3 neighbour blocks in flight (was 4): node-major / detector
# GPU tests, then the bench twice (in-step kernel times)
set -o pipefail
OUT=gpurun_out/r02ao; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "node_major or detector or b256 or c5 or C5 or bf16 or c4 or captured" > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $OUT/gpu_tests.txt | head -20; exit 1; }
for i in 1 2; do
timeout -k 10 400 python bench.py --no-pmc --no-cpu-baseline > $OUT/bench$i.json 2> $OUT/bench$i.err || { tail -20 $OUT/bench$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['c4']['value'], d['mlp_tier']['value'], d['kernels_us']['gcn_fwd'])"
done
