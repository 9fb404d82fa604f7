#!/bin/bash
# r02ak: dropout seed slots re-drawn by one device kernel (no torch RNG fills in the replay):
# full -m gpu suite, step kernel list, bench
set -o pipefail
OUT=gpurun_out/r02ak; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $OUT/gpu_tests.txt | head -20; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-c4 --no-tier-leg --steps 20 --warmup 5 > $OUT/bench_prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/prof
python3 tools/trace_step.py $OUT/kernel_trace.csv > $OUT/step_kernels.txt; rm -f $OUT/kernel_trace.csv
sed -n '/headline step/,/^sum/p' $OUT/step_kernels.txt
timeout -k 10 400 python bench.py --no-pmc --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us'])"
