#!/bin/bash
# r03j: default forward = producer/consumer + fp16x2: full -m gpu suite, smoke, bench, rocprofv3 stats
set -o pipefail
OUT=gpurun_out/r03j; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -3 $OUT/gpu_tests.txt; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $OUT/gpu_tests.txt | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['roofline']['traffic'], d['roofline_bwd']['frac'], d['stream_copy']['GBps']); print(d['kernels_us']); print(d.get('c5'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-c4 --no-tier-leg --steps 20 --warmup 5 > $OUT/bench_prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/prof -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/prof
python3 tools/trace_step.py $OUT/kernel_trace.csv > $OUT/step_kernels.txt; rm -f $OUT/kernel_trace.csv
head -12 $OUT/kernel_stats.csv | cut -c1-150
