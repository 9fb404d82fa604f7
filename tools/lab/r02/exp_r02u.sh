#!/bin/bash
# r02u: rocprofv3 kernel trace of the bench step (for the per-step kernel list)
set -o pipefail
OUT=gpurun_out/r02u; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-c4 --no-tier-leg --steps 20 --warmup 5 > $OUT/bench_prof.json 2> /tmp/prof.err || { tail -20 /tmp/prof.err; exit 1; }
find $OUT/prof -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 tools/trace_step.py $OUT/kernel_trace.csv > $OUT/step_kernels.txt; rm -f $OUT/kernel_trace.csv; timeout -k 10 300 python -u -m pytest tests/test_gpu_library.py tests/test_graph_step.py -q --timeout 120 --timeout-method thread -k "adamw" 2>&1 | tail -2
cat $OUT/step_kernels.txt
