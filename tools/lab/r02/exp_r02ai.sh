#!/bin/bash
# r02ai: round-2 closing validation: full -m gpu suite, smoke, default bench line (driver
# command), rocprofv3 kernel stats + per-step list, PMC summary of the hot kernels
set -o pipefail
OUT=gpurun_out/r02ai; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $OUT/gpu_tests.txt | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline_bwd']['frac'], d['roofline_bwd']['traffic'], d['stream_copy']['GBps']); print(d['mlp_tier']['value'], d['c4']['value'], d['e2e_training']['value'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-c4 --no-tier-leg --steps 20 --warmup 5 > $OUT/bench_prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 tools/trace_step.py $OUT/kernel_trace.csv > $OUT/step_kernels.txt; rm -f $OUT/kernel_trace.csv
timeout -k 10 600 python -u tools/pmc_kernels.py --out $OUT --tag r02ai > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
grep -E "==|HBM_bytes|L2_hit|duration" $OUT/pmc_r02ai.txt
