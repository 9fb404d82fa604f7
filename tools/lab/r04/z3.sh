#!/bin/bash
# r04z3: the final bench line (after the GRU f16x2 work) (all legs: PMC traffic, step kernel trace, cpu_baseline, C4, C5,
# bf16 tier) and rocprofv3 --kernel-trace --stats of the same step
set -o pipefail
OUT=gpurun_out/r04z3; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d[k] for k in ('value','ms_per_step','step_gap_us')}, d['roofline'], d['roofline_bwd'].get('frac'), d.get('cpu_baseline'), d['kernels_us'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-c4 --no-c5 --no-tier-leg > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof failed"; tail -20 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
