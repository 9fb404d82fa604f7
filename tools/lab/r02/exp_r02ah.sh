#!/bin/bash
# r02ah: last layer's output mask as bits (lg_gcn_fwd_nm_bits / lg_gcn_bwd_nm_bits): timings, tests, bench, trace
set -o pipefail
OUT=gpurun_out/r02ah; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python tools/kbench.py --which gcn_fwd_nm_train,gcn_bwd_nm,gcn_bwd_nm_y,gcn_bwd_nm_l0 --iters 40 > $OUT/kb.txt 2>&1 || { tail -20 $OUT/kb.txt; exit 1; }
grep -v amdgpu $OUT/kb.txt | tail -8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -3 $OUT/gpu_tests.txt; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $OUT/gpu_tests.txt | head -20; exit 1; }
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['roofline_bwd'], d['kernels_us']); print(d['mlp_tier']['value'], d['c4']['value'], d['e2e_training']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-c4 --no-tier-leg --steps 20 --warmup 5 > $OUT/bench_prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 tools/trace_step.py $OUT/kernel_trace.csv > $OUT/step_kernels.txt; rm -f $OUT/kernel_trace.csv
sed -n '/one step/,$p' $OUT/step_kernels.txt | head -24
