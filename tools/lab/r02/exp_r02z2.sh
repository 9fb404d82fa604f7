#!/bin/bash
# r02z2: rocprofv3 kernel trace/stats of the bench command, per-step kernel list, PMC summary
# of the hot kernels, and the CLI harness tests (detector CLI on the fused loss / ClipAdamW)
set -o pipefail
OUT=gpurun_out/r02z2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_harness.py -q --timeout 240 --timeout-method thread > $OUT/harness.txt 2>&1; rc=$?; tail -2 $OUT/harness.txt; [ $rc = 0 ] || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $OUT/bench_prof.json 2> /tmp/prof.err || { tail -20 /tmp/prof.err; exit 1; }
find $OUT/prof -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
python3 tools/trace_step.py $OUT/kernel_trace.csv > $OUT/step_kernels.txt; rm -f $OUT/kernel_trace.csv
head -40 $OUT/step_kernels.txt
timeout -k 10 600 python -u tools/pmc_kernels.py --out $OUT --tag r02z > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
grep -E "==|WAIT_INST_ANY/|MFMA_busy|duration|HBM_bytes|L2_hit" $OUT/pmc_r02z.txt
