#!/bin/bash
# r02k: full GPU suite, bench, rocprofv3 kernel stats (after the kink-aware parity fix)
set -o pipefail
OUT=gpurun_out/r02k; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1
grep -E "FAILED|passed|failed" $OUT/tests.log | tail -12
grep -E "^E  " $OUT/tests.log | head -30
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-c4 --steps 20 --warmup 5 > $OUT/bench_prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 - <<'P'
import csv
for r in list(csv.DictReader(open('gpurun_out/r02k/kernel_stats.csv')))[:24]:
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
P
