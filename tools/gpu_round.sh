#!/bin/bash
# One GPU-box pass: parity tests, bench line, rocprofv3 kernel stats.  Each GPU step has
# its own time limit and the chain stops at the first failure.
#   bash tools/gpu_round.sh <tag> [tests|bench|prof|all]
set -o pipefail
TAG=${1:-run}; WHAT=${2:-all}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
if [[ $WHAT == all || $WHAT == tests ]]; then
  timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/tests.log"; exit 1; }
  tail -3 "$OUT/tests.log"
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
  timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --steps 20 --warmup 5 > "$OUT/bench_prof.json" 2> "$OUT/prof.err" || { echo "prof failed"; tail -20 "$OUT/prof.err"; exit 1; }
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
  head -25 "$OUT/kernel_stats.csv" | cut -c1-200
fi
