#!/bin/bash
# r04k: trunk backward on the f16x2 transform: the whole suite, timings, bench
set -o pipefail
OUT=gpurun_out/r04k; mkdir -p $OUT
export TMPDIR=/tmp
T="--timeout 120 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -q $T -m gpu > $OUT/tests.log 2>&1; echo "suite rc=$?"; grep -E "FAILED|passed|failed|^E " $OUT/tests.log | head -30
timeout -k 10 300 python -u tools/kbench.py --which gcn_bwd_nm_l0s,gcn_bwd_x0,gcn_bwd_nm --iters 50 > $OUT/kb.txt 2>&1 || { tail -20 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --no-c5 --no-pmc --no-tier-leg > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_bwd']['frac'], d['kernels_us'])"
