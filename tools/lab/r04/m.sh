#!/bin/bash
# r04m: the fused scatter only with a window per CU (C4 regression), the node-init bits
# kernel with four tiles per thread: suite, kbench, bench with C4
set -o pipefail
OUT=gpurun_out/r04m; mkdir -p $OUT
export TMPDIR=/tmp
T="--timeout 120 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -q $T -m gpu > $OUT/tests.log 2>&1; echo "suite rc=$?"; grep -E "FAILED|passed|failed" $OUT/tests.log | head -20
timeout -k 10 300 python -u tools/kbench.py --which node_init_bits,edge_bwd --iters 50 > $OUT/kb.txt 2>&1 || { tail -20 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
timeout -k 10 400 python bench.py --no-cpu-baseline --no-c5 --no-pmc --no-tier-leg > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['c4']['value'], d['c4']['ms_per_step'], d['kernels_us'])"
