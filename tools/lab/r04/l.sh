#!/bin/bash
# r04l: layer 0 on the compressed node init with the sensor rows added by the consumers
set -o pipefail
OUT=gpurun_out/r04l; mkdir -p $OUT
export TMPDIR=/tmp
T="--timeout 120 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_x0.py -x -q $T -m gpu > $OUT/x0.log 2>&1; echo "x0 rc=$?"; grep -E "FAILED|passed|failed|^E " $OUT/x0.log | head -20
timeout -k 10 300 python -u tools/kbench.py --which node_init_bits,gcn_fwd_x0,gcn_fwd_nm_train --nmlab dflt --iters 50 > $OUT/kb.txt 2>&1 || { tail -20 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
timeout -k 10 900 python -u -m pytest tests -q $T -m gpu > $OUT/tests.log 2>&1; echo "suite rc=$?"; grep -E "FAILED|passed|failed" $OUT/tests.log | head -20
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --no-c5 --no-pmc --no-tier-leg > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
