#!/bin/bash
# r04e: compressed node init (x0), the f16x2 EdgeHead forward, the streamed EdgeHead node
# scatter (pipe schedule, ABI 22); timings; the bench; deferred-reduction tests; the suite
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT
export TMPDIR=/tmp
T="--timeout 120 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_x0.py -x -q $T -m gpu > $OUT/x0.log 2>&1 || { echo "x0 tests failed"; tail -40 $OUT/x0.log; exit 1; }
tail -1 $OUT/x0.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_library.py -x -q $T -m gpu -k "edge or heads or incidence or scatter" > $OUT/edge.log 2>&1 || { echo "edge tests failed"; tail -60 $OUT/edge.log; exit 1; }
tail -1 $OUT/edge.log
timeout -k 10 300 python -u tools/kbench.py --which edge_fwd,edge_bwd,node_init,node_init_bits,gcn_fwd_x0,gcn_bwd_x0,gcn_fwd_nm_train,gcn_bwd_nm_l0s,copy --nmlab dflt --iters 50 > $OUT/kb.txt 2>&1 || { tail -20 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --no-c5 --no-pmc --no-tier-leg > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'], d.get('step_gap_us'))"
timeout -k 10 800 python -u -m pytest tests -x -q $T -m gpu > $OUT/tests.log 2>&1; echo "suite rc=$?"; tail -3 $OUT/tests.log
