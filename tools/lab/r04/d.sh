#!/bin/bash
# r04d: compressed node init after the unconditional-load fix, the latency-first sensor
# projection, the per-workgroup dynamic tile dealing in pc; then the deferred-reduction
# graph tests and the whole suite
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_x0.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/x0.log 2>&1 || { echo "x0 tests failed"; tail -40 $OUT/x0.log; exit 1; }
tail -1 $OUT/x0.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "edge or heads" > $OUT/edge.log 2>&1 || { echo "edge tests failed"; tail -40 $OUT/edge.log; exit 1; }
tail -1 $OUT/edge.log
timeout -k 10 300 python -u tools/kbench.py --which edge_fwd,edge_bwd --iters 50 > $OUT/kb_edge.txt 2>&1 || { tail -5 $OUT/kb_edge.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb_edge.txt
timeout -k 10 300 python -u tools/kbench.py --which node_init,node_init_bits,gcn_fwd_x0,gcn_bwd_x0,gcn_fwd_nm_train,gcn_bwd_nm_l0s,copy --nmlab dflt,dflt+mask --iters 50 > $OUT/kb.txt 2>&1 || { tail -5 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
LEAKGNN_LIB=leak-det-gnn_amd/lib/stamps/libleakgnn.so timeout -k 10 300 python -u tools/kbench.py --which none --nmlab dflt --stamps --iters 30 > $OUT/kb_stamps.txt 2>&1 || { tail -5 $OUT/kb_stamps.txt; exit 1; }
grep stamps $OUT/kb_stamps.txt | cut -c1-1500
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --no-c5 --no-pmc --no-tier-leg > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
LEAKGNN_DEFER_REDUCE=1 timeout -k 10 300 python -u -m pytest tests/test_graph_step.py tests/test_gpu_library.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/defer_tests.log 2>&1; echo "defer tests rc=$?"; tail -3 $OUT/defer_tests.log
LEAKGNN_DEFER_REDUCE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --no-c5 --no-pmc --no-tier-leg > $OUT/bench_defer.json 2> $OUT/bench_defer.err || { echo "bench defer failed"; tail -20 $OUT/bench_defer.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench_defer.json')); print('defer', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/tests.log 2>&1; echo "suite rc=$?"; tail -3 $OUT/tests.log
