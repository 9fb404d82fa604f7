#!/bin/bash
# r04b: the compressed node init (x0 bits) on the GPU: its parity tests first, then the
# whole GPU suite, the trunk-forward variants and pc timeline, and the bench (in-step A/B
# of the fp32-tier transform and of the compressed node init).
set -o pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_x0.py -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/x0.log 2>&1 || { echo "x0 tests failed"; tail -40 $OUT/x0.log; exit 1; }
tail -2 $OUT/x0.log
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/kbench.py --which copy,node_init --nmlab dflt,x3,nm3,dflt+mask,bf16,bf16+pc --iters 50 > $OUT/kb.txt 2>&1 || { tail -5 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
LEAKGNN_LIB=leak-det-gnn_amd/lib/stamps/libleakgnn.so timeout -k 10 300 python -u tools/kbench.py --which none --nmlab dflt,nm3 --stamps --iters 30 > $OUT/kb_stamps.txt 2>&1 || { tail -5 $OUT/kb_stamps.txt; exit 1; }
grep stamps $OUT/kb_stamps.txt
for v in 0 0x8000 0x20000; do
  LEAKGNN_GCN_FWD_NM_FLAGS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --no-c5 --no-pmc --no-tier-leg > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v failed"; tail -20 $OUT/bench_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
