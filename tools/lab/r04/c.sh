#!/bin/bash
# r04c: deferred-reduction thread diagnostics, then the trunk-forward variants, the pc
# timeline and the bench A/B (fp32-tier transform; deferred reductions on/off)
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/diag/diag_defer.py > $OUT/defer.txt 2>&1; echo "defer diag rc=$?"; tail -12 $OUT/defer.txt | cut -c1-600
timeout -k 10 300 python -u tools/kbench.py --which copy,node_init --nmlab dflt,x3,nm3,dflt+mask,bf16,bf16+pc --iters 50 > $OUT/kb.txt 2>&1 || { tail -5 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
LEAKGNN_LIB=leak-det-gnn_amd/lib/stamps/libleakgnn.so timeout -k 10 300 python -u tools/kbench.py --which none --nmlab dflt,nm3 --stamps --iters 30 > $OUT/kb_stamps.txt 2>&1 || { tail -5 $OUT/kb_stamps.txt; exit 1; }
grep stamps $OUT/kb_stamps.txt
for v in 0 0x8000 0x20000; do
  LEAKGNN_GCN_FWD_NM_FLAGS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --no-c5 --no-pmc --no-tier-leg > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v failed"; tail -20 $OUT/bench_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
LEAKGNN_DEFER_REDUCE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --no-c5 --no-pmc --no-tier-leg > $OUT/bench_defer.json 2> $OUT/bench_defer.err || { echo "bench defer failed"; tail -20 $OUT/bench_defer.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench_defer.json')); print('defer', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
