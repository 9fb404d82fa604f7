#!/bin/bash
# EdgeHead prefetch loads in flight (unconditional, exact-width ids, unconditional body pairs): A/B, parity, bench
set -o pipefail
OUT=gpurun_out/r02aa; mkdir -p $OUT
for v in old new; do
  if [ $v = old ]; then export LEAKGNN_LIB=$PWD/leak-det-gnn_amd/lib/ab/old.so; else unset LEAKGNN_LIB; fi
  echo "== $v"; timeout -k 10 180 python tools/kbench.py --which edge_fwd,edge_bwd --iters 30 > $OUT/kb_$v.txt 2>&1 || exit 1
  grep -v amdgpu $OUT/kb_$v.txt | tail -5
done
unset LEAKGNN_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "head or edge or b256 or b64 or detector or captured or bf16 or c4 or C4" > $OUT/tests.txt 2>&1; rc=$?; tail -5 $OUT/tests.txt; [ $rc = 0 ] || exit 1
timeout -k 10 600 python bench.py --no-pmc --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us']); print(d['mlp_tier']['value'], d['c4']['value'], d['e2e_training']['value'])"
