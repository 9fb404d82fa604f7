#!/bin/bash
# r04j: the EdgeHead backward on the f16x2 transform: parity, timing (product + lab), bench
set -o pipefail
OUT=gpurun_out/r04j; mkdir -p $OUT
export TMPDIR=/tmp
T="--timeout 120 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_library.py tests/test_gpu_configs.py -x -q $T -m gpu -k "edge or heads or scatter or detector or b256 or c4" > $OUT/edge.log 2>&1; echo "edge tests rc=$?"; grep -E "FAILED|passed|failed|^E " $OUT/edge.log | head -20
timeout -k 10 300 python -u tools/kbench.py --which edge_bwd --iters 50 > $OUT/kb.txt 2>&1 || { tail -20 $OUT/kb.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb.txt
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 300 python -u tools/kbench.py --which edge_bwd --edgebwdlab 4 --iters 50 > $OUT/kb_lab.txt 2>&1 || { tail -20 $OUT/kb_lab.txt; exit 1; }
grep -v amdgpu.ids $OUT/kb_lab.txt | grep lab
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --no-c5 --no-pmc --no-tier-leg > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
