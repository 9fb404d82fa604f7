#!/bin/bash
# r02ag: bench with the HIP copy-kernel peak beside torch copy_, and the PMC counter summary
# of the hot kernels in the RCM-scheduled state
set -o pipefail
OUT=gpurun_out/r02ag; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['stream_copy'], d['roofline']['frac'], d['roofline']['frac_of_measured_copy'], d['roofline']['traffic'], d['roofline_bwd']['traffic'])"
timeout -k 10 600 python -u tools/pmc_kernels.py --out $OUT --tag r02ag > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
grep -E "==|WAIT_INST_ANY/|MFMA_busy|duration|HBM_bytes|L2_hit" $OUT/pmc_r02ag.txt
