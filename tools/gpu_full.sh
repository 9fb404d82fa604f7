#!/bin/bash
# Full GPU pass: every -m gpu test (no -x, so one failure does not hide the rest), then the
# bench line, the rocprofv3 stats run and the kbench isolates.  Stops before the bench if the
# tests ended in anything but pass/fail (a timeout, abort or fault).
#   bash tools/gpu_full.sh <tag>
set -o pipefail
TAG=${1:-run}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?
tail -4 "$OUT/tests.log"
if [[ $rc -gt 1 ]] || grep -q "+++ Timeout" "$OUT/tests.log"; then echo "tests ended abnormally (rc=$rc)"; exit 1; fi
bash tools/gpu_round.sh "$TAG" bench && bash tools/gpu_round.sh "$TAG" prof || exit 1
timeout -k 10 200 python tools/kbench.py --which gcn_bwd_nm,gcn_bwd_nm_l0,gcn_bwd_nm_l0s,node_init --iters 30 > "$OUT/kb.txt" 2>&1 || exit 1
tail -3 "$OUT/kb.txt"
exit $rc
