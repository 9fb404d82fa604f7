#!/bin/bash
# r04z4: the committed state once more: the full GPU suite and the driver's smoke()
set -o pipefail
OUT=gpurun_out/r04z4; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
rc=$?; echo "rc=$rc"; tail -2 $OUT/tests.log; tail -3 $OUT/smoke.txt; exit $rc
