#!/bin/bash
# Collect PMC counter passes for kbench kernels (run on the GPU box via gpurun).
#   bash tools/pmc.sh <which> <outdir> [B]
# One rocprofv3 invocation per counter group (gfx950 cannot co-schedule them all);
# kernel-trace only, never combined with sys/runtime tracing.
set -e
WHICH=${1:-gcn_fwd}; OUT=${2:-gpurun_out/pmc}; B=${3:-256}; shift 3; EXTRA="$@"
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
  "FETCH_SIZE" "WRITE_SIZE" \
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_MFMA"; do
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- \
      python3 tools/kbench.py --which "$WHICH" --B "$B" --iters 20 $EXTRA > "$OUT/p$i.log" 2>&1
  i=$((i+1))
done
