#!/bin/bash
# r02c: graph-timed forward sweep (nm3 vs nm2 schedules) + PMC counters of nm3 / nm2 / bwd
set -o pipefail
OUT=gpurun_out/r02c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python tools/kbench.py --which gcn_fwd_nm,gcn_fwd_nm_train,spmm,copy,gcn_bwd_nm --B 256 --iters 100 > $OUT/kb.txt 2>&1 || { cat $OUT/kb.txt; exit 1; }
cat $OUT/kb.txt
LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so timeout -k 10 300 python tools/kbench.py --which none --B 256 --iters 100 \
  --nmlab nm2,nm2+bpc3,nm2+bpc2,nm2+nomfma,nm2+noload,nomfma,noload,nomfma+noload,w8,f32,bpc2,bpc3,w8+bpc1 > $OUT/kblab.txt 2>&1 || { cat $OUT/kblab.txt; exit 1; }
cat $OUT/kblab.txt
timeout -k 10 200 python tools/kbench.py --which gcn_fwd_nm_train,copy --B 1024 --iters 50 > $OUT/kb1024.txt 2>&1 && cat $OUT/kb1024.txt
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_SMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $OUT/pmc/p$i -o run --output-format csv -- \
      python3 tools/kbench.py --which gcn_fwd_nm_train,gcn_bwd_nm --B 256 --iters 20 --eager > $OUT/pmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc_p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
