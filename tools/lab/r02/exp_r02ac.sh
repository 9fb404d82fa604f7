#!/bin/bash
# r02ac: occupancy of the node-major forward: 5-wave (3 per CU: 15 waves/CU) and 8-wave
# (<= 128 VGPRs, 2 per CU) workgroups against the 4-wave default (3 per CU by LDS)
set -o pipefail
OUT=gpurun_out/r02ac; mkdir -p $OUT
timeout -k 10 240 python tools/kbench.py --which gcn_fwd_nm_train --nmlab "bpc3,w5+bpc3,w8+bpc2,bpc3,w5+bpc3,w8+bpc2" --iters 40 > $OUT/kb.txt 2>&1 || { tail -20 $OUT/kb.txt; exit 1; }
grep -v amdgpu $OUT/kb.txt | tail -14
