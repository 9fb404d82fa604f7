#!/bin/bash
# r03z: C5 gather-structure lab (tools/lab/c5_lab.hip, built in-tree as build/c5_lab)
set -o pipefail
OUT=gpurun_out/r03z; mkdir -p $OUT
timeout -k 10 120 build/c5_lab > $OUT/c5_lab.txt 2>&1; rc=$?; cat $OUT/c5_lab.txt; exit $rc
