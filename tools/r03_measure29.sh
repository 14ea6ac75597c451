#!/bin/bash
# Round 3, session 2: Gets per read-role thread (RPT 1 / 2 / 4) on B1 and the N=8 per-GPU round.
mkdir -p gpurun_out/m29
export TMPDIR=/tmp
L=node-replication_amd/lib
N8='--ops-per-gpu 1700000 --write-ratio 47'
timeout -k 10 900 python3 tools/sweep.py "b1_r2||" "b1_r1|NRGPU_LIB=$L/libnrgpu_rpt1.so|" "b1_r4|NRGPU_LIB=$L/libnrgpu_rpt4.so|" \
  "n8_r2||$N8" "n8_r1|NRGPU_LIB=$L/libnrgpu_rpt1.so|$N8" "n8_r4|NRGPU_LIB=$L/libnrgpu_rpt4.so|$N8" \
  "r0_r2||--write-ratio 0" "r0_r4|NRGPU_LIB=$L/libnrgpu_rpt4.so|--write-ratio 0" \
  "b1_r2b||" "b1_r4b|NRGPU_LIB=$L/libnrgpu_rpt4.so|" > gpurun_out/m29/sweep.txt 2>&1
rc=$?; cat gpurun_out/m29/sweep.txt; exit $rc
