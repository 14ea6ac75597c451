#!/bin/bash
# Round 3, session 2: K1 1 vs 2 on read-dominated rounds (B1 and the N = 2 / 4 per-GPU rounds),
# one Get per read thread.
mkdir -p gpurun_out/m36
export TMPDIR=/tmp
N2='--ops-per-gpu 1100000 --write-ratio 18'
N4='--ops-per-gpu 1300000 --write-ratio 31'
timeout -k 10 900 python3 tools/sweep.py "n2_k2||$N2" "n2_k1||$N2 --knob K1=1" "n4_k2||$N4" "n4_k1||$N4 --knob K1=1" \
  "w20_k2||--write-ratio 20" "w20_k1||--write-ratio 20 --knob K1=1" "w5_k2||--write-ratio 5" "w5_k1||--write-ratio 5 --knob K1=1" \
  "n2_k2b||$N2" "n2_k1b||$N2 --knob K1=1" > gpurun_out/m36/sweep.txt 2>&1
rc=$?; cat gpurun_out/m36/sweep.txt; exit $rc
