#!/bin/bash
# Round 3, session 2: K1 2 vs 4 on the per-GPU rounds of the headline's N = 2 / 4 / 8 legs
# (10 % writes of every GPU's 1M ops replayed everywhere: 200k / 400k / 800k Puts + 900k Gets).
mkdir -p gpurun_out/m22
export TMPDIR=/tmp
N2='--ops-per-gpu 1100000 --write-ratio 18'
N4='--ops-per-gpu 1300000 --write-ratio 31'
N6='--ops-per-gpu 1500000 --write-ratio 40'
timeout -k 10 900 python3 tools/sweep.py "n2_k2||$N2" "n2_k4||$N2 --knob K1=4" "n4_k2||$N4" "n4_k4||$N4 --knob K1=4" \
  "n6_k2||$N6" "n6_k4||$N6 --knob K1=4" "n8_k1||--ops-per-gpu 1700000 --write-ratio 47 --knob K1=1" > gpurun_out/m22/sweep.txt 2>&1
rc=$?; cat gpurun_out/m22/sweep.txt; exit $rc
