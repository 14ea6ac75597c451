#!/bin/bash
# Round 3, session 2: round-launch block order A/B (index, apply, reads vs index/read blocks
# alternating first; NRG_RK_MIX build), over B1 and the write-heavy shapes.
mkdir -p gpurun_out/m23
export TMPDIR=/tmp
M="NRGPU_LIB=node-replication_amd/lib/libnrgpu_mix.so"
N8='--ops-per-gpu 1700000 --write-ratio 47'
N4='--ops-per-gpu 1300000 --write-ratio 31'
timeout -k 10 900 python3 tools/sweep.py "b1||" "b1_mix|$M|" "n8||$N8" "n8_mix|$M|$N8" "n8_k2_mix|$M|$N8 --knob K1=2" \
  "n4||$N4" "n4_mix|$M|$N4" "w50||--write-ratio 50" "w50_mix|$M|--write-ratio 50" "b1b||" "b1b_mix|$M|" > gpurun_out/m23/sweep.txt 2>&1
rc=$?; cat gpurun_out/m23/sweep.txt; exit $rc
