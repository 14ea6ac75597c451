#!/bin/bash
# Round 3, session 2: Puts per stamp-index thread (K1 2 vs 4) by round size.
mkdir -p gpurun_out/m21
export TMPDIR=/tmp
N8='--ops-per-gpu 1700000 --write-ratio 47'
timeout -k 10 900 python3 tools/sweep.py "w50_k2||--write-ratio 50" "w50_k4||--write-ratio 50 --knob K1=4" \
  "n8_k2||$N8" "n8_k4||$N8 --knob K1=4" "w100_k2||--write-ratio 100" "w100_k4||--write-ratio 100 --knob K1=4" \
  "p2m_k2||--ops-per-gpu 2000000 --write-ratio 100 --pool 16" "p2m_k4||--ops-per-gpu 2000000 --write-ratio 100 --pool 16 --knob K1=4" \
  "b1_k2||" "b1_k4||--knob K1=4" "n8_k2b||$N8" "n8_k4b||$N8 --knob K1=4" > gpurun_out/m21/sweep.txt 2>&1
rc=$?; cat gpurun_out/m21/sweep.txt; exit $rc
