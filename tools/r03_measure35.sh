#!/bin/bash
# Round 3, session 2: K1 (Puts per stamp-index thread) re-checked with one Get per read thread.
mkdir -p gpurun_out/m35
export TMPDIR=/tmp
N8='--ops-per-gpu 1700000 --write-ratio 47'
timeout -k 10 900 python3 tools/sweep.py "b1_k2||" "b1_k1||--knob K1=1" "b1_k4||--knob K1=4" \
  "n8_k4||$N8" "n8_k2||$N8 --knob K1=2" "w50_k2||--write-ratio 50" "w50_k1||--write-ratio 50 --knob K1=1" "w50_k4||--write-ratio 50 --knob K1=4" \
  "b1_k2b||" "b1_k1b||--knob K1=1" > gpurun_out/m35/sweep.txt 2>&1
rc=$?; cat gpurun_out/m35/sweep.txt; exit $rc
