#!/bin/bash
# Round 3, session 2: stack kernel A/B -- this round's speculative queries (waves 1-3 answer the
# unmatched Pops while wave 0 does the look-back) vs the round-2 stack.hip, same box, alternating.
mkdir -p gpurun_out/m31
export TMPDIR=/tmp
L=node-replication_amd/lib
timeout -k 10 600 python3 tools/sweep.py "st||--workload stack" "st_r2|NRGPU_LIB=$L/libnrgpu_stkr2.so|--workload stack" \
  "st_b||--workload stack" "st_r2b|NRGPU_LIB=$L/libnrgpu_stkr2.so|--workload stack" \
  "st_c||--workload stack" "st_r2c|NRGPU_LIB=$L/libnrgpu_stkr2.so|--workload stack" > gpurun_out/m31/sweep.txt 2>&1
rc=$?; cat gpurun_out/m31/sweep.txt; exit $rc
