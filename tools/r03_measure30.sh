#!/bin/bash
# Round 3, session 2: RPT 1 (new default) vs 2 confirmation -- hashmap parity, then alternating
# 400-step and 20-step (driver command) lines, reads-only and Zipf rounds.
mkdir -p gpurun_out/m30
export TMPDIR=/tmp
L=node-replication_amd/lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_hashmap.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m30/tests.log 2>&1
rc=$?; tail -2 gpurun_out/m30/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 tools/sweep.py "b1_r1||" "b1_r2|NRGPU_LIB=$L/libnrgpu_rpt2.so|" "b1_r1b||" "b1_r2b|NRGPU_LIB=$L/libnrgpu_rpt2.so|" \
  "s20_r1||--steps 20 --warmup 5" "s20_r2|NRGPU_LIB=$L/libnrgpu_rpt2.so|--steps 20 --warmup 5" \
  "r0_r1||--write-ratio 0" "r0_r2|NRGPU_LIB=$L/libnrgpu_rpt2.so|--write-ratio 0" \
  "z50_r1||--dist zipf --write-ratio 50" "z50_r2|NRGPU_LIB=$L/libnrgpu_rpt2.so|--dist zipf --write-ratio 50" \
  "w50_r1||--write-ratio 50" "w50_r2|NRGPU_LIB=$L/libnrgpu_rpt2.so|--write-ratio 50" > gpurun_out/m30/sweep.txt 2>&1
rc=$?; cat gpurun_out/m30/sweep.txt; exit $rc
