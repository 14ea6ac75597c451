#!/bin/bash
# Round 3 session 2: apply stores {key, val} in one 16-B store (lib_a16) vs the 8-B value store --
# hashmap suites on lib_a16, then write-heavy rows A/B/A/B.
mkdir -p gpurun_out/m42
export TMPDIR=/tmp
A16=$PWD/node-replication_amd/lib_a16/libnrgpu.so
NRGPU_LIB=$A16 timeout -k 10 600 python -u -m pytest tests/test_gpu_hashmap.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m42/tests.log 2>&1
rc=$?; tail -2 gpurun_out/m42/tests.log; [ $rc -ne 0 ] && exit $rc
N8='--ops-per-gpu 1700000 --write-ratio 47'
C2='--ops-per-gpu 4500000 --write-ratio 89 --pool 16'
timeout -k 10 1000 python3 tools/sweep.py "w100||--write-ratio 100" "w100_a16|NRGPU_LIB=$A16|--write-ratio 100" \
  "c2||$C2" "c2_a16|NRGPU_LIB=$A16|$C2" "n8||$N8" "n8_a16|NRGPU_LIB=$A16|$N8" \
  "w100b||--write-ratio 100" "w100_a16b|NRGPU_LIB=$A16|--write-ratio 100" "c2b||$C2" "c2_a16b|NRGPU_LIB=$A16|$C2" \
  "b1||" "b1_a16|NRGPU_LIB=$A16|" > gpurun_out/m42/sweep.txt 2>&1
rc=$?; cat gpurun_out/m42/sweep.txt; exit $rc
