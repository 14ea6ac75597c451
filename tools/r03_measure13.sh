#!/bin/bash
# Round 3, session 2: combiner wake tree (per-waiter futex words) -- parity, then the combiner bench.
mkdir -p gpurun_out/m13
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_combiner.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m13/tests.log 2>&1
rc=$?; tail -3 gpurun_out/m13/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 ./microbench/combiner_bench 2 > gpurun_out/m13/combiner.txt 2>&1; rc=$?
cat gpurun_out/m13/combiner.txt; exit $rc
