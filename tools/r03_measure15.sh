#!/bin/bash
# Round 3, session 2: small rounds with Gets resolved beside the Puts -- parity, combiner bench, trace.
mkdir -p gpurun_out/m15
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_hashmap.py tests/test_gpu_combiner.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/m15/tests.log 2>&1
rc=$?; tail -3 gpurun_out/m15/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 ./microbench/combiner_bench 2 16 32 0 -1 0  64 32 0 -1 0  128 32 0 -1 0  256 32 0 -1 0 > gpurun_out/m15/combiner.txt 2>&1; rc=$?
cat gpurun_out/m15/combiner.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/m15/kt_comb -o run -- ./microbench/combiner_bench 1 64 32 0 -1 0 > gpurun_out/m15/kt_comb.txt 2>&1 || exit 1
T=$(find gpurun_out/m15/kt_comb -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $T | head -4 | cut -c1-60,100-
