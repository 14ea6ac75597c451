#!/bin/bash
# Round 3, session 2: one-launch small hashmap rounds (the combiner's) -- parity, combiner bench,
# combiner kernel trace; host time of the first round calls after a sync.
mkdir -p gpurun_out/m12
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_hashmap.py tests/test_gpu_combiner.py tests/test_gpu_replica_api.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/m12/tests.log 2>&1
rc=$?; tail -3 gpurun_out/m12/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 ./microbench/combiner_bench 2 > gpurun_out/m12/combiner.txt 2>&1; rc=$?
cat gpurun_out/m12/combiner.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/m12/kt_comb -o run -- ./microbench/combiner_bench 1 64 32 0 -1 0 > gpurun_out/m12/kt_comb.txt 2>&1 || exit 1
T=$(find gpurun_out/m12/kt_comb -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $T | head -8
timeout -k 10 120 python3 microbench/host_steps.py > gpurun_out/m12/host_steps.txt 2>&1; rc=$?
cat gpurun_out/m12/host_steps.txt | grep -v amdgpu.ids; exit $rc
