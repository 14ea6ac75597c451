#!/bin/bash
# Round 3, session 2: synthetic sums with batched loads + packed ranked touches; the partition's
# op-record prefetch depth (1, 2, 4 wave rounds) A/B. Parity of the default build first.
mkdir -p gpurun_out/m10
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_synthetic.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/m10/tests.log 2>&1
rc=$?; tail -3 gpurun_out/m10/tests.log; [ $rc -ne 0 ] && exit $rc
L=node-replication_amd/lib
timeout -k 10 400 python3 tools/sweep.py 'sy_pd1||--workload synthetic' "sy_pd2|NRGPU_LIB=$L/libnrgpu_pd2.so|--workload synthetic" \
  "sy_pd4|NRGPU_LIB=$L/libnrgpu_pd4.so|--workload synthetic" 'sy_pd1b||--workload synthetic' \
  "sy_pd4b|NRGPU_LIB=$L/libnrgpu_pd4.so|--workload synthetic" > gpurun_out/m10/sy.txt 2>&1
rc=$?; cat gpurun_out/m10/sy.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 microbench/synth_phases.py > gpurun_out/m10/synth_phases.txt 2>&1; rc=$?
head -16 gpurun_out/m10/synth_phases.txt; exit $rc
