#!/bin/bash
# Round 3 session 2: sum workgroups of SYS_T tiles (default 2) vs 1 (lib_t1) -- synthetic suites,
# then synthetic bench lines A/B/A/B and the phase profile of the default.
mkdir -p gpurun_out/m39
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_synthetic.py tests/test_gpu_golden.py tests/test_gpu_group.py tests/test_gpu_group_multi.py tests/test_gpu_combiner.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m39/tests.log 2>&1
rc=$?; tail -2 gpurun_out/m39/tests.log; [ $rc -ne 0 ] && exit $rc
T1=NRGPU_LIB=$PWD/node-replication_amd/lib_t1/libnrgpu.so
timeout -k 10 900 python3 tools/sweep.py "t2||--workload synthetic" "t1|$T1|--workload synthetic" "t2b||--workload synthetic" "t1b|$T1|--workload synthetic" > gpurun_out/m39/sweep.txt 2>&1
rc=$?; cat gpurun_out/m39/sweep.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 microbench/synth_phases.py > gpurun_out/m39/synth_phases.txt 2>&1; rc=$?
head -12 gpurun_out/m39/synth_phases.txt; exit $rc
