#!/bin/bash
# Round 3, session 2: synthetic after the tile-map barrier fix -- parity (default and op-major V
# builds, synthetic + golden + group suites), then the bench A/B.
mkdir -p gpurun_out/m25
export TMPDIR=/tmp
L=node-replication_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_synthetic.py tests/test_gpu_golden.py tests/test_gpu_group_multi.py tests/test_gpu_combiner.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m25/tests.log 2>&1
rc=$?; tail -2 gpurun_out/m25/tests.log; [ $rc -ne 0 ] && exit $rc
NRGPU_LIB=$L/libnrgpu_vop.so timeout -k 10 300 python -u -m pytest tests/test_gpu_synthetic.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m25/vop_tests.log 2>&1
rc=$?; tail -2 gpurun_out/m25/vop_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 tools/sweep.py 'sy||--workload synthetic' "sy_vop|NRGPU_LIB=$L/libnrgpu_vop.so|--workload synthetic" \
  'sy_b||--workload synthetic' "sy_vop_b|NRGPU_LIB=$L/libnrgpu_vop.so|--workload synthetic" > gpurun_out/m25/sy.txt 2>&1
rc=$?; cat gpurun_out/m25/sy.txt; exit $rc
