#!/bin/bash
# Round 3, session 2: synthetic bucket pass size (SYB_PER 8 = 4096 touches per pass, 10 = 5120:
# two passes per 1M-op bucket instead of three), E positions recomputed instead of kept.
mkdir -p gpurun_out/m19
export TMPDIR=/tmp
L=node-replication_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_synthetic.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m19/tests8.log 2>&1
rc=$?; tail -2 gpurun_out/m19/tests8.log; [ $rc -ne 0 ] && exit $rc
NRGPU_LIB=$L/libnrgpu_per10.so timeout -k 10 300 python -u -m pytest tests/test_gpu_synthetic.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m19/tests10.log 2>&1
rc=$?; tail -2 gpurun_out/m19/tests10.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 tools/sweep.py 'sy_per8||--workload synthetic' "sy_per10|NRGPU_LIB=$L/libnrgpu_per10.so|--workload synthetic" \
  'sy_per8b||--workload synthetic' "sy_per10b|NRGPU_LIB=$L/libnrgpu_per10.so|--workload synthetic" > gpurun_out/m19/sy.txt 2>&1
rc=$?; cat gpurun_out/m19/sy.txt; exit $rc
