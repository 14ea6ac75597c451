#!/bin/bash
# Round 3, session 2: K1 = 1 for small stamp rounds -- hashmap parity suites, then B1 lines.
mkdir -p gpurun_out/m37
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hashmap.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_log.py tests/test_gpu_edge.py tests/test_gpu_group_multi.py tests/test_gpu_replica_api.py tests/test_gpu_partition.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m37/tests.log 2>&1
rc=$?; tail -2 gpurun_out/m37/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 tools/sweep.py "b1||" "b1_20|| --steps 20 --warmup 5" "b1b||" "n2||--ops-per-gpu 1100000 --write-ratio 18" > gpurun_out/m37/sweep.txt 2>&1
rc=$?; cat gpurun_out/m37/sweep.txt; exit $rc
