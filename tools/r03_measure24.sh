#!/bin/bash
# Round 3, session 2: combiner wake tree fan-out 2 vs 4 (alternating runs on one box).
mkdir -p gpurun_out/m24
C="2 16 32 0 -1 0  64 32 0 -1 0  128 32 0 -1 0  256 32 0 -1 0"
for r in a b; do
  timeout -k 10 150 ./microbench/combiner_bench $C > gpurun_out/m24/fan2_$r.txt 2>&1 || exit 1
  timeout -k 10 150 ./microbench/combiner_bench_f4 $C > gpurun_out/m24/fan4_$r.txt 2>&1 || exit 1
done
for f in fan2_a fan4_a fan2_b fan4_b; do echo "== $f"; grep Mops gpurun_out/m24/$f.txt; done
# synthetic: op-major seen values (NRG_SY_VOP build) -- parity, then A/B
export TMPDIR=/tmp
L=node-replication_amd/lib
NRGPU_LIB=$L/libnrgpu_vop.so timeout -k 10 300 python -u -m pytest tests/test_gpu_synthetic.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m24/vop_tests.log 2>&1
rc=$?; tail -2 gpurun_out/m24/vop_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 tools/sweep.py 'sy||--workload synthetic' "sy_vop|NRGPU_LIB=$L/libnrgpu_vop.so|--workload synthetic" \
  'sy_b||--workload synthetic' "sy_vop_b|NRGPU_LIB=$L/libnrgpu_vop.so|--workload synthetic" > gpurun_out/m24/sy.txt 2>&1
rc=$?; cat gpurun_out/m24/sy.txt; exit $rc
