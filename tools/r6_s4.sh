#!/bin/bash
# Stack: response-store race stress (unfixed/fixed, 8 and 4 ops per lane), parity suite on the
# 4-op build, and the bench A/B of the fixed builds
set -o pipefail
O=gpurun_out/s4; mkdir -p $O
for v in lib_s8u lib lib_s4 lib_s4f; do
  L=node-replication_amd/$v/libnrgpu.so; [ $v = lib ] && L=node-replication_amd/lib/libnrgpu.so
  NRGPU_LIB=$L ROUNDS=24 timeout -k 10 150 python -u microbench/stack_stress.py > $O/stress_$v.txt 2>&1 || { echo "stress $v rc=$?"; tail -5 $O/stress_$v.txt; exit 1; }
  echo "$v: $(grep TOTAL_BAD $O/stress_$v.txt)"
done
NRGPU_LIB=node-replication_amd/lib_s4f/libnrgpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack.py tests/test_gpu_verify_stack.py tests/test_gpu_golden.py tests/test_gpu_stream_order.py > $O/t4.log 2>&1 || { tail -30 $O/t4.log; exit 1; }
tail -1 $O/t4.log
for i in 1 2; do
  for v in lib_s4f lib; do
    L=node-replication_amd/$v/libnrgpu.so; [ $v = lib ] && L=node-replication_amd/lib/libnrgpu.so
    NRGPU_LIB=$L timeout -k 10 200 python bench.py --workload stack --steps 400 --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read()); print('$v', d['value'], round(d['ms_per_step']*1e3,3), d['roofline']['avg_launch_us'])"
  done
done
