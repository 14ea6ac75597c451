#!/bin/bash
# Stack: streamed `some` bytes (lib_some), streamed finish stores (lib_fin), both (lib_both) vs lib
set -o pipefail
O=gpurun_out/stnt; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_both/libnrgpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack.py tests/test_gpu_verify_stack.py tests/test_gpu_golden.py tests/test_gpu_stream_order.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
NRGPU_LIB=node-replication_amd/lib_both/libnrgpu.so ROUNDS=24 timeout -k 10 150 python -u microbench/stack_stress.py > $O/stress_both.txt 2>&1 || exit $?
grep TOTAL_BAD $O/stress_both.txt
for i in 1 2; do
  for v in lib lib_some lib_fin lib_both; do
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --workload stack --steps 400 --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read()); print('%-9s' % '$v', d['value'], round(d['ms_per_step']*1e3,3), d['roofline']['avg_launch_us'])"
  done
done
