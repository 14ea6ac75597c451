#!/bin/bash
# Stack response-store policy: A/B of the unfixed (lib_s8u) and fixed (lib) builds on one box,
# race stress on the fixed build, then the full GPU suite on it
set -o pipefail
O=gpurun_out/resp; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib/libnrgpu.so ROUNDS=48 timeout -k 10 200 python -u microbench/stack_stress.py > $O/stress_lib.txt 2>&1 || exit $?
grep TOTAL_BAD $O/stress_lib.txt
for i in 1 2 3; do
  for v in lib_s8u lib; do
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --workload stack --steps 400 --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read()); print('$v', d['value'], round(d['ms_per_step']*1e3,3), d['roofline']['avg_launch_us'])"
  done
done
timeout -k 10 900 python -u -m pytest -x -q --durations=5 --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1; rc=$?
tail -8 $O/suite.log; exit $rc
