#!/bin/bash
# stack finish workgroups: tiles per workgroup (NRG_ST_FIN_T builds), parity then A/B on one box
set -o pipefail
O=gpurun_out/stfin; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_t4/libnrgpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack.py tests/test_gpu_verify_stack.py > $O/t4.log 2>&1 || exit $?
NRGPU_LIB=node-replication_amd/lib_t8/libnrgpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack.py > $O/t8.log 2>&1 || exit $?
for i in 1 2; do for T in 1 2 4 8; do
  NRGPU_LIB=node-replication_amd/lib_t$T/libnrgpu.so timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline > $O/b_${T}_$i.json 2> $O/b_${T}_$i.err || exit $?
done; done
tail -1 $O/t4.log; tail -1 $O/t8.log
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
