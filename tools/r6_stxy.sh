#!/bin/bash
# stack: look-back loads after the query-structure barrier (X = lib_t9), plus the previous chunk's tile minima copied to LDS by wave 0 (W = lib_t8)
set -o pipefail
O=gpurun_out/stxw; mkdir -p $O
X=node-replication_amd/lib_t9/libnrgpu.so; W=node-replication_amd/lib_t8/libnrgpu.so
timeout -k 10 300 env NRGPU_LIB=$W python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack.py tests/test_gpu_verify_stack.py tests/test_gpu_golden.py tests/test_gpu_stream_order.py -m gpu > $O/tW.log 2>&1 || exit $?
timeout -k 10 300 env NRGPU_LIB=$X python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack.py tests/test_gpu_golden.py -m gpu > $O/tX.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline > $O/b_lib_$i.json 2> $O/b_lib_$i.err || exit $?
  NRGPU_LIB=$X timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline > $O/b_X_$i.json 2> $O/b_X_$i.err || exit $?
  NRGPU_LIB=$W timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline > $O/b_W_$i.json 2> $O/b_W_$i.err || exit $?
done
for v in lib X W; do L=node-replication_amd/$([ $v = lib ] && echo lib || ([ $v = X ] && echo lib_t9 || echo lib_t8))/libnrgpu.so
  NRGPU_LIB=$L BB=8 timeout -k 10 200 python -u microbench/stack_phases.py > $O/ph_$v.txt 2>&1 || exit $?; done
tail -1 $O/tW.log; tail -1 $O/tX.log
for f in $O/b*.json; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['ms_per_step']*1e3, d['roofline']['avg_launch_us'])"; done
for v in lib X W; do echo "== $v"; grep -E "publish|last tile end|lookback|queries  " $O/ph_$v.txt; done
