#!/bin/bash
# stack: the previous chunk's finish inside the tile workgroups (lib_v) vs separate finish workgroups (lib)
set -o pipefail
O=gpurun_out/stm; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_v/libnrgpu.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack.py tests/test_gpu_verify_stack.py tests/test_gpu_golden.py tests/test_gpu_stream_order.py tests/test_gpu_group_multi.py tests/test_gpu_combiner.py -k "stack or golden or order" > $O/t.log 2>&1 || exit $?
for i in 1 2 3; do for v in lib lib_v; do
  NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
done; done
tail -1 $O/t.log
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
