#!/bin/bash
set -o pipefail
O=gpurun_out/sysu; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_v/libnrgpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_synthetic.py > $O/t.log 2>&1 || exit $?
for i in 1 2 3; do for v in lib lib_v; do
  NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --workload synthetic --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
done; done
tail -1 $O/t.log
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
