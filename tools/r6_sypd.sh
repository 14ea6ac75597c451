#!/bin/bash
set -o pipefail
O=gpurun_out/sypd; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_pd4/libnrgpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_synthetic.py > $O/t4.log 2>&1 || exit $?
for i in 1 2 3; do for v in lib lib_pd2 lib_pd4; do
  NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --workload synthetic --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
done; done
tail -1 $O/t4.log
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
