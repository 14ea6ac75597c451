#!/bin/bash
# B1: stamp rounds log copy streamed (lib_lg) vs lib
set -o pipefail
O=gpurun_out/lg; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_lg/libnrgpu.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hashmap.py tests/test_gpu_golden.py -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  for v in lib lib_lg; do
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read()); print('%-8s' % '$v', d['value'], round(d['ms_per_step']*1e3,3), d['roofline']['avg_launch_us'])"
  done
done
