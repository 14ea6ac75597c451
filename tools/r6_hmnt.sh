#!/bin/bash
# B1: streamed apply value stores (lib_ap), streamed index tags (lib_tag), both (lib_at) vs lib
set -o pipefail
O=gpurun_out/hmnt; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_at/libnrgpu.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hashmap.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
  for v in lib lib_ap lib_tag lib_at; do
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-prev-variant > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read()); print('%-8s' % '$v', d['value'], round(d['ms_per_step']*1e3,3), d['roofline']['avg_launch_us'])"
  done
done
