#!/bin/bash
# Partition apply value stores streamed (lib_pa) vs lib: parity, then N = 8 / configs[2] / 50 % writes per-GPU rounds
set -o pipefail
O=gpurun_out/pant; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_pa/libnrgpu.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hashmap.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_partition.py -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
B="python bench.py --no-cpu-baseline --no-prev-variant"
for i in 1 2; do
  for v in lib lib_pa; do
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 $B --ops-per-gpu 1700000 --write-ratio 47 > $O/n8_${v}_$i.json 2> $O/n8_${v}_$i.err || exit $?
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 $B --write-ratio 50 > $O/w50_${v}_$i.json 2> $O/w50_${v}_$i.err || exit $?
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 $B --steps 60 --ops-per-gpu 4500000 --write-ratio 89 > $O/c2_${v}_$i.json 2> $O/c2_${v}_$i.err || exit $?
    for w in n8 w50 c2; do python3 -c "import json; d=json.loads(open('$O/${w}_${v}_$i.json').read()); print('%-4s %-7s' % ('$w', '$v'), d['value'], round(d['ms_per_step']*1e3,3), d['roofline']['avg_launch_us'])"; done
  done
done
