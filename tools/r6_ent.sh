#!/bin/bash
# Partition apply value stores streamed for rounds of <= 2M Puts (lib) vs plain (lib_ent)
set -o pipefail
O=gpurun_out/ent; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_ent/libnrgpu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hashmap.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_partition.py tests/test_gpu_group_multi.py tests/test_gpu_group_threads.py -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
B="python bench.py --no-cpu-baseline --no-prev-variant"
for i in 1 2; do
  for v in lib_ent lib; do
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 $B --ops-per-gpu 1700000 --write-ratio 47 > $O/n8_${v}_$i.json 2> $O/n8_${v}_$i.err || exit $?
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 $B --write-ratio 100 > $O/w100_${v}_$i.json 2> $O/w100_${v}_$i.err || exit $?
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 $B --steps 60 --ops-per-gpu 4500000 --write-ratio 89 > $O/c2_${v}_$i.json 2> $O/c2_${v}_$i.err || exit $?
    for w in n8 w100 c2; do python3 -c "import json; d=json.loads(open('$O/${w}_${v}_$i.json').read()); print('%-4s %-8s' % ('$w', '$v'), d['value'], round(d['ms_per_step']*1e3,3), d['roofline']['avg_launch_us'])"; done
  done
done
