#!/bin/bash
# Previous-value rounds: apply value stores + answers streamed (lib_pv) vs lib
set -o pipefail
O=gpurun_out/pv; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_pv/libnrgpu.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hashmap.py tests/test_gpu_golden.py tests/test_gpu_partition.py tests/test_gpu_reference_examples.py -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  for v in lib lib_pv; do
    for w in 10 50; do
      NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --write-ratio $w > $O/b_${v}_${w}_$i.json 2> $O/b_${v}_${w}_$i.err || exit $?
      python3 -c "import json; d=json.loads(open('$O/b_${v}_${w}_$i.json').read()); print('%-7s w%-3s' % ('$v', '$w'), d['value'], 'prev-values variant', d['variants']['prev_value_responses_Mops'])"
    done
  done
done
