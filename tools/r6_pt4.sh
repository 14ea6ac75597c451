#!/bin/bash
set -o pipefail
O=gpurun_out/pt4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_partition.py tests/test_gpu_group_multi.py -k "partition" > $O/t.log 2>&1 &&
for i in 1 2 3; do for x in 0 0x8000; do timeout -k 10 200 python bench.py --partitioned --no-cpu-baseline --no-prev-variant --knob EXP=$x > $O/b_${x}_$i.json 2> $O/b_${x}_$i.err || exit $?; done; done
rc=$?; tail -3 $O/t.log
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['round']['host_enqueue_us'])"; done
exit $rc
