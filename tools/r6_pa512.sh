#!/bin/bash
# 512-thread partition apply as the default: hashmap suites + the N = 8 / configs[2] per-GPU rounds
set -o pipefail
O=gpurun_out/pa512; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hashmap.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_group_multi.py tests/test_gpu_combiner.py -m gpu > $O/t.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-prev-variant --ops-per-gpu 1700000 --write-ratio 47 > $O/n8.json 2> $O/n8.err &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-prev-variant --steps 60 --ops-per-gpu 4500000 --write-ratio 89 > $O/c2.json 2> $O/c2.err
rc=$?; tail -3 $O/t.log
for f in $O/*.json; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step']*1e3, d['roofline']['avg_launch_us'])"; done
exit $rc
