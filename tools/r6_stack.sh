#!/bin/bash
set -o pipefail
O=gpurun_out/st; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack.py tests/test_gpu_verify_stack.py tests/test_gpu_golden.py tests/test_gpu_stream_order.py > $O/t.log 2>&1 &&
BB=8 timeout -k 10 120 python microbench/stack_phases.py > $O/phases.txt 2>&1 &&
for i in 1 2; do timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline > $O/b$i.json 2> $O/b$i.err || exit $?; done
rc=$?; tail -3 $O/t.log; head -9 $O/phases.txt
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
exit $rc
