#!/bin/bash
# stack: wave 0 issues no store before its look-back (hand-off) vs round 5 (EXP bit 7)
set -o pipefail
O=gpurun_out/sth; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack.py tests/test_gpu_verify_stack.py tests/test_gpu_golden.py tests/test_gpu_stream_order.py -m gpu > $O/t.log 2>&1 &&
BB=8 timeout -k 10 200 python -u microbench/stack_phases.py > $O/ph8.txt 2>&1 &&
for i in 1 2; do for x in 0 0x80; do
  timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline --knob EXP=$x > $O/b_${x}_$i.json 2> $O/b_${x}_$i.err || exit $?
done; done
rc=$?
tail -2 $O/t.log; cat $O/ph8.txt
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
exit $rc
