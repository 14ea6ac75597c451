#!/bin/bash
# synthetic one-launch round: parity (synthetic, golden, group, combiner, stream-order suites) and A/B
set -o pipefail
O=gpurun_out/sy; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_synthetic.py tests/test_gpu_golden.py tests/test_gpu_stream_order.py > $O/t.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_group_multi.py tests/test_gpu_group_threads.py tests/test_gpu_combiner.py -k "synth or sy_" > $O/t2.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload synthetic --no-cpu-baseline > $O/f$i.json 2> $O/f$i.err &&
  timeout -k 10 200 python bench.py --workload synthetic --no-cpu-baseline --knob SY_FUSED=0 > $O/u$i.json 2> $O/u$i.err || exit $?
done
rc=$?; tail -3 $O/t.log; tail -3 $O/t2.log
for f in $O/*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
exit $rc
