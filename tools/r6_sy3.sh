#!/bin/bash
# fused synthetic round A/B: streaming stores for the outputs, sums placement
set -o pipefail
O=gpurun_out/sy3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_synthetic.py -k "bench_size or heavy or pipelined" > $O/t.log 2>&1 || exit $?
for i in 1 2; do for x in 0 0x3C0 0x40 0x140 0x4000; do
  timeout -k 10 200 python bench.py --workload synthetic --no-cpu-baseline --knob EXP=$x > $O/b_${x}_$i.json 2> $O/b_${x}_$i.err || exit $?
done; done
tail -2 $O/t.log
for f in $O/b_*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
