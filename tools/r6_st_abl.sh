#!/bin/bash
set -o pipefail
O=gpurun_out/stabl; mkdir -p $O
for i in 1 2; do for x in 0 0x10000 0x20000 0x30000; do
  timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline --knob EXP=$x > $O/b_${x}_$i.json 2> $O/b_${x}_$i.err || exit $?
done; done
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
