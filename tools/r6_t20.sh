#!/bin/bash
# the driver's 20-step line: opening variants, alternating runs on one box
set -o pipefail
O=gpurun_out/t20; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-prev-variant --steps 20 --warmup 5"
for i in 1 2 3 4 5; do
  for m in "spin" "spin --prime-call" "keep" "keep --prime-call"; do
    tag=$(echo $m | tr -d ' -')
    timeout -k 10 120 $B --opening $m > $O/${tag}_$i.json 2> $O/${tag}_$i.err || exit $?
    python3 -c "import json; b=json.loads(open('$O/${tag}_$i.json').read().strip().splitlines()[-1]); print('$tag', $i, b['value'], b['ms_per_step'], b['round']['host_first_steps_us'])"
  done
done
