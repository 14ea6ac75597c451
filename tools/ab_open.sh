#!/bin/bash
# A/B of the timed region's opening (bench.py --opening sync|spin) at the driver's 20 steps:
# alternating runs on one box. Usage (through gpurun): tools/ab_open.sh TAG [runs]
set -o pipefail
TAG=${1:-abopen}; N=${2:-5}
OUT=gpurun_out/$TAG; mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-prev-variant --steps 20 --warmup 5"
for i in $(seq 1 $N); do
  for m in sync spin; do
    timeout -k 10 120 $B --opening $m > $OUT/${m}_$i.json 2> $OUT/${m}_$i.err || exit $?
    python3 -c "import json; b=json.loads(open('$OUT/${m}_$i.json').read().strip().splitlines()[-1]); print('$m', $i, b['value'], b['ms_per_step'], b['round']['host_first_steps_us'], b['roofline']['avg_launch_us'])"
  done
done
