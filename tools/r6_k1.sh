#!/bin/bash
# stamp-round Puts per index thread (NRG_KNOB_K1; 0 = by round size: 1 for <= 2^18 Puts) at B1 and the N = 2 round
set -o pipefail
O=gpurun_out/k1; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-prev-variant --steps 400"
for i in 1 2; do for k in 0 2 4; do
  timeout -k 10 200 $B --knob K1=$k > $O/b1_${k}_$i.json 2> $O/b1_${k}_$i.err || exit $?
  timeout -k 10 200 $B --ops-per-gpu 1100000 --write-ratio 18 --knob K1=$k > $O/n2_${k}_$i.json 2> $O/n2_${k}_$i.err || exit $?
done; done
for f in $O/*.json; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step']*1e3, d['roofline']['avg_launch_us'])"; done
