#!/bin/bash
# partition-round apply width at the emulated N = 4 / 8 per-GPU rounds (NRG_KNOB_PA_TPB; 0 = default 1024)
set -o pipefail
O=gpurun_out/patpb; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-prev-variant --steps 200 --warmup 20"
for i in 1 2; do for t in 0 512 256; do
  timeout -k 10 200 $B --ops-per-gpu 1700000 --write-ratio 47 --knob PA_TPB=$t > $O/n8_${t}_$i.json 2> $O/n8_${t}_$i.err || exit $?
  timeout -k 10 200 $B --ops-per-gpu 1300000 --write-ratio 31 --knob PA_TPB=$t > $O/n4_${t}_$i.json 2> $O/n4_${t}_$i.err || exit $?
done; done
for f in $O/*.json; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step']*1e3, d['roofline']['avg_launch_us'])"; done
