#!/bin/bash
# partition-round apply width on the other partition-round workloads (NRG_KNOB_PA_TPB; 0 = default 1024)
set -o pipefail
O=gpurun_out/patpb2; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-prev-variant --warmup 10"
for i in 1 2; do for t in 0 512; do
  timeout -k 10 200 $B --steps 60 --ops-per-gpu 4500000 --write-ratio 89 --knob PA_TPB=$t > $O/c2_${t}_$i.json 2> $O/c2_${t}_$i.err || exit $?
  timeout -k 10 200 $B --steps 200 --write-ratio 100 --knob PA_TPB=$t > $O/w100_${t}_$i.json 2> $O/w100_${t}_$i.err || exit $?
  timeout -k 10 200 $B --steps 200 --write-ratio 50 --dist zipf --knob PA_TPB=$t > $O/z50_${t}_$i.json 2> $O/z50_${t}_$i.err || exit $?
  timeout -k 10 200 $B --steps 200 --write-ratio 50 --knob PA_TPB=$t > $O/w50_${t}_$i.json 2> $O/w50_${t}_$i.err || exit $?
done; done
for f in $O/*.json; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step']*1e3, d['roofline']['avg_launch_us'])"; done
