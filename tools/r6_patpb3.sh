#!/bin/bash
# partition-round apply width on skewed streams (default warmup: the skew sample has switched them to partition rounds)
set -o pipefail
O=gpurun_out/patpb3; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-prev-variant --steps 200"
for i in 1 2; do for t in 0 512 256; do
  timeout -k 10 200 $B --write-ratio 50 --dist zipf --knob PA_TPB=$t > $O/z50_${t}_$i.json 2> $O/z50_${t}_$i.err || exit $?
  timeout -k 10 200 $B --write-ratio 10 --dist zipf --knob PA_TPB=$t > $O/z10_${t}_$i.json 2> $O/z10_${t}_$i.err || exit $?
  timeout -k 10 200 $B --write-ratio 50 --dist zipf --scramble --knob PA_TPB=$t > $O/z50s_${t}_$i.json 2> $O/z50s_${t}_$i.err || exit $?
done; done
for f in $O/*.json; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step']*1e3, d['roofline']['avg_launch_us'])"; done
