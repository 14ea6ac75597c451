#!/bin/bash
# fused synthetic round: phases, role-order A/B, kernel trace + PMC traffic
set -o pipefail
O=gpurun_out/sy2; mkdir -p $O
timeout -k 10 120 python microbench/synth_phases.py > $O/phases.txt 2>&1 &&
for i in 1 2; do for x in 0 0x1000 0x2000; do
  timeout -k 10 200 python bench.py --workload synthetic --no-cpu-baseline --knob EXP=$x > $O/b_${x}_$i.json 2> $O/b_${x}_$i.err || exit $?
done; done &&
bash tools/profile.sh r6_synth_fused --workload synthetic --steps 100 > $O/prof.log 2>&1
rc=$?; head -30 $O/phases.txt
for f in $O/b_*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
exit $rc
