#!/bin/bash
# round-6 validation after the store-policy changes (stack responses/finish, B1 apply, partition
# apply): the GPU suite, smoke(), the bench lines, then B1's and the stack's kernel trace + PMC traffic
set -o pipefail
bash tools/r6_final.sh && bash tools/profile.sh b1f > gpurun_out/prof_b1f.log 2>&1 &&
bash tools/profile.sh st6d --workload stack --steps 100 > gpurun_out/prof_st6d.log 2>&1
rc=$?; tail -2 gpurun_out/prof_b1f.log gpurun_out/prof_st6d.log
for f in gpurun_out/final/bench_*.json; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); print('$f', d['value'], round(d['ms_per_step']*1e3,3), d['roofline'].get('frac'))"; done
exit $rc
