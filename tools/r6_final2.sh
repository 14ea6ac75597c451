#!/bin/bash
# round-6 validation after the stack store-policy changes: the GPU suite, smoke(), the bench
# lines, then the stack's kernel trace + PMC traffic (tools/profile.sh)
set -o pipefail
bash tools/r6_final.sh && bash tools/profile.sh st6c --workload stack --steps 100 > gpurun_out/prof_st6c.log 2>&1
rc=$?; tail -3 gpurun_out/prof_st6c.log
for f in gpurun_out/final/bench_*.json; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); print('$f', d['value'], round(d['ms_per_step']*1e3,3), d['roofline'].get('frac'))"; done
exit $rc
