#!/bin/bash
# round-6 validation after the synthetic response streaming: the GPU suite, smoke(), the bench
# lines, then the synthetic's kernel trace + PMC traffic
set -o pipefail
bash tools/r6_final.sh && bash tools/profile.sh sy6f --workload synthetic --steps 100 > gpurun_out/prof_sy6f.log 2>&1
rc=$?
for f in gpurun_out/final/bench_*.json; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); print('$f', d['value'], round(d['ms_per_step']*1e3,3), d['roofline'].get('frac'))"; done
exit $rc
