#!/bin/bash
# Previous-value variant of B1 under several elector settings (run through gpurun).
# Usage: tools/prev_sweep.sh 'NAME|ENV=V ...' ...
for spec in "$@"; do
  name=${spec%%|*}; envs=${spec#*|}
  out=$(env $envs timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 100 --warmup 20 2>/dev/null | tail -1)
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); print('%-16s headline %9.1f  prev %9.1f Mops/s' % (sys.argv[1], d['value'], d['variants']['prev_value_responses_Mops']))" "$name" "$out" || { echo "$name failed"; exit 1; }
done
