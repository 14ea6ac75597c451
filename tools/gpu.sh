#!/bin/bash
# Run a command on the GPU box through gpurun, retrying only when the box could not be
# prepared (transient; nothing ran). Usage: tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for a in $(seq 1 ${GPU_TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_last.txt 2>&1
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$st" = "transient" ] || [ $rc -eq 3 ]; then echo "[gpu.sh] transient (attempt $a), retrying in 100s" >&2; sleep 100; continue; fi
  tail -3 /tmp/gpurun_last.txt
  exit $rc
done
echo "[gpu.sh] giving up after transient failures" >&2; exit 3
