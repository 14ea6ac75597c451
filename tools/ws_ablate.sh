#!/bin/bash
# Write-set round ablations (NRG_KNOB_EXP >> 20; results wrong, timing only) on the B1 bench.
TAG=${1:-wsab}
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-prev-variant "$@" > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.err || { tail -5 gpurun_out/${TAG}_b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_b.json')); print('$*'.ljust(50), d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
}
run --knob WS=1
run --knob WS=0
run --knob WS_EPOS=100
for x in 1 2 4 8 16 32 3 6 9; do run --knob EXP=$((x << 20)); done
