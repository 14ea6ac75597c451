#!/bin/bash
# Write-set rounds on the GPU box: hashmap parity suites, then B1 bench lines (ws vs stamp).
TAG=${1:-ws}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_hashmap.py tests/test_gpu_edge.py tests/test_gpu_golden.py tests/test_gpu_stream_order.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1
rc=$?; tail -15 gpurun_out/${TAG}_t.log
[ $rc -ne 0 ] && exit $rc
for k in "WS=1" "WS=0" "WS=1 --knob WS_EPOS=0" "WS=1 --knob WS_EPOS=60"; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-prev-variant --knob $k > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_b.json')); print('$k', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
