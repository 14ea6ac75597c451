#!/bin/bash
# Round-3 measurements: native combiner throughput, and the driver's 20-step bench line beside
# the 400-step line (timed region without events; roofline region after it).
mkdir -p gpurun_out/m1
export TMPDIR=/tmp
timeout -k 10 120 ./microbench/combiner_bench 2 > gpurun_out/m1/combiner.txt 2>&1 || { cat gpurun_out/m1/combiner.txt; exit 1; }
cat gpurun_out/m1/combiner.txt
for s in 20 400; do
  w=$([ $s = 20 ] && echo 5 || echo 40)
  timeout -k 10 200 python3 bench.py --steps $s --warmup $w --no-cpu-baseline > gpurun_out/m1/b$s.json 2> gpurun_out/m1/b$s.err || exit 1
  python3 -c "import json; b=json.loads(open('gpurun_out/m1/b$s.json').read().strip().splitlines()[-1]); print('steps $s', b['value'], b['ms_per_step'], b['roofline']['avg_launch_us'], b['roofline']['frac'], b.get('variants'))"
done
