#!/bin/bash
# Round 3, session 2: the driver's 20-step line with Python's GC held off in the timed region,
# three runs, beside a 400-step line.
mkdir -p gpurun_out/m20
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/m20/b20_$r.json 2> gpurun_out/m20/b20_$r.err || exit 1
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/m20/b400.json 2> gpurun_out/m20/b400.err || exit 1
for f in b20_1 b20_2 b20_3 b400; do
  python3 -c "import json; b=json.loads(open('gpurun_out/m20/$f.json').read().strip().splitlines()[-1]); print('$f', b['value'], b['ms_per_step'], b['round']['host_first_steps_us'], b['roofline']['avg_launch_us'])"
done
