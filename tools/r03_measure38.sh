#!/bin/bash
# Round 3, session 2 final records: full GPU suite + smoke, the driver's command and the default
# line, stack / synthetic lines, B1 kernel trace + PMC traffic (tools/profile.sh), combiner bench.
mkdir -p gpurun_out/m38
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/m38/tests.log 2>&1
rc=$?; tail -3 gpurun_out/m38/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/m38/smoke.txt 2>&1 || { cat gpurun_out/m38/smoke.txt; exit 1; }
tail -1 gpurun_out/m38/smoke.txt
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/m38/driver.json 2> gpurun_out/m38/driver.err || exit 1
timeout -k 10 240 python3 bench.py > gpurun_out/m38/default.json 2> gpurun_out/m38/default.err || exit 1
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 200 $B --workload stack > gpurun_out/m38/stack.json 2> gpurun_out/m38/stack.err || exit 1
timeout -k 10 200 $B --workload synthetic > gpurun_out/m38/synthetic.json 2> gpurun_out/m38/synthetic.err || exit 1
for f in driver default stack synthetic; do
  python3 -c "import json; b=json.loads(open('gpurun_out/m38/$f.json').read().strip().splitlines()[-1]); r=b['roofline']; print('$f', b['value'], b['ms_per_step'], r.get('avg_launch_us'), r['frac'])"
done
bash tools/profile.sh r03f_b1 --steps 200 --no-prev-variant || exit 1
timeout -k 10 200 ./microbench/combiner_bench 2 > gpurun_out/m38/combiner.txt 2>&1; rc=$?
grep Mops gpurun_out/m38/combiner.txt; exit $rc
