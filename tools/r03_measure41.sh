#!/bin/bash
# Round 3 session 2 final check at HEAD: full GPU suite, smoke, the driver's command, synthetic line.
mkdir -p gpurun_out/m41
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/m41/tests.log 2>&1
rc=$?; tail -2 gpurun_out/m41/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/m41/smoke.txt 2>&1 || { cat gpurun_out/m41/smoke.txt; exit 1; }
tail -1 gpurun_out/m41/smoke.txt
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/m41/driver.json 2> gpurun_out/m41/driver.err || exit 1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload synthetic > gpurun_out/m41/synthetic.json 2> gpurun_out/m41/synthetic.err || exit 1
for f in driver synthetic; do
  python3 -c "import json; b=json.loads(open('gpurun_out/m41/$f.json').read().strip().splitlines()[-1]); r=b['roofline']; print('$f', b['value'], b['ms_per_step'], r.get('avg_launch_us'), r['frac'])"
done
