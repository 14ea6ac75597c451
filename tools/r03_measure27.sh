#!/bin/bash
# Round 3, session 2 final records (after the synthetic pass-size change and its race fix): full GPU suite + smoke, the driver's bench command and the default
# line, stack / synthetic lines, rocprof kernel traces + PMC traffic passes (tools/profile.sh).
mkdir -p gpurun_out/m27
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/m27/tests.log 2>&1
rc=$?; tail -3 gpurun_out/m27/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/m27/smoke.txt 2>&1 || { cat gpurun_out/m27/smoke.txt; exit 1; }
tail -1 gpurun_out/m27/smoke.txt
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/m27/driver.json 2> gpurun_out/m27/driver.err || exit 1
timeout -k 10 240 python3 bench.py > gpurun_out/m27/default.json 2> gpurun_out/m27/default.err || exit 1
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 200 $B --workload stack > gpurun_out/m27/stack.json 2> gpurun_out/m27/stack.err || exit 1
timeout -k 10 200 $B --workload synthetic > gpurun_out/m27/synthetic.json 2> gpurun_out/m27/synthetic.err || exit 1
for f in driver default stack synthetic; do
  python3 -c "import json; b=json.loads(open('gpurun_out/m27/$f.json').read().strip().splitlines()[-1]); r=b['roofline']; print('$f', b['value'], b['ms_per_step'], r.get('avg_launch_us'), r['frac'])"
done
P="--steps 200"
bash tools/profile.sh r03f_synth --workload synthetic $P || exit 1
echo profiles done
