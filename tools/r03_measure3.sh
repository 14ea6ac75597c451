#!/bin/bash
# Round 3: full GPU suite, then the stack / synthetic / headline bench lines and a kernel trace
# of the stack and B1 runs (each step under its own limit; stops at the first failure).
mkdir -p gpurun_out/m3
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/m3/tests.log 2>&1
rc=$?; tail -4 gpurun_out/m3/tests.log; [ $rc -ne 0 ] && exit $rc
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 200 $B --workload stack > gpurun_out/m3/stack.json 2> gpurun_out/m3/stack.err || exit 1
timeout -k 10 200 $B --workload synthetic > gpurun_out/m3/synth.json 2> gpurun_out/m3/synth.err || exit 1
timeout -k 10 200 $B --steps 20 --warmup 5 > gpurun_out/m3/b20.json 2> gpurun_out/m3/b20.err || exit 1
timeout -k 10 200 $B > gpurun_out/m3/b400.json 2> gpurun_out/m3/b400.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/m3/kt_stack -o run -- \
    python3 bench.py --no-cpu-baseline --workload stack --steps 200 > gpurun_out/m3/kt_stack.json 2>/dev/null || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/m3/kt_b1 -o run -- \
    python3 bench.py --no-cpu-baseline --no-prev-variant --steps 200 > gpurun_out/m3/kt_b1.json 2>/dev/null || exit 1
for f in stack synth b20 b400; do
  python3 -c "import json; b=json.loads(open('gpurun_out/m3/$f.json').read().strip().splitlines()[-1]); r=b['roofline']; print('$f', b['value'], b['ms_per_step'], r['avg_launch_us'], r['frac'])"
done
