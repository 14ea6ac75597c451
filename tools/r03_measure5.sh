#!/bin/bash
# Round 3, session 2 (container re-created; earlier measurements lost): the full GPU suite, the
# default bench line (as the driver runs it), the 20-step line, stack / synthetic lines and the
# combiner bench. Each step has its own limit; the script stops at the first failure.
O=gpurun_out/m5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python3 bench.py > $O/default.json 2> $O/default.err || exit 1
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 120 $B --steps 20 --warmup 5 > $O/b20.json 2> $O/b20.err || exit 1
for w in stack synthetic; do
  timeout -k 10 200 $B --workload $w > $O/$w.json 2> $O/$w.err || exit 1
done
for f in default b20 stack synthetic; do
  python3 -c "import json; b=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); r=b['roofline']; print('$f', b['value'], b['ms_per_step'], r.get('avg_launch_us'), r['frac'])"
done
timeout -k 10 150 ./microbench/combiner_bench 2 > $O/combiner.txt 2>&1; rc=$?
cat $O/combiner.txt; exit $rc
