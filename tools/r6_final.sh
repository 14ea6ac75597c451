#!/bin/bash
# round-6 validation: the GPU suite (with durations), smoke(), and the bench lines
set -o pipefail
O=gpurun_out/final; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --durations=15 --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err &&
timeout -k 10 300 python -u bench.py --workload stack > $O/bench_stack.json 2> $O/bench_stack.err &&
timeout -k 10 300 python -u bench.py --workload synthetic > $O/bench_synth.json 2> $O/bench_synth.err &&
timeout -k 10 300 python -u bench.py --partitioned > $O/bench_part.json 2> $O/bench_part.err
rc=$?; tail -20 $O/tests.log; exit $rc
