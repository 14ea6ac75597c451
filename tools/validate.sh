#!/bin/bash
# End-of-round validation on the GPU box (through gpurun, from the repo root): the GPU test suite,
# smoke(), the default bench line, the stack, synthetic and partitioned bench lines.
# Outputs: gpurun_out/final/ (copied into profiles/r05_final/).
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/final/t.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench_20.json 2> gpurun_out/final/bench_20.err &&
timeout -k 10 300 python bench.py --workload stack > gpurun_out/final/bench_stack.json 2> gpurun_out/final/bench_stack.err &&
timeout -k 10 300 python bench.py --workload synthetic > gpurun_out/final/bench_synth.json 2> gpurun_out/final/bench_synth.err &&
timeout -k 10 300 python bench.py --partitioned --no-cpu-baseline > gpurun_out/final/bench_part.json 2> gpurun_out/final/bench_part.err
rc=$?; tail -3 gpurun_out/final/t.log; cat gpurun_out/final/smoke.log 2>/dev/null | tail -1
for f in gpurun_out/final/bench*.json; do echo "$f"; tail -1 "$f" | cut -c1-300; done
exit $rc
