#!/bin/bash
# End-of-round validation on the GPU box (through gpurun, from the repo root): the GPU test suite,
# smoke(), the default bench line, the stack bench line, and a PMC profile of the stack kernel.
# Outputs: gpurun_out/final/, gpurun_out/prof_r04f_stack/ (tools/prof_summary.py -> profiles/).
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/final/t.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err &&
timeout -k 10 300 python bench.py --workload stack > gpurun_out/final/bench_stack.json 2> gpurun_out/final/bench_stack.err &&
bash tools/profile.sh r04f_stack --workload stack --steps 100 > gpurun_out/final/p.log 2>&1
