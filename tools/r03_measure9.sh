#!/bin/bash
# Round 3, session 2: synthetic 4-B seen values -- parity first, then the bench line and phases.
mkdir -p gpurun_out/m9
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_synthetic.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/m9/tests.log 2>&1
rc=$?; tail -4 gpurun_out/m9/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/sweep.py 'sy_v32||--workload synthetic' 'sy_v32b||--workload synthetic' > gpurun_out/m9/sy.txt 2>&1
rc=$?; cat gpurun_out/m9/sy.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 microbench/synth_phases.py > gpurun_out/m9/synth_phases.txt 2>&1; rc=$?
head -16 gpurun_out/m9/synth_phases.txt; exit $rc
