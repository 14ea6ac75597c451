#!/bin/bash
# Round 3, session 2: synthetic bucket pass in sweeps for WriteOnly-free chunks -- parity, bench, phases.
mkdir -p gpurun_out/m11
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_synthetic.py tests/test_gpu_golden.py tests/test_gpu_group_multi.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/m11/tests.log 2>&1
rc=$?; tail -3 gpurun_out/m11/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/sweep.py 'sy_sweeps||--workload synthetic' 'sy_sweeps_b||--workload synthetic' > gpurun_out/m11/sy.txt 2>&1
rc=$?; cat gpurun_out/m11/sy.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 microbench/synth_phases.py > gpurun_out/m11/synth_phases.txt 2>&1; rc=$?
head -20 gpurun_out/m11/synth_phases.txt; [ $rc -ne 0 ] && exit $rc
# combiner: waiting policy (spinning clients) and rounds in flight
timeout -k 10 200 ./microbench/combiner_bench 2 16 32 0 -1 0  16 32 0 0 0  64 32 0 -1 0  64 32 0 4 0  64 32 0 0 0 \
    64 32 0 0 3  64 32 0 4 3  256 32 0 0 0  256 32 0 4 0 > gpurun_out/m11/combiner.txt 2>&1; rc=$?
cat gpurun_out/m11/combiner.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-prev-variant --steps 20 --warmup 5 > gpurun_out/m11/b20.json 2> gpurun_out/m11/b20.err || exit 1
tail -1 gpurun_out/m11/b20.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/m11/kt_comb -o run -- ./microbench/combiner_bench 1 16 32 0 -1 0 > gpurun_out/m11/kt_comb.txt 2>&1 || exit 1
T=$(find gpurun_out/m11/kt_comb -name '*kernel_stats.csv' | head -1); head -8 $T | cut -d, -f1-8
