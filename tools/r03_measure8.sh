#!/bin/bash
# Round 3, session 2: synthetic phase stamps (partition, sums, bucket pass), the 20-step headline's
# launch timeline, and the combiner bench with 16 threads beside the default cases.
mkdir -p gpurun_out/m8
export TMPDIR=/tmp
timeout -k 10 120 python3 microbench/synth_phases.py > gpurun_out/m8/synth_phases.txt 2>&1 || { tail -20 gpurun_out/m8/synth_phases.txt; exit 1; }
cat gpurun_out/m8/synth_phases.txt
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d gpurun_out/m8/kt20 -o run -- \
    python3 bench.py --no-cpu-baseline --no-prev-variant --steps 20 --warmup 5 > gpurun_out/m8/b20.json 2> gpurun_out/m8/b20.err || exit 1
T=$(find gpurun_out/m8/kt20 -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py $T hm_round 0 40 > gpurun_out/m8/timeline20.txt; cat gpurun_out/m8/timeline20.txt
timeout -k 10 200 ./microbench/combiner_bench 2 16 32 0 64 32 0 256 32 0 > gpurun_out/m8/combiner.txt 2>&1; rc=$?
cat gpurun_out/m8/combiner.txt; exit $rc
