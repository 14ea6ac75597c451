#!/bin/bash
# Round 3, session 2: combiner CPU use per client (user/system) at 64-256 threads.
mkdir -p gpurun_out/m14
timeout -k 10 200 ./microbench/combiner_bench 2 64 32 0 -1 0  128 32 0 -1 0  192 32 0 -1 0  256 32 0 -1 0 > gpurun_out/m14/combiner.txt 2>&1; rc=$?
cat gpurun_out/m14/combiner.txt; exit $rc
