#!/bin/bash
# Round 3 session 2: native combiner policy at the current build -- rounds in flight (depth) and
# client spinning at 64 and 256 client threads x 32 ops (microbench/combiner_bench, 2 s per case).
mkdir -p gpurun_out/m43
timeout -k 10 300 ./microbench/combiner_bench 2 64 32 0 -1 0  64 32 0 0 1  64 32 0 0 3  64 32 0 0 4 \
   64 32 0 2 0  64 32 0 8 0  64 32 0 4 3  64 32 0 -1 0  128 32 0 0 3  256 32 0 0 3  256 32 0 -1 0 \
   > gpurun_out/m43/combiner.txt 2>&1; rc=$?
grep Mops gpurun_out/m43/combiner.txt; exit $rc
