#!/bin/bash
# Round 3 session 2: a few spinning clients (spin cap 1/2/4) at 64/128/256 client threads x 32 ops,
# against the default (parked clients), interleaved (microbench/combiner_bench, 2 s per case).
mkdir -p gpurun_out/m44
timeout -k 10 400 ./microbench/combiner_bench 2 64 32 0 -1 0  64 32 0 1 0  64 32 0 2 0  64 32 0 4 0 \
   64 32 0 -1 0  64 32 0 2 0  128 32 0 -1 0  128 32 0 2 0  256 32 0 -1 0  256 32 0 2 0 \
   16 32 0 -1 0  16 32 0 2 0  64 32 1 -1 0  64 32 1 2 0  256 32 1 -1 0  256 32 1 2 0 \
   > gpurun_out/m44/combiner.txt 2>&1; rc=$?
grep Mops gpurun_out/m44/combiner.txt; exit $rc
