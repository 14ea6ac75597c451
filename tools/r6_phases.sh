#!/bin/bash
set -o pipefail
O=gpurun_out/ph; mkdir -p $O
BB=8 timeout -k 10 120 python microbench/stack_phases.py > $O/stack.txt 2>&1 &&
timeout -k 10 120 python microbench/synth_phases.py > $O/synth.txt 2>&1
rc=$?; cat $O/stack.txt | tail -14; tail -20 $O/synth.txt; exit $rc
