#!/bin/bash
# stack look-back timeline: publish / build / wait marks (diagnostic build marks, EXP 2)
set -o pipefail
O=gpurun_out/stlb; mkdir -p $O
timeout -k 10 200 python -u microbench/stack_phases.py > $O/ph1.txt 2>&1 &&
BB=8 timeout -k 10 200 python -u microbench/stack_phases.py > $O/ph8.txt 2>&1
rc=$?; cat $O/ph1.txt $O/ph8.txt; exit $rc
