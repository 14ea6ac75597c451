#!/bin/bash
set -o pipefail
O=gpurun_out/stbm; mkdir -p $O
NRGPU_LIB=node-replication_amd/lib_t8/libnrgpu.so timeout -k 10 200 python -u microbench/stack_build_marks.py > $O/marks.txt 2>&1
rc=$?; cat $O/marks.txt; exit $rc
