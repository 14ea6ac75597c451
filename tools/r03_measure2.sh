#!/bin/bash
# Round 3: sorted rounds and the futex-parking combiner -- parity first, then measurements.
mkdir -p gpurun_out/m2
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_combiner.py \
    -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/m2/tests.log 2>&1
rc=$?; tail -5 gpurun_out/m2/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./microbench/combiner_bench 2 > gpurun_out/m2/combiner.txt 2>&1; rc=$?
cat gpurun_out/m2/combiner.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 tools/sweep.py \
  'b1||' 'b1_sorted||--knob SORT_MIN=1' \
  'n8_stamp||--ops-per-gpu 1700000 --write-ratio 47 --knob SORT_MIN=0' \
  'n8_sorted||--ops-per-gpu 1700000 --write-ratio 47 --knob SORT_MIN=1' \
  'w50_stamp||--write-ratio 50 --knob SORT_MIN=0' 'w50_sorted||--write-ratio 50 --knob SORT_MIN=1' \
  'w100_stamp||--write-ratio 100 --knob SORT_MIN=0' 'w100_sorted||--write-ratio 100 --knob SORT_MIN=1' \
  'c2_stamp||--ops-per-gpu 4500000 --write-ratio 89 --knob SORT_MIN=0 --pool 16' \
  'c2_sorted||--ops-per-gpu 4500000 --write-ratio 89 --knob SORT_MIN=1 --pool 16' \
  > gpurun_out/m2/sweep.txt 2>&1
rc=$?; cat gpurun_out/m2/sweep.txt; exit $rc
