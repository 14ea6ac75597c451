#!/bin/bash
# Round 3, session 2: stamp rounds' apply from win/over epoch tags (no random stamp read per Put):
# parity (hashmap, full-size, group, log, golden), then the write sweep and B1.
mkdir -p gpurun_out/m17
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hashmap.py tests/test_gpu_fullsize.py tests/test_gpu_group_multi.py tests/test_gpu_log.py tests/test_gpu_golden.py tests/test_gpu_edge.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/m17/tests.log 2>&1
rc=$?; tail -3 gpurun_out/m17/tests.log; [ $rc -ne 0 ] && exit $rc
N8='--ops-per-gpu 1700000 --write-ratio 47'
C2='--ops-per-gpu 4500000 --write-ratio 89 --pool 16'
timeout -k 10 900 python3 tools/sweep.py "n8||$N8" "n8_noapply||$N8 --knob EXP=0x200000" "c2||$C2" "c2_noapply||$C2 --knob EXP=0x200000" \
  "w50||--write-ratio 50" "w100||--write-ratio 100" "b1||" "b1b||" > gpurun_out/m17/sweep.txt 2>&1
rc=$?; cat gpurun_out/m17/sweep.txt; exit $rc
