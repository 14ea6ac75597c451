#!/bin/bash
# Round 3, session 2: synthetic ranking A/B (ballots vs LDS peer masks; XCD bucket order), then the
# write-round sweep (sorted rounds vs stamp rounds) that session 1's lost run measured.
mkdir -p gpurun_out/m7
export TMPDIR=/tmp
L=node-replication_amd/lib
timeout -k 10 600 python3 tools/sweep.py \
  'sy_ballot_xcd||--workload synthetic' 'sy_mask_xcd|NRGPU_LIB='$L'/libnrgpu_symask.so|--workload synthetic' \
  'sy_ballot_noxcd|NRGPU_LIB='$L'/libnrgpu_noremap.so|--workload synthetic' \
  'sy_ballot_xcd2||--workload synthetic' 'sy_mask_xcd2|NRGPU_LIB='$L'/libnrgpu_symask.so|--workload synthetic' \
  'b1||' 'stack||--workload stack' \
  > gpurun_out/m7/sy.txt 2>&1
rc=$?; cat gpurun_out/m7/sy.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 tools/sweep.py \
  'n8_stamp||--ops-per-gpu 1700000 --write-ratio 47 --knob SORT_MIN=0' \
  'n8_sorted||--ops-per-gpu 1700000 --write-ratio 47 --knob SORT_MIN=1' \
  'w50_stamp||--write-ratio 50 --knob SORT_MIN=0' 'w50_sorted||--write-ratio 50 --knob SORT_MIN=1' \
  'w100_stamp||--write-ratio 100 --knob SORT_MIN=0' 'w100_sorted||--write-ratio 100 --knob SORT_MIN=1' \
  'c2_stamp||--ops-per-gpu 4500000 --write-ratio 89 --knob SORT_MIN=0 --pool 16' \
  'c2_sorted||--ops-per-gpu 4500000 --write-ratio 89 --knob SORT_MIN=1 --pool 16' \
  'c2_default||--ops-per-gpu 4500000 --write-ratio 89 --pool 16' \
  'n8_default||--ops-per-gpu 1700000 --write-ratio 47' \
  > gpurun_out/m7/wr.txt 2>&1
rc=$?; cat gpurun_out/m7/wr.txt; exit $rc
