#!/bin/bash
# combiner batch round trip: doorbell + records in host memory vs device memory written by the host
set -o pipefail
O=gpurun_out/door2; mkdir -p $O
for m in 1 0; do for sz in "4608 4608" "1024 1024" "16384 16384"; do
  timeout -k 10 60 ./microbench/door_rt $m $sz 4000 >> $O/rt.txt 2>&1; rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ] && [ $rc -ne 4 ]; then echo "rc=$rc" >> $O/rt.txt; exit $rc; fi
done; done
cat $O/rt.txt
