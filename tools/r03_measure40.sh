#!/bin/bash
# Round 3 session 2: HIP runtime + kernel trace of the driver's 20-step B1 line (two runs), to
# place the first-steps host stalls (inside a HIP API call or between calls).
export TMPDIR=/tmp
for k in 1 2; do
  OUT=gpurun_out/rt20_$k; mkdir -p $OUT
  timeout -k 10 240 rocprofv3 --runtime-trace --kernel-trace -f csv -d $OUT -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-prev-variant > $OUT/bench.json 2> $OUT/bench.err || exit 1
  tail -1 $OUT/bench.json | cut -c1-200
done
find gpurun_out/rt20_1 -name '*.csv' | xargs ls -la
