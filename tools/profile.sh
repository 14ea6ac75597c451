#!/bin/bash
# GPU-box profiling recipe for bench.py (run through gpurun from the repo root):
#   1. kernel trace + stats of the bench command (per-kernel average durations)
#   2. separate PMC passes (FETCH_SIZE, then WRITE_SIZE) for HBM traffic per launch
#   3. with ATOMIC=1, a third pass counting atomics at the L2 (TCC_ATOMIC), atomics the L2 sends
#      on to memory (TCC_EA0_ATOMIC) and memory read requests (TCC_EA0_RDREQ)
# Results land in gpurun_out/prof_<tag>/; tools/prof_summary.py turns them into profiles/.
# Usage: tools/profile.sh TAG [bench.py args...]
set -eo pipefail
TAG=$1; shift
ARGS="$@"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- \
    python3 bench.py --no-cpu-baseline $ARGS > $OUT/bench_trace.json 2> $OUT/bench_trace.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- \
    python3 bench.py --no-cpu-baseline --no-prev-variant $ARGS > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- \
    python3 bench.py --no-cpu-baseline --no-prev-variant $ARGS > $OUT/bench_write.json 2> $OUT/bench_write.err
if [ "${ATOMIC:-0}" = 1 ]; then
  timeout -s KILL 120 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum -f csv -d $OUT/atomic -o run -- \
      python3 bench.py --no-cpu-baseline --no-prev-variant $ARGS > $OUT/bench_atomic.json 2> $OUT/bench_atomic.err
fi
echo "profile $TAG done"
