#!/bin/bash
# Where does a short timed region lose time? Runs bench.py at the
# driver's --steps 20 --warmup 5 with and without event bracketing, the 400-step line beside
# them, and a kernel + HIP-API trace of the 20-step run (same clock domain for host calls and
# kernels). Usage (through gpurun, from the repo root): tools/t20.sh TAG
set -o pipefail
TAG=${1:-t20}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-prev-variant"
timeout -k 10 120 $B --steps 20 --warmup 5 > $OUT/s20.json 2> $OUT/s20.err &&
timeout -k 10 120 $B --steps 20 --warmup 5 --no-kernel-timing > $OUT/s20_nt.json 2> $OUT/s20_nt.err &&
timeout -k 10 120 $B --steps 400 --warmup 40 --no-kernel-timing > $OUT/s400_nt.json 2> $OUT/s400_nt.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --hip-trace -f csv -d $OUT/trace -o run -- \
    python3 bench.py --no-cpu-baseline --no-prev-variant --steps 20 --warmup 5 --no-kernel-timing \
    > $OUT/trace.json 2> $OUT/trace.err
rc=$?
for f in s20 s20_nt s400_nt trace; do
  python3 -c "import json,sys; b=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', b['value'], b['ms_per_step'])" 2>/dev/null
done
exit $rc
