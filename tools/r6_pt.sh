#!/bin/bash
# partitioned N=1: HIP API + kernel trace of the bench (where the host's ~57 us per call go)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pt; mkdir -p $O
timeout -k 10 200 python bench.py --partitioned --no-cpu-baseline --no-prev-variant --steps 50 --warmup 5 > $O/b.json 2> $O/b.err &&
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -f csv -d $O/trace -o run -- python3 bench.py --partitioned --no-cpu-baseline --no-prev-variant --steps 50 --warmup 5 --no-kernel-timing > $O/bt.json 2> $O/bt.err
rc=$?; python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['round']['host_enqueue_us'])"; exit $rc
