#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pt3; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 bench.py --partitioned --no-cpu-baseline --no-prev-variant --steps 50 --warmup 5 --no-kernel-timing > $O/bt.json 2> $O/bt.err
