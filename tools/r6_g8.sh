#!/bin/bash
# launcher rehearsal at 8 ranks on the box's one GPU (gloo all-gather of the write segments)
set -o pipefail
O=gpurun_out/g8; mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 8 --backend gloo --share-gpu --steps 20 --warmup 5 --no-cpu-baseline > $O/b8.json 2> $O/b8.err
rc=$?; tail -5 $O/b8.err; tail -1 $O/b8.json | cut -c1-600; exit $rc
