#!/bin/bash
# Bench variants on the GPU box (each a separate bench.py process): B1 headline, 50% writes,
# Zipf (adjacent and scrambled hot keys), stack, and 2-rank gloo rehearsals of the N>1 path on
# the box's one GPU. Results: gpurun_out/variants/<name>.json
set -o pipefail
mkdir -p gpurun_out/variants
S=${STEPS:-200}
run() {
    name=$1; shift
    if timeout -k 10 240 "$@" > gpurun_out/variants/$name.json 2> gpurun_out/variants/$name.err; then
        echo "ok $name"
    else
        echo "FAILED $name"; tail -5 gpurun_out/variants/$name.err; return 1
    fi
}
run b1 python bench.py --steps $S --no-cpu-baseline &&
run b1_w50 python bench.py --steps $S --write-ratio 50 --no-cpu-baseline &&
run zipf_w50 python bench.py --steps $S --dist zipf --write-ratio 50 --no-cpu-baseline &&
run zipf_w50_scr python bench.py --steps $S --dist zipf --scramble --write-ratio 50 --no-cpu-baseline &&
run stack python bench.py --workload stack --steps $S &&
run g2_gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29513 bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo --share-gpu --no-cpu-baseline \
    --no-prev-variant &&
run g2_gloo_stack python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29514 bench.py --workload stack --gpus 2 --steps 10 --warmup 2 --backend gloo --share-gpu \
    --no-cpu-baseline
