#!/bin/bash
# Round 3, session 2: 2-rank rehearsal of bench.py's N > 1 path on the box's one GPU (gloo
# all-gather, both ranks on device 0), hashmap / stack / synthetic.
mkdir -p gpurun_out/m34
export TMPDIR=/tmp
R="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 300 $R --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo --share-gpu --no-cpu-baseline --no-prev-variant > gpurun_out/m34/g2_hm.json 2> gpurun_out/m34/g2_hm.err || { tail -5 gpurun_out/m34/g2_hm.err; exit 1; }
timeout -k 10 300 $R --master-port 29532 bench.py --workload stack --gpus 2 --steps 10 --warmup 2 --backend gloo --share-gpu --no-cpu-baseline > gpurun_out/m34/g2_st.json 2> gpurun_out/m34/g2_st.err || { tail -5 gpurun_out/m34/g2_st.err; exit 1; }
timeout -k 10 300 $R --master-port 29533 bench.py --workload synthetic --gpus 2 --steps 10 --warmup 2 --backend gloo --share-gpu --no-cpu-baseline > gpurun_out/m34/g2_sy.json 2> gpurun_out/m34/g2_sy.err || { tail -5 gpurun_out/m34/g2_sy.err; exit 1; }
for f in g2_hm g2_st g2_sy; do tail -1 gpurun_out/m34/$f.json | cut -c1-300; done
