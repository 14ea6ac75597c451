#!/bin/bash
# Round 3, one box: the full GPU suite, then the combiner bench, the write-round sweep (sorted vs
# stamp), the stack / synthetic / headline bench lines and kernel traces. Each step has its own
# limit; the script stops at the first failure.
mkdir -p gpurun_out/m4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_combiner.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/m4/tests.log 2>&1
rc=$?; tail -4 gpurun_out/m4/tests.log; [ $rc -ne 0 ] && exit $rc
B="python3 bench.py --no-cpu-baseline"
for w in stack synthetic; do
  timeout -k 10 200 $B --workload $w > gpurun_out/m4/$w.json 2> gpurun_out/m4/$w.err || exit 1
done
timeout -k 10 200 $B --steps 20 --warmup 5 > gpurun_out/m4/b20.json 2> gpurun_out/m4/b20.err || exit 1
timeout -k 10 200 $B > gpurun_out/m4/b400.json 2> gpurun_out/m4/b400.err || exit 1
for f in stack synthetic b20 b400; do
  python3 -c "import json; b=json.loads(open('gpurun_out/m4/$f.json').read().strip().splitlines()[-1]); r=b['roofline']; print('$f', b['value'], b['ms_per_step'], r['avg_launch_us'], r['frac'])"
done
timeout -k 10 900 python3 tools/sweep.py \
  'n8_stamp||--ops-per-gpu 1700000 --write-ratio 47 --knob SORT_MIN=0' \
  'n8_sorted||--ops-per-gpu 1700000 --write-ratio 47 --knob SORT_MIN=1' \
  'w50_stamp||--write-ratio 50 --knob SORT_MIN=0' 'w50_sorted||--write-ratio 50 --knob SORT_MIN=1' \
  'c2_stamp||--ops-per-gpu 4500000 --write-ratio 89 --knob SORT_MIN=0 --pool 16' \
  'c2_sorted||--ops-per-gpu 4500000 --write-ratio 89 --knob SORT_MIN=1 --pool 16' \
  'b1_sorted||--knob SORT_MIN=1' 'b1_rpt2||' 'b1_rpt1|NRGPU_LIB=node-replication_amd/lib/libnrgpu_rpt1.so|' \
  'r100_rpt2||--write-ratio 0' 'r100_rpt1|NRGPU_LIB=node-replication_amd/lib/libnrgpu_rpt1.so|--write-ratio 0' \
  'sy_xcd||--workload synthetic' 'sy_noxcd|NRGPU_LIB=node-replication_amd/lib/libnrgpu_noremap.so|--workload synthetic' \
  > gpurun_out/m4/sweep.txt 2>&1
rc=$?; cat gpurun_out/m4/sweep.txt; [ $rc -ne 0 ] && exit $rc
P="--steps 200"
bash tools/profile.sh r03_stack --workload stack $P && bash tools/profile.sh r03_synth --workload synthetic $P || exit 1
C="--steps 50 --ops-per-gpu 4500000 --write-ratio 89 --pool 8"
bash tools/profile.sh r03_c2_sorted $C && bash tools/profile.sh r03_c2_stamp $C --knob SORT_MIN=0 || exit 1
timeout -k 10 150 ./microbench/combiner_bench 2 > gpurun_out/m4/combiner.txt 2>&1; rc=$?
cat gpurun_out/m4/combiner.txt; [ $rc -ne 0 ] && exit $rc
echo done
