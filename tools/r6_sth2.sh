#!/bin/bash
# stack, same box: round-5 kernel (lib) vs the wave-0 hand-off build (lib_t9, EXP 0 = hand-off, 0x80 = own stores)
set -o pipefail
O=gpurun_out/sth2; mkdir -p $O
V=node-replication_amd/lib_t9/libnrgpu.so
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline > $O/b_lib_$i.json 2> $O/b_lib_$i.err || exit $?
  NRGPU_LIB=$V timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline > $O/b_h_$i.json 2> $O/b_h_$i.err || exit $?
  NRGPU_LIB=$V timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline --knob EXP=0x80 > $O/b_o_$i.json 2> $O/b_o_$i.err || exit $?
done
BB=8 timeout -k 10 200 python -u microbench/stack_phases.py > $O/ph8_lib.txt 2>&1
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"; done
cat $O/ph8_lib.txt
