#!/bin/bash
# synthetic: HEAD (lib) vs a variant build (lib_t9), same box
set -o pipefail
O=gpurun_out/${SYV_OUT:-syv}; mkdir -p $O
V=node-replication_amd/lib_t9/libnrgpu.so
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --workload synthetic --no-cpu-baseline > $O/b_lib_$i.json 2> $O/b_lib_$i.err || exit $?
  NRGPU_LIB=$V timeout -k 10 200 python bench.py --workload synthetic --no-cpu-baseline > $O/b_v_$i.json 2> $O/b_v_$i.err || exit $?
done
for f in $O/b*.json; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['ms_per_step']*1e3, d['roofline']['avg_launch_us'])"; done
