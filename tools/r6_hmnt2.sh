#!/bin/bash
# B1: streamed apply value stores (lib_ap) vs lib, 400-step and the driver's 20-step command
set -o pipefail
O=gpurun_out/hmnt2; mkdir -p $O
for i in 1 2 3; do
  for v in lib lib_ap; do
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-prev-variant > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read()); print('%-8s' % '$v', d['value'], round(d['ms_per_step']*1e3,3), d['roofline']['avg_launch_us'])"
    NRGPU_LIB=node-replication_amd/$v/libnrgpu.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/t_${v}_$i.json 2> $O/t_${v}_$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/t_${v}_$i.json').read()); print('%-8s' % '$v', '20-step', d['value'], round(d['ms_per_step']*1e3,3))"
  done
done
