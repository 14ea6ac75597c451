#!/bin/bash
# stack diagnostic: tile-pass stores skipped (results wrong): EXP bit 8 = log copy, bit 9 = responses
set -o pipefail
O=gpurun_out/stdiag; mkdir -p $O
V=node-replication_amd/lib_t9/libnrgpu.so
for x in 0 0x100 0x200 0x300; do
  NRGPU_LIB=$V EXP=$((2 | x)) BB=8 timeout -k 10 200 python -u microbench/stack_phases.py > $O/ph_$x.txt 2>&1 || exit $?
  NRGPU_LIB=$V timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline --knob EXP=$x > $O/b_$x.json 2> $O/b_$x.err || exit $?
done
for x in 0 0x100 0x200 0x300; do echo "== $x"; python3 -c "import json; d=json.loads([l for l in open('$O/b_$x.json') if l.startswith('{')][-1]); print(d['ms_per_step']*1e3, d['roofline']['avg_launch_us'])"; grep -E "publish|last tile end|loads " $O/ph_$x.txt; done
