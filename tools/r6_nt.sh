#!/bin/bash
# Single-word streamed stores made real (st_out): hashmap / synthetic / stack suites on the new
# build, then one-box A/B against the previous build (lib_prev): B1 (default, and with the
# stamp-round reads streamed: EXP bit 17), N = 8 and configs[2] per-GPU partition rounds,
# synthetic (default, touch records / seen values / responses streamed: EXP bits 7 / 8 / 9)
set -o pipefail
O=gpurun_out/nt; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hashmap.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_synthetic.py tests/test_gpu_stack.py tests/test_gpu_partition.py -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
B="python bench.py --no-cpu-baseline --no-prev-variant"
run() { # name lib args...
  n=$1; l=$2; shift 2
  NRGPU_LIB=node-replication_amd/$l/libnrgpu.so timeout -k 10 200 $B "$@" > $O/$n.json 2> $O/$n.err || { echo "FAILED $n"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads([x for x in open('$O/$n.json') if x.startswith('{')][-1]); print('%-14s' % '$n', d['value'], round(d['ms_per_step']*1e3,3), d['roofline']['avg_launch_us'])"
}
for i in 1 2; do
  run b1_prev_$i lib_prev
  run b1_new_$i lib
  run b1_ntr_$i lib --knob EXP=0x20000
done
for i in 1 2; do
  run n8_prev_$i lib_prev --ops-per-gpu 1700000 --write-ratio 47
  run n8_new_$i lib --ops-per-gpu 1700000 --write-ratio 47
done
run c2_prev lib_prev --steps 60 --ops-per-gpu 4500000 --write-ratio 89
run c2_new lib --steps 60 --ops-per-gpu 4500000 --write-ratio 89
for i in 1 2; do
  run sy_prev_$i lib_prev --workload synthetic
  run sy_new_$i lib --workload synthetic
  run sy_e_$i lib --workload synthetic --knob EXP=0x80
  run sy_v_$i lib --workload synthetic --knob EXP=0x100
  run sy_r_$i lib --workload synthetic --knob EXP=0x200
done
