#!/bin/bash
# Round 6 first GPU call: the bench launcher test, the loopback join/deadline tests, baseline lines.
set -o pipefail
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_launch.py tests/test_gpu_group_threads.py > $O/t.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-prev-variant > $O/b20.json 2> $O/b20.err &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-prev-variant > $O/b400.json 2> $O/b400.err &&
timeout -k 10 200 python bench.py --workload stack --no-cpu-baseline > $O/st.json 2> $O/st.err &&
timeout -k 10 200 python bench.py --workload synthetic --no-cpu-baseline > $O/sy.json 2> $O/sy.err
rc=$?; tail -3 $O/t.log
for f in $O/*.json; do echo $f; cut -c1-200 $f; done
exit $rc
