#!/bin/bash
# full GPU suite, then fresh r06 kernel traces + PMC traffic for the B1 and stack rounds
set -o pipefail
O=gpurun_out/val; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/t.log 2>&1 &&
bash tools/profile.sh r6_b1 --steps 100 > $O/p1.log 2>&1 &&
bash tools/profile.sh r6_stack --workload stack --steps 100 > $O/p2.log 2>&1
rc=$?; tail -3 $O/t.log; exit $rc
