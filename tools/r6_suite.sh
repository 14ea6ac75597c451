#!/bin/bash
# the whole GPU suite
set -o pipefail
O=gpurun_out/suite; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --durations=5 --timeout 300 --timeout-method thread tests -m gpu > $O/t.log 2>&1
rc=$?; tail -8 $O/t.log; exit $rc
