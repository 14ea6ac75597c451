#!/bin/bash
# Replica mirror: blocking flat-combining wait, locked pending queues
set -o pipefail
O=gpurun_out/rep; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --durations=12 --timeout 300 --timeout-method thread tests/test_gpu_reference_examples.py tests/test_gpu_replica_api.py tests/test_gpu_verify_stack.py -m gpu > $O/t.log 2>&1
rc=$?; tail -20 $O/t.log; exit $rc
