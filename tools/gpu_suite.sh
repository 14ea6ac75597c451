#!/bin/bash
# The GPU test suite on the box, one pytest process per step, each under its own time limit;
# stops at the first failing step. Usage (through gpurun): tools/gpu_suite.sh TAG [first test file]
TAG=${1:-suite}
mkdir -p gpurun_out
if [ -n "$2" ]; then
  timeout -k 10 400 python -u -m pytest "$2" -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_first.log 2>&1
  rc=$?; tail -25 gpurun_out/${TAG}_first.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_all.log 2>&1
rc=$?; tail -8 gpurun_out/${TAG}_all.log
exit $rc
