#!/bin/bash
set -o pipefail
O=gpurun_out/syv2; mkdir -p $O
timeout -k 10 600 env NRGPU_LIB=node-replication_amd/lib_t9/libnrgpu.so python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_synthetic.py tests/test_gpu_golden.py tests/test_gpu_stream_order.py -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
SYV_OUT=syv2 bash tools/r6_syv.sh
