#!/bin/bash
# Round 3, session 2: Zipf 0.99 streams (BASELINE configs[3]) on the current build, with the
# bucket-elector phase stamps for the 50 % write stream.
mkdir -p gpurun_out/m26
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/sweep.py "z10||--dist zipf" "z50||--dist zipf --write-ratio 50" \
  "z50s||--dist zipf --scramble --write-ratio 50" "z90s||--dist zipf --scramble --write-ratio 90" > gpurun_out/m26/sweep.txt 2>&1
rc=$?; cat gpurun_out/m26/sweep.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/m26/kt -o run -- \
    python3 bench.py --no-cpu-baseline --no-prev-variant --dist zipf --write-ratio 50 --steps 200 > gpurun_out/m26/kt.json 2>/dev/null || exit 1
T=$(find gpurun_out/m26/kt -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$T')))[:6]:
    print('%-50s calls %6s avg %8.2f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))"
