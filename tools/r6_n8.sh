#!/bin/bash
# N = 8 per-GPU round components (one-GPU emulation): kernel traces
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/n8; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-prev-variant --steps 100 --warmup 10 --no-kernel-timing"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/full -o run -- $B --ops-per-gpu 1700000 --write-ratio 47 > $O/full.json 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/puts -o run -- $B --ops-per-gpu 800000 --write-ratio 100 > $O/puts.json 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/gets -o run -- $B --ops-per-gpu 900000 --write-ratio 0 > $O/gets.json 2>&1
rc=$?
for v in full puts gets; do echo "== $v"; tail -1 $O/$v.json | cut -c1-150; python3 - $O/$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'hm_' in r['Name']:
        print("  %-60s calls %5s avg %8.2f us" % (r['Name'].split('(')[0][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
exit $rc
