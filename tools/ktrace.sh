#!/bin/bash
# Kernel-trace a bench.py run on the GPU box and print the per-kernel stats (rocprofv3).
# Usage (from the repo root, through gpurun): tools/ktrace.sh TAG [bench.py args...]
# Tuning knobs go through bench.py --knob NAME=VALUE (nrg_test_set_knob), e.g. --knob K1=2.
# Output: gpurun_out/kt_<TAG>/ (trace CSVs, bench JSON line) and a summary on stdout.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/kt_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- \
    python3 bench.py --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?
if [ $rc -ne 0 ]; then echo "[ktrace $TAG] rc=$rc"; tail -5 $OUT/bench.err; exit $rc; fi
S=$(find $OUT -name '*kernel_stats.csv' | head -1)
python3 - "$S" "$TAG" "$OUT/bench.json" <<'EOF'
import csv, json, sys
path, tag, bj = sys.argv[1:4]
rows = list(csv.DictReader(open(path)))
b = json.loads(open(bj).read().strip().splitlines()[-1])
print(f"[{tag}] value={b['value']} ms/step={b['ms_per_step']} prev={b.get('variants', {}).get('prev_value_responses_Mops')}")
for r in rows[:8]:
    n = r["Name"].split("(")[0].replace("void ", "")[:60]
    print(f"   {n:60s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:8.2f} pct={float(r['Percentage']):6.2f}")
EOF
