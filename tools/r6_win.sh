#!/bin/bash
# roofline window timing (stream events around rounds 1..n-1) vs dispatch-bracketed launches vs rocprof
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/win; mkdir -p $O
for w in hashmap stack synthetic; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/b_$w.json 2> $O/b_$w.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$w -o run -- python3 bench.py --workload $w --no-cpu-baseline --no-prev-variant > $O/kt_$w.json 2> $O/kt_$w.err || exit $?
done
for w in hashmap stack synthetic; do
python3 - $O $w <<'PY'
import csv, glob, json, sys
O, w = sys.argv[1], sys.argv[2]
for tag in ("b", "kt"):
    l = [x for x in open(f"{O}/{tag}_{w}.json") if x.startswith("{")][-1]
    r = json.loads(l)["roofline"]
    print(w, tag, "ms/step %.2f" % (json.loads(l)["ms_per_step"] * 1e3), "window", r["avg_launch_us"], "bracketed", r["bracketed_avg_launch_us"], "frac", r["frac"])
f = glob.glob(f"{O}/kt_{w}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("hm_round", "hm_papply", "st_round", "sy_round")):
        print("   rocprof", r["Name"].split("(")[0][:50], r["Calls"], "avg %.2f us" % (float(r["AverageNs"]) / 1e3))
PY
done
