#!/bin/bash
# microbench/req_gran: random 32-B slot reads under allocation kinds and cache-policy bits, timed
# and with memory-side request sizes (one PMC pass per configuration).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/gran; mkdir -p $O
for a in 0 1 2; do for l in 0 1 2 3; do
  timeout -k 10 60 ./microbench/req_gran $a $l >> $O/timed.txt 2>&1 || exit $?
done; done
cat $O/timed.txt
for a in 0 1 2; do for l in 0 2; do
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
     -d $O/p_${a}_$l -o run --output-format csv -- ./microbench/req_gran $a $l > $O/p_${a}_$l.log 2>&1 || exit $?
done; done
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob('gpurun_out/gran/p_*')):
    import os
    if not os.path.isdir(d): continue
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
        for r in csv.DictReader(open(f)):
            if 'gets' not in r['Kernel_Name']: continue
            acc[r['Kernel_Name']][r['Counter_Name']] += float(r['Counter_Value'])
            n[(r['Kernel_Name'], r['Counter_Name'])] += 1
        for k, c in acc.items():
            L = max(n[(k, x)] for x in c)
            print(d, {x: round(v / L / 900000, 4) for x, v in sorted(c.items())}, 'per Get')
PY
