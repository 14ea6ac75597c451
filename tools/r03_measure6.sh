#!/bin/bash
# Round 3, session 2: kernel traces of the synthetic round (XCD-remapped buckets and the plain
# order), the B1 headline and the stack round.
export TMPDIR=/tmp
bash tools/ktrace.sh sy_xcd --workload synthetic --steps 200 &&
NRGPU_LIB=node-replication_amd/lib/libnrgpu_noremap.so bash tools/ktrace.sh sy_noxcd --workload synthetic --steps 200 &&
bash tools/ktrace.sh b1 --steps 200 --no-prev-variant &&
bash tools/ktrace.sh stack --workload stack --steps 200
