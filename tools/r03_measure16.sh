#!/bin/bash
# Round 3, session 2: where the write-heavy stamp round's time goes (N=8 per-GPU round: 800k Puts +
# 900k Gets; configs[2] per GPU: 4M Puts + 500k Gets). EXP 0x100000 no stamp atomics, 0x200000 no
# apply, 0x400000 no index role, 0x800000 no reads (results wrong; timing only); K1 Puts per thread.
mkdir -p gpurun_out/m16
export TMPDIR=/tmp
N8='--ops-per-gpu 1700000 --write-ratio 47'
C2='--ops-per-gpu 4500000 --write-ratio 89 --pool 16'
timeout -k 10 900 python3 tools/sweep.py "n8||$N8" "n8_noatom||$N8 --knob EXP=0x100000" "n8_noapply||$N8 --knob EXP=0x200000" \
  "n8_noindex||$N8 --knob EXP=0x400000" "n8_noreads||$N8 --knob EXP=0x800000" "n8_k1||$N8 --knob K1=1" "n8_k4||$N8 --knob K1=4" \
  "c2||$C2" "c2_noatom||$C2 --knob EXP=0x100000" "c2_noapply||$C2 --knob EXP=0x200000" "c2_k4||$C2 --knob K1=4" \
  "w100||--write-ratio 100" "w100_noatom||--write-ratio 100 --knob EXP=0x100000" "w100_noapply||--write-ratio 100 --knob EXP=0x200000" \
  > gpurun_out/m16/sweep.txt 2>&1
rc=$?; cat gpurun_out/m16/sweep.txt; exit $rc
