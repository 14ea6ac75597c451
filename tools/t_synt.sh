set -o pipefail
mkdir -p gpurun_out/synt
timeout -k 10 600 python tools/sweep.py \
 'sy|| --workload synthetic' 'sy_log|| --workload synthetic --knob EXP=64' 'sy_E|| --workload synthetic --knob EXP=128' \
 'sy_V|| --workload synthetic --knob EXP=256' 'sy_resp|| --workload synthetic --knob EXP=512' \
 'syb|| --workload synthetic' 'syb_log|| --workload synthetic --knob EXP=64' 'syb_E|| --workload synthetic --knob EXP=128' \
 'syb_V|| --workload synthetic --knob EXP=256' 'syb_resp|| --workload synthetic --knob EXP=512' \
 > gpurun_out/synt/sweep.txt 2>&1
