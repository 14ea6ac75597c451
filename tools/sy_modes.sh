set -e
mkdir -p gpurun_out/sym
export TMPDIR=/tmp
for m in ${MODES:-0 256 512 768}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sym/m$m -o run -- python3 bench.py --knob EXP=$m --workload synthetic --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sym/m$m.json 2>/dev/null
  grep -h "sy_" gpurun_out/sym/m$m/*/run_kernel_stats.csv gpurun_out/sym/m$m/run_kernel_stats.csv 2>/dev/null | cut -d, -f1-5 | sed "s/^/m$m /"
done
