# bench config 3 (no CPU leg) under rocprofv3 kernel stats -> gpurun_out/prof3
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-3}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof$CFG -o run --output-format csv -- python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof$CFG.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof$CFG.log; exit 4; }
tail -1 gpurun_out/prof$CFG.log
python3 tools/kstats.py gpurun_out/prof$CFG/run_kernel_stats.csv
