# bench config 3 + 2 (no CPU leg) then the PMC passes of tools/pmc_lloyd.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { echo BENCH3_FAIL; tail -20 gpurun_out/bench3.err; exit 2; }
cat gpurun_out/bench3.json
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo BENCH2_FAIL; tail -20 gpurun_out/bench2.err; exit 3; }
cat gpurun_out/bench2.json
bash tools/pmc_lloyd.sh
