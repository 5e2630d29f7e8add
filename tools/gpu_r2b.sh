# Round 2: GPU parity after a kernel change + benches of configs 3 / 2 / 3@12.5M.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { echo BENCH3_FAIL; tail -20 gpurun_out/bench3.err; exit 3; }
cat gpurun_out/bench3.json
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo BENCH2_FAIL; tail -20 gpurun_out/bench2.err; exit 4; }
cat gpurun_out/bench2.json
timeout -k 10 300 python -u bench.py --config 3 --n-total 12500000 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/bench3s.json 2> gpurun_out/bench3s.err || { echo BENCH3S_FAIL; tail -20 gpurun_out/bench3s.err; exit 5; }
cat gpurun_out/bench3s.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3s -o run --output-format csv -- python3 bench.py --config 3 --n-total 12500000 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/prof3s.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof3s.log; exit 6; }
echo ALL_OK
