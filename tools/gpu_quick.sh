#!/bin/bash
# Quick GPU check: kmeans parity tests + config-3 bench (no CPU baseline).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench3q.json 2> gpurun_out/bench3q.err || { echo BENCH3_FAIL; tail -20 gpurun_out/bench3q.err; exit 2; }
cat gpurun_out/bench3q.json
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/bench2q.json 2> gpurun_out/bench2q.err || { echo BENCH2_FAIL; tail -20 gpurun_out/bench2q.err; exit 3; }
cat gpurun_out/bench2q.json
