# Round 2 re-entry check: all GPU tests, smoke, default bench + kernel stats,
# config 4 (simulated log) bench + kernel stats, config 5 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_default.err; exit 3; }
cat gpurun_out/bench_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof3.log 2>&1 || { echo PROF3_FAIL; tail -20 gpurun_out/prof3.log; exit 4; }
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo BENCH4_FAIL; tail -20 gpurun_out/bench4.err; exit 5; }
cat gpurun_out/bench4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof4.log 2>&1 || { echo PROF4_FAIL; tail -20 gpurun_out/prof4.log; exit 6; }
timeout -k 10 400 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo BENCH5_FAIL; tail -20 gpurun_out/bench5.err; exit 7; }
cat gpurun_out/bench5.json
timeout -k 10 300 python -u bench.py --config 4-ingest --steps 10 --warmup 2 > gpurun_out/bench4i.json 2> gpurun_out/bench4i.err || { echo BENCH4I_FAIL; tail -20 gpurun_out/bench4i.err; exit 8; }
cat gpurun_out/bench4i.json
echo ALL_OK
