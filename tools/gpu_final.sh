# Round-end check: all GPU tests, smoke, default bench, ingest leg + its kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_default.err; exit 3; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python -u bench.py --config 4-ingest --steps 10 --warmup 2 > gpurun_out/bench4i.json 2> gpurun_out/bench4i.err || { echo BENCH4I_FAIL; tail -20 gpurun_out/bench4i.err; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4i -o run --output-format csv -- python3 bench.py --config 4-ingest --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof4i.log 2>&1 || { echo PROF4I_FAIL; tail -20 gpurun_out/prof4i.log; exit 5; }
echo ALL_OK
