# One GPU call: ingest + features GPU tests, the config-4 ingest bench leg,
# and rocprofv3 kernel stats of it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_features_pipeline.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_ingest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_ingest.log; exit 1; }
tail -2 gpurun_out/pytest_ingest.log
timeout -k 10 300 python -u bench.py --config 4-ingest --steps 10 --warmup 2 > gpurun_out/bench4i.json 2> gpurun_out/bench4i.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench4i.err; exit 2; }
cat gpurun_out/bench4i.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4i -o run --output-format csv -- python3 bench.py --config 4-ingest --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof4i.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof4i.log; exit 3; }
python tools/kstats.py gpurun_out/prof4i/run_kernel_stats.csv 2>/dev/null | head -20 || true
echo ALL_OK
