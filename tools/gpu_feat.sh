# features + ingest GPU tests, config-4 and ingest benches with kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_features_pipeline.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_feat.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_feat.log; exit 1; }
tail -1 gpurun_out/pytest_feat.log
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo BENCH4_FAIL; tail -20 gpurun_out/bench4.err; exit 2; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof4.log 2>&1 || { echo PROF4_FAIL; tail -20 gpurun_out/prof4.log; exit 3; }
timeout -k 10 300 python -u bench.py --config 4-ingest --steps 10 --warmup 2 > gpurun_out/bench4i.json 2> gpurun_out/bench4i.err || { echo BENCH4I_FAIL; tail -20 gpurun_out/bench4i.err; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4i -o run --output-format csv -- python3 bench.py --config 4-ingest --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof4i.log 2>&1 || { echo PROF4I_FAIL; tail -20 gpurun_out/prof4i.log; exit 5; }
echo ALL_OK
