# Hand-written group-by + device simulator: parity tests, config-4 bench, rocprof.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_groupby.py tests/test_gpu_simulate.py tests/test_gpu_features_pipeline.py \
  tests/test_gpu_ingest.py tests/test_spark_semantics.py > gpurun_out/pytest_r2g.log 2>&1 \
  || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_r2g.log; exit 2; }
tail -3 gpurun_out/pytest_r2g.log
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo BENCH4_FAIL; tail -30 gpurun_out/bench4.err; exit 3; }
cat gpurun_out/bench4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 -u bench.py --config 4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench4_prof.json 2> gpurun_out/bench4_prof.err || { echo PROF_FAIL; tail -30 gpurun_out/bench4_prof.err; exit 4; }
for f in $(find gpurun_out/prof4 -name "*kernel_stats.csv"); do python3 tools/kstats.py $f > gpurun_out/prof4_table.txt; done
cat gpurun_out/prof4_table.txt
echo ALL_OK
