# prefetching wave buckets: group-by tests + config-4 bench/stats; L1 ablation microbenchmark.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/micro/big_l1 > gpurun_out/big_l1.txt 2>&1 || { echo MICRO_FAIL; cat gpurun_out/big_l1.txt; exit 9; }
cat gpurun_out/big_l1.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 90 --timeout-method thread -m gpu tests/test_gpu_groupby.py tests/test_gpu_features_pipeline.py tests/test_gpu_simulate.py tests/test_gpu_features_dist.py > gpurun_out/pytest_gb.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gb.log; exit 1; }
tail -1 gpurun_out/pytest_gb.log
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo BENCH4_FAIL; tail -20 gpurun_out/bench4.err; exit 5; }
python3 -c "import json;d=json.load(open('gpurun_out/bench4.json'));print('c4',d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof4.log 2>&1 || { echo PROF4_FAIL; tail -20 gpurun_out/prof4.log; exit 6; }
python3 tools/kstats.py gpurun_out/prof4/run_kernel_stats.csv gb_ > gpurun_out/prof4_gb.txt; cat gpurun_out/prof4_gb.txt
echo ALL_OK
