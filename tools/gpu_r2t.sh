# device-resident large-k loop: loop + large-k tests, config-5 bench + kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_kmeans.py -k "loop or large_k or config5" > gpurun_out/pytest_big.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_big.log; exit 1; }
tail -1 gpurun_out/pytest_big.log
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo BENCH5_FAIL; tail -20 gpurun_out/bench5.err; exit 5; }
python3 -c "import json;d=json.load(open('gpurun_out/bench5.json'));print('c5',d['ms_per_step'],d['step_kernels_ms'],d['roofline']['kernel'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['fallback_frac'],d.get('replica_scoring_ms'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof5.log 2>&1 || { echo PROF5_FAIL; tail -20 gpurun_out/prof5.log; exit 8; }
python3 tools/kstats.py gpurun_out/prof5/run_kernel_stats.csv > gpurun_out/prof5_table.txt; head -16 gpurun_out/prof5_table.txt
echo ALL_OK
