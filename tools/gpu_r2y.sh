# seeding with exact pruning: seeding tests, bench seed_s at configs 3 and 5, seed kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kmeans.py tests/test_gpu_loop.py -k "seed or reference or config3 or config5 or two_shards or sharded" > gpurun_out/pytest_seed.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_seed.log; exit 1; }
tail -1 gpurun_out/pytest_seed.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b3.json 2> gpurun_out/b3.err || { echo B3_FAIL; tail -5 gpurun_out/b3.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/b3.json'));print('c3 seed_s',d['seed_s'],'ms',d['ms_per_step'],'shift',d['final_shift'],'inertia',d['final_inertia'])"
timeout -k 10 300 python -u bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b5.json 2> gpurun_out/b5.err || { echo B5_FAIL; tail -5 gpurun_out/b5.err; exit 4; }
python3 -c "import json;d=json.load(open('gpurun_out/b5.json'));print('c5 seed_s',d['seed_s'],'ms',d['ms_per_step'],'shift',d['final_shift'],'inertia',d['final_inertia'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5s -o run --output-format csv -- python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof5s.log 2>&1 || { echo PROF_FAIL; tail -5 gpurun_out/prof5s.log; exit 5; }
python3 tools/kstats.py gpurun_out/prof5s/run_kernel_stats.csv seed walk xfer search approx ccd > gpurun_out/prof5s.txt; cat gpurun_out/prof5s.txt
echo ALL_OK
