# screen_big_sp (software-pipelined L1): large-k tests, config-5 bench A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kmeans.py -k "large_k" > gpurun_out/pytest_big.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_big.log; exit 1; }
tail -1 gpurun_out/pytest_big.log
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5_sp.json 2> gpurun_out/bench5_sp.err || { echo BENCH5_FAIL; tail -20 gpurun_out/bench5_sp.err; exit 5; }
python3 -c "import json;d=json.load(open('gpurun_out/bench5_sp.json'));print('sp512',d['ms_per_step'],d['roofline']['kernel'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['fallback_frac'])"
CDR_BIG_SP_NT=768 timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5_sp768.json 2> gpurun_out/bench5_sp768.err || { echo BENCH5b_FAIL; tail -20 gpurun_out/bench5_sp768.err; exit 6; }
python3 -c "import json;d=json.load(open('gpurun_out/bench5_sp768.json'));print('sp768',d['ms_per_step'],d['roofline']['kernel'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['fallback_frac'])"
CDR_BIG_L1=0 timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5_old.json 2> gpurun_out/bench5_old.err || { echo BENCH5c_FAIL; tail -20 gpurun_out/bench5_old.err; exit 7; }
python3 -c "import json;d=json.load(open('gpurun_out/bench5_old.json'));print('old',d['ms_per_step'],d['roofline']['kernel'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['fallback_frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof5.log 2>&1 || { echo PROF5_FAIL; tail -20 gpurun_out/prof5.log; exit 8; }
python3 tools/kstats.py gpurun_out/prof5/run_kernel_stats.csv > gpurun_out/prof5_table.txt; head -12 gpurun_out/prof5_table.txt
echo ALL_OK
