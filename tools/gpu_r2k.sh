# medians (new pipeline) + F64 sums + config-5 bench with replica scoring.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_medians_scoring.py tests/test_gpu_f64_update.py "tests/test_gpu_loop.py::test_config5_full_size_and_scoring" > gpurun_out/pytest_r2k.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_r2k.log; exit 2; }
grep -E "PASSED|FAILED|F64 2M|passed|failed" gpurun_out/pytest_r2k.log | tail -14
timeout -k 10 400 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo BENCH5_FAIL; tail -30 gpurun_out/bench5.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/bench5.json'));print('c5',d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['seed_s'],d.get('replica_scoring_ms'))"
echo ALL_OK
