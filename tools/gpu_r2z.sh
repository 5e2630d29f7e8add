# ingest parse: SWAR field scan + 32-bit dates. Ingest tests, bench 4-ingest + kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ingest.py tests/test_gpu_features_pipeline.py tests/test_gpu_features_dist.py > gpurun_out/pytest_ing.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_ing.log; exit 1; }
tail -1 gpurun_out/pytest_ing.log
timeout -k 10 300 python -u bench.py --config 4-ingest --steps 10 --warmup 2 > gpurun_out/bench4i.json 2> gpurun_out/bench4i.err || { echo B_FAIL; tail -5 gpurun_out/bench4i.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/bench4i.json'));print('ingest',d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4i -o run --output-format csv -- python3 bench.py --config 4-ingest --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof4i.log 2>&1 || { echo PROF_FAIL; tail -5 gpurun_out/prof4i.log; exit 5; }
python3 tools/kstats.py gpurun_out/prof4i/run_kernel_stats.csv > gpurun_out/prof4i.txt; head -12 gpurun_out/prof4i.txt
echo ALL_OK
