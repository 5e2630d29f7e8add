# Group-by variants at config 4: dense vs hash buckets, rocprof of the default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_groupby.py tests/test_gpu_simulate.py > gpurun_out/pytest_r2h.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_r2h.log; exit 2; }
tail -1 gpurun_out/pytest_r2h.log
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo BENCH4_FAIL; tail -30 gpurun_out/bench4.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/bench4.json'));print('dense',d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['partition_ms'],d['groupby'])"
CDR_GB_HASH=1 timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench4h.json 2> gpurun_out/bench4h.err || { echo BENCH4H_FAIL; tail -30 gpurun_out/bench4h.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/bench4h.json'));print('hash',d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['partition_ms'],d['groupby'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 -u bench.py --config 4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench4_prof.json 2> gpurun_out/bench4_prof.err || { echo PROF_FAIL; tail -30 gpurun_out/bench4_prof.err; exit 4; }
for f in $(find gpurun_out/prof4 -name "*kernel_stats.csv"); do python3 tools/kstats.py $f gb_ > gpurun_out/prof4_table.txt; done
cat gpurun_out/prof4_table.txt
echo ALL_OK
