set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_medians_scoring.py > gpurun_out/pytest_r2l.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_r2l.log; exit 2; }
tail -1 gpurun_out/pytest_r2l.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 -u bench.py --config 5 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench5p.json 2> gpurun_out/bench5p.err || { echo BENCH5_FAIL; tail -30 gpurun_out/bench5p.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/bench5p.json'));print('c5',d['ms_per_step'],d['roofline']['kernel_ms'],d.get('replica_scoring_ms'))"
for f in $(find gpurun_out/prof5 -name "*kernel_stats.csv"); do python3 tools/kstats.py $f > gpurun_out/prof5_table.txt; done
head -30 gpurun_out/prof5_table.txt > gpurun_out/prof5_head.txt; cat gpurun_out/prof5_head.txt
echo ALL_OK
