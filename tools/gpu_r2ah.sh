# Full regression (round 2 close): GPU tests, smoke, bench configs 3 / 2 / 4 / 5, config-3 rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_default.err; exit 3; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo BENCH2_FAIL; tail -20 gpurun_out/bench2.err; exit 4; }
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo BENCH4_FAIL; tail -20 gpurun_out/bench4.err; exit 5; }
timeout -k 10 400 python -u bench.py --config 5 --steps 10 --warmup 2 > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo BENCH5_FAIL; tail -20 gpurun_out/bench5.err; exit 6; }
for f in bench2 bench4 bench5; do python3 -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['frac'],d.get('cpu_baseline',{}).get('value'))"; done

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof3.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof3.log; exit 7; }
find gpurun_out/prof3 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof3_kernel_stats.csv
echo ALL_OK
