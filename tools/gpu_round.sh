# One GPU call: all GPU tests, bench config 3 (with CPU leg) and 2, rocprofv3
# kernel stats of the config-3 bench, PMC passes for configs 3 and 2, config 5,
# and the config-4 ingest leg with its kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 11; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { echo BENCH3_FAIL; tail -20 gpurun_out/bench3.err; exit 2; }
cat gpurun_out/bench3.json
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo BENCH2_FAIL; tail -20 gpurun_out/bench2.err; exit 3; }
cat gpurun_out/bench2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof3.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof3.log; exit 4; }
bash tools/pmc_lloyd.sh 100000000 16 64 c3 || exit 5
python tools/pmc_summary.py gpurun_out/pmc_c3 --json 3 100000000 > gpurun_out/pmc_c3.txt || exit 7
bash tools/pmc_lloyd.sh 10000000 8 16 c2 || exit 6
python tools/pmc_summary.py gpurun_out/pmc_c2 --json 2 10000000 > gpurun_out/pmc_c2.txt || exit 8
cp profiles/pmc_traffic.json gpurun_out/ || true
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo BENCH5_FAIL; tail -20 gpurun_out/bench5.err; exit 9; }
cat gpurun_out/bench5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof5.log 2>&1 || { echo PROF5_FAIL; tail -20 gpurun_out/prof5.log; exit 10; }
timeout -k 10 300 python -u bench.py --config 4-ingest --steps 10 --warmup 2 > gpurun_out/bench4i.json 2> gpurun_out/bench4i.err || { echo BENCH4I_FAIL; tail -20 gpurun_out/bench4i.err; exit 12; }
cat gpurun_out/bench4i.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4i -o run --output-format csv -- python3 bench.py --config 4-ingest --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof4i.log 2>&1 || { echo PROF4I_FAIL; tail -20 gpurun_out/prof4i.log; exit 13; }
echo ALL_OK
