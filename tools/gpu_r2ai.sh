# screen32h address / wait bookkeeping trim: parity, bench x2, config-3 rocprofv3 kernel stats (csv).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_trim.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_trim.log; exit 3; }
tail -2 gpurun_out/pytest_trim.log
for R in 1 2; do
  timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/trim.json 2> gpurun_out/trim.err || { echo BENCH_FAIL; tail -5 gpurun_out/trim.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/trim.json'));r=d['roofline'];print(round(d['ms_per_step'],4),r['kernel'],round(r['kernel_ms'],4),round(r['frac'],3),round(r.get('kernel_frac',0),3),'fb',d['fallback_frac'])" | tee -a gpurun_out/trim_ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof3.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof3.log; exit 7; }
find gpurun_out/prof3 -name "*kernel_stats.csv" > gpurun_out/prof3_files.txt
cat gpurun_out/prof3_files.txt
echo ALL_OK
