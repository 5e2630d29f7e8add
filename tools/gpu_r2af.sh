# screen32h (raw v_sqrt): parity, config-3 bench x2, PMC passes of the hi-only screen.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ho.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_ho.log; exit 3; }
tail -2 gpurun_out/pytest_ho.log
for R in 1 2; do
  timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ho.json 2> gpurun_out/ho.err || { echo BENCH_FAIL; tail -5 gpurun_out/ho.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/ho.json'));print(round(d['ms_per_step'],4),d['roofline']['kernel'],round(d['roofline']['kernel_ms'],4),round(d['roofline']['frac'],3),'fb',d['fallback_frac'])" | tee -a gpurun_out/ho_ab.txt
done
bash tools/pmc_lloyd.sh 100000000 16 64 c3h || exit 5
python3 tools/pmc_summary.py gpurun_out/pmc_c3h --want screen32d,fixup32 > gpurun_out/pmc_c3h.txt; cat gpurun_out/pmc_c3h.txt
echo ALL_OK
