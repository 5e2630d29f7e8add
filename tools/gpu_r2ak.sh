# hi-only screen for d <= 8 (screen32h1): parity, config 2 A/B vs the split copy, config 3 check.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_h1.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_h1.log; exit 3; }
tail -2 gpurun_out/pytest_h1.log
for R in 1 2; do
for HO in 1 0; do
  CDR_S32D_HO=$HO timeout -k 10 200 python -u bench.py --config 2 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/h1.json 2> gpurun_out/h1.err || { echo BENCH_FAIL; tail -5 gpurun_out/h1.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/h1.json'));r=d['roofline'];print('c2 HO=$HO',round(d['ms_per_step'],4),r['kernel'],round(r['kernel_ms'],4),round(r['frac'],3),round(r.get('kernel_frac',0),3),'fb',d['fallback_frac'])" | tee -a gpurun_out/h1_ab.txt
done
done
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/h1c3.json 2> gpurun_out/h1c3.err || { echo BENCH_FAIL; tail -5 gpurun_out/h1c3.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/h1c3.json'));r=d['roofline'];print('c3',round(d['ms_per_step'],4),r['kernel'],round(r['kernel_ms'],4),round(r['frac'],3))"
echo ALL_OK
