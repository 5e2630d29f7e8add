# fixup32 regions per workgroup A/B (CDR_FIX_FR): parity at 16, step time at 12.5M and 100M.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CDR_FIX_FR=16 timeout -k 10 500 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fr.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_fr.log; exit 3; }
tail -2 gpurun_out/pytest_fr.log
for R in 1 2; do
for FR in 4 8 16; do
  CDR_FIX_FR=$FR timeout -k 10 200 python -u bench.py --config 3 --steps 50 --warmup 3 --n-total 12500000 --no-cpu-baseline > gpurun_out/fr.json 2> gpurun_out/fr.err || { echo BENCH_FAIL; tail -5 gpurun_out/fr.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/fr.json'));r=d['roofline'];print('12.5M FR=$FR',round(d['ms_per_step'],4),round(r['kernel_ms'],4),round(d['step_kernels_ms'],4))" | tee -a gpurun_out/fr_ab.txt
  CDR_FIX_FR=$FR timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/fr.json 2> gpurun_out/fr.err || { echo BENCH_FAIL; tail -5 gpurun_out/fr.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/fr.json'));r=d['roofline'];print('100M FR=$FR',round(d['ms_per_step'],4),round(r['kernel_ms'],4),round(d['step_kernels_ms'],4))" | tee -a gpurun_out/fr_ab.txt
done
done
echo ALL_OK
