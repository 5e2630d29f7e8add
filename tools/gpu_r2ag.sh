# screen32h LDS ring: parity (kmeans incl. near ties + loop), then LR A/B at config 3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lr.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_lr.log; exit 3; }
tail -2 gpurun_out/pytest_lr.log
for R in 1 2; do
for LR in 4 3 2 0; do
  CDR_S32H_LR=$LR timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lr.json 2> gpurun_out/lr.err || { echo BENCH_FAIL $LR; tail -5 gpurun_out/lr.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/lr.json'));r=d['roofline'];print('LR=$LR',round(d['ms_per_step'],4),r['kernel'],round(r['kernel_ms'],4),round(r['frac'],3),round(r.get('kernel_frac',0),3),'fb',d['fallback_frac'])" | tee -a gpurun_out/lr_ab.txt
done
done
echo ALL_OK
