# screen32h: parity (kmeans + loop GPU tests), then prefetch depth A/B at config 3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ho.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_ho.log; exit 3; }
tail -2 gpurun_out/pytest_ho.log
for R in 1 2; do
for V in "1 2" "1 3" "1 4" "0 2"; do
  set -- $V
  CFG="--config 3 --steps 20"
  CDR_S32D_HO=$1 CDR_S32D_PD=$2 timeout -k 10 200 python -u bench.py $CFG --warmup 3 --no-cpu-baseline > gpurun_out/ho.json 2> gpurun_out/ho.err || { echo BENCH_FAIL $V; tail -5 gpurun_out/ho.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/ho.json'));print('HO,PD=$1,$2',round(d['ms_per_step'],4),d['roofline']['kernel'],round(d['roofline']['kernel_ms'],4),round(d['roofline']['frac'],3),'fb',d['fallback_frac'],'inertia',d['final_inertia'])" | tee -a gpurun_out/ho_ab.txt
done
done
echo ALL_OK
