# one-byte label copy in screen32d: parity (kmeans + loop GPU tests), then NT A/B at config 3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lab8.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_lab8.log; exit 3; }
tail -2 gpurun_out/pytest_lab8.log
for R in 1 2 3; do
for NT in 0 1; do
  CFG="--config 3 --steps 20"
  CDR_S32D_NT=$NT timeout -k 10 200 python -u bench.py $CFG --warmup 3 --no-cpu-baseline > gpurun_out/nt.json 2> gpurun_out/nt.err || { echo BENCH_FAIL $NT $CFG; tail -5 gpurun_out/nt.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/nt.json'));print('NT=$NT','$CFG',round(d['ms_per_step'],4),d['roofline']['kernel'],round(d['roofline']['kernel_ms'],4),round(d['roofline']['frac'],3))" | tee -a gpurun_out/nt_ab.txt
done
done
echo ALL_OK
