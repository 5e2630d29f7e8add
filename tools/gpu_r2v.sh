# screen32d prefetch depth A/B (PD = 2, 3, 4): configs 2, 3 and the 8-GPU shard of config 3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kmeans.py tests/test_gpu_loop.py -k "incremental or two_shards or loop_matches" > gpurun_out/pytest_pd.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_pd.log; exit 1; }
tail -1 gpurun_out/pytest_pd.log
for PD in 2 3 4; do
  for CFG in "--config 2 --steps 50" "--config 3 --steps 20" "--config 3 --steps 50 --n-total 12500000"; do
    CDR_S32D_PD=$PD timeout -k 10 200 python -u bench.py $CFG --warmup 3 --no-cpu-baseline > gpurun_out/pd.json 2> gpurun_out/pd.err || { echo BENCH_FAIL $PD $CFG; tail -5 gpurun_out/pd.err; exit 3; }
    python3 -c "import json;d=json.load(open('gpurun_out/pd.json'));print('PD=$PD','$CFG',round(d['ms_per_step'],4),d['roofline']['kernel'],round(d['roofline']['kernel_ms'],4),round(d['roofline']['frac'],3))" | tee -a gpurun_out/pd_ab.txt
  done
done
echo ALL_OK
