# kmeans GPU parity tests + config 3/2 bench lines (no CPU leg)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_k.log; exit 1; }
tail -2 gpurun_out/pytest_k.log
for c in 3 2; do
timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench$c.json 2> gpurun_out/bench$c.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench$c.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/bench$c.json'));print('$c', 'ms/step',d['ms_per_step'],'kernel',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'],'stepk',d['step_kernels_ms'],'fb',d['fallback_frac'])"
done
