# kmeans GPU tests with the default lib, then A/B/C of the prefetch-depth builds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_k.log; exit 1; }
tail -1 gpurun_out/pytest_k.log
for r in 1 2; do for D in 1 2 3; do
CDR_LIB=build_alt/libcdr_d$D.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_d$D.json 2> gpurun_out/ab.err || { echo AB_FAIL; tail -20 gpurun_out/ab.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/ab_d$D.json'));print('depth $D', 'ms/step %.4f kernel %.4f stepk %.4f' % (d['ms_per_step'],d['roofline']['kernel_ms'],d['step_kernels_ms']))"
done; done
