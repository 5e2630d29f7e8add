set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_loop.py tests/test_gpu_kmeans.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_c.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_c.log; exit 2; }
tail -2 gpurun_out/pytest_c.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { echo BENCH3_FAIL; tail -20 gpurun_out/bench3.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/bench3.json'));print('c3',d['ms_per_step'],d['step_kernels_ms'],d['roofline']['kernel_ms'])"
timeout -k 10 300 python -u bench.py --config 3 --n-total 12500000 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/bench3s.json 2> gpurun_out/bench3s.err || { echo BENCH3S_FAIL; tail -20 gpurun_out/bench3s.err; exit 5; }
python3 -c "import json;d=json.load(open('gpurun_out/bench3s.json'));print('c3s',d['ms_per_step'],d['step_kernels_ms'],d['roofline']['kernel_ms'])"
CDR_LIB=$PWD/clustering-driven-replication-strategy_amd/libcdr_exp.so timeout -k 10 300 python -u tools/screen_ablate.py 100000000 16 64 0,1,2,3,8,9,11 > gpurun_out/ablate.log 2>&1 || { echo ABL_FAIL; tail -20 gpurun_out/ablate.log; exit 6; }
cat gpurun_out/ablate.log
echo ALL_OK
