# sharded device loop (two contexts, device all-reduce buffer) + loop tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loop.py > gpurun_out/pytest_loop.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_loop.log; exit 1; }
tail -3 gpurun_out/pytest_loop.log
echo ALL_OK
