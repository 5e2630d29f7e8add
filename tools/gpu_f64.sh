set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f64_update.py > gpurun_out/pytest_f64.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_f64.log; exit 2; }
grep -E "PASSED|FAILED|F64 2M|passed|failed" gpurun_out/pytest_f64.log | tail -8
