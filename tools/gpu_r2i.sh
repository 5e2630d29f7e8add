# Sharded features on the device + PMC of the group-by kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_features_dist.py > gpurun_out/pytest_r2i.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_r2i.log; exit 2; }
tail -4 gpurun_out/pytest_r2i.log
bash tools/gpu_pmc4.sh
