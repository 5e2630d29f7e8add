# The documented A/B switches stay green: kmeans + loop GPU tests with the split-copy DELTA screen
# (CDR_S32D_HO=0) and with register prefetch for the hi-only screen (CDR_S32H_LR=0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CDR_S32D_HO=0 timeout -k 10 500 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ho0.log 2>&1 || { echo PYTEST_HO0_FAIL; tail -30 gpurun_out/pytest_ho0.log; exit 3; }
tail -1 gpurun_out/pytest_ho0.log
CDR_S32H_LR=0 timeout -k 10 500 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lr0.log 2>&1 || { echo PYTEST_LR0_FAIL; tail -30 gpurun_out/pytest_lr0.log; exit 4; }
tail -1 gpurun_out/pytest_lr0.log
echo ALL_OK
