# Lean-step parity (kmeans + loop tests) and the fixup/finalize split at 12.5M and 100M.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_loop.py tests/test_gpu_kmeans.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_d.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_d.log; exit 2; }
tail -2 gpurun_out/pytest_d.log
bash tools/gpu_fixabl.sh && NTOT=100000000 bash tools/gpu_fixabl.sh
