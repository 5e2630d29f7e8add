set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_k.log; exit 1; }
tail -2 gpurun_out/pytest_k.log
timeout -k 10 200 python -u tools/screen_ablate.py 100000000 16 64 0,1,2,8 > gpurun_out/abl_a.log 2>&1 || { echo ABL_FAIL; tail gpurun_out/abl_a.log; exit 2; }
cat gpurun_out/abl_a.log
CDR_LIB=build_alt/libcdr.so timeout -k 10 200 python -u tools/screen_ablate.py 100000000 16 64 0,1,2,8 > gpurun_out/abl_b.log 2>&1 || { echo ABL_FAIL; tail gpurun_out/abl_b.log; exit 3; }
cat gpurun_out/abl_b.log
