# Spark null-timestamp / duplicate-path semantics and the F32X gate on the device.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_spark_semantics.py tests/test_gpu_ingest.py tests/test_gpu_features_pipeline.py \
  "tests/test_gpu_kmeans.py::test_f32x_gate_keeps_numpy_mean_exact" > gpurun_out/pytest_r2f.log 2>&1 \
  || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_r2f.log; exit 2; }
tail -3 gpurun_out/pytest_r2f.log
echo ALL_OK
