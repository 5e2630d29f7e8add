# ingest tests + one PMC pass over the ingest bench (parse kernel)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_ingest2.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_ingest2.log; exit 1; }
tail -1 gpurun_out/pytest_ingest2.log
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS -d gpurun_out/pmc4i -o p --output-format csv -- python3 bench.py --config 4-ingest --steps 2 --warmup 0 --no-cpu-baseline --n-total 4000000 > gpurun_out/pmc4i.log 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc4i.log; exit 2; }
echo PMC_OK
