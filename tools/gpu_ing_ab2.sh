# ingest tests + A/B of the parse kernel against the previous library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_ingest2.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_ingest2.log; exit 1; }
tail -1 gpurun_out/pytest_ingest2.log
for v in "" _a _b "" _a _b; do
  CDR_LIB=$PWD/clustering-driven-replication-strategy_amd/libcdr$v.so timeout -k 10 200 python -u bench.py --config 4-ingest --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab$v.json 2> gpurun_out/ab$v.err || { echo FAIL $v; tail -5 gpurun_out/ab$v.err; exit 1; }
  python -c "import json,sys; r=json.load(open('gpurun_out/ab$v.json')); print('lib$v', round(r['roofline']['kernel_ms'],3), round(r['ms_per_step'],3))"
done
