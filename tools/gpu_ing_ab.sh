# A/B of ingest parse tile shapes (libcdr variants built with -DCDR_ING_REC/-DCDR_ING_STAGE).
set -o pipefail
mkdir -p gpurun_out
for v in "" _a _b _c; do
  CDR_LIB=$PWD/clustering-driven-replication-strategy_amd/libcdr$v.so timeout -k 10 200 python -u bench.py --config 4-ingest --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab$v.json 2> gpurun_out/ab$v.err || { echo FAIL $v; tail -5 gpurun_out/ab$v.err; exit 1; }
  python -c "import json,sys; r=json.load(open('gpurun_out/ab$v.json')); print('$v', round(r['roofline']['kernel_ms'],3), round(r['ms_per_step'],3))"
done
