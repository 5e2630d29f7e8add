set -o pipefail
mkdir -p gpurun_out
for lib in ${LIBS:-libcdr_prev.so libcdr.so}; do
CDR_BENCH_STEP_TIMES=1 CDR_LIB=$PWD/clustering-driven-replication-strategy_amd/$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$lib.json 2>gpurun_out/ab_$lib.err || { tail -20 gpurun_out/ab_$lib.err; exit 1; }
echo $lib; grep "step ms" gpurun_out/ab_$lib.err
python3 -c "import json; r=json.load(open('gpurun_out/ab_$lib.json')); print('ms/step %.4f kernel %.4f step_kernels %.4f fb %.5f' % (r['ms_per_step'], r['roofline']['kernel_ms'], r['step_kernels_ms'], r['fallback_frac']))"
done
