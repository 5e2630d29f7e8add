set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b3_$i.json 2>gpurun_out/b3_$i.err || { tail -20 gpurun_out/b3_$i.err; exit 1; }
python3 -c "import json; r=json.load(open('gpurun_out/b3_$i.json')); print('ms/step %.4f kernel %.4f step_kernels %.4f fb %.5f' % (r['ms_per_step'], r['roofline']['kernel_ms'], r['step_kernels_ms'], r['fallback_frac']))"
done
