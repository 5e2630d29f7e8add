# A/B: bench config 3 with the in-tree libcdr.so vs build_alt/libcdr.so
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_a$i.json 2> gpurun_out/bench_a.err || { echo A_FAIL; tail -20 gpurun_out/bench_a.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_a$i.json'));print('A',d['ms_per_step'],d['roofline']['kernel_ms'],d['step_kernels_ms'])"
CDR_LIB=build_alt/libcdr.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_b$i.json 2> gpurun_out/bench_b.err || { echo B_FAIL; tail -20 gpurun_out/bench_b.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_b$i.json'));print('B',d['ms_per_step'],d['roofline']['kernel_ms'],d['step_kernels_ms'])"
done
