# 12.5M-row shard (the 8-GPU per-rank share of config 3) and config 2 with the hi-only screen: bench + kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --config 3 --steps 50 --warmup 3 --n-total 12500000 --no-cpu-baseline > gpurun_out/b12.json 2> gpurun_out/b12.err || { echo BENCH_FAIL; tail -5 gpurun_out/b12.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/b12.json'));r=d['roofline'];print('12.5M',round(d['ms_per_step'],4),r['kernel'],round(r['kernel_ms'],4),round(r['frac'],3),d.get('step_kernels_ms'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof12 -o run -- python3 bench.py --config 3 --steps 50 --warmup 3 --n-total 12500000 --no-cpu-baseline > gpurun_out/prof12.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof12.log; exit 7; }
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/prof12/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f))):
    if int(r['Calls'])>=50: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
PY
echo ALL_OK
