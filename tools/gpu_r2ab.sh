# screen32d non-temporal loads A/B (interleaved runs), configs 3 and the 12.5M shard.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for R in 1 2; do
for NT in 0 1; do
  for CFG in "--config 3 --steps 20" "--config 3 --steps 50 --n-total 12500000"; do
    CDR_S32D_NT=$NT timeout -k 10 200 python -u bench.py $CFG --warmup 3 --no-cpu-baseline > gpurun_out/nt.json 2> gpurun_out/nt.err || { echo BENCH_FAIL $NT $CFG; tail -5 gpurun_out/nt.err; exit 3; }
    python3 -c "import json;d=json.load(open('gpurun_out/nt.json'));print('NT=$NT','$CFG',round(d['ms_per_step'],4),d['roofline']['kernel'],round(d['roofline']['kernel_ms'],4),round(d['roofline']['frac'],3))" | tee -a gpurun_out/nt_ab.txt
  done
done
done
echo ALL_OK
