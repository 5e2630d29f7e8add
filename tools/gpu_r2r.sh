# cand_big ablations (experiments build): config-5 step time with parts of L2 switched off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export CDR_LIB=$PWD/clustering-driven-replication-strategy_amd/libcdr_exp.so
for A in 0 1 4 6; do
  CDR_BIG_ABL=$A timeout -k 10 300 python -u bench.py --config 5 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b5abl$A.json 2> gpurun_out/b5abl$A.err || { echo ABL_FAIL $A; tail -5 gpurun_out/b5abl$A.err; exit 3; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/b5abl$A.json'));print('abl',$A,round(d['ms_per_step'],3),round(d['step_kernels_ms'],3),round(d['roofline']['kernel_ms'],3))"
done
echo ALL_OK
