# Kernel-time split of the DELTA step's fixup / finalize (experiments build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export CDR_LIB=$PWD/clustering-driven-replication-strategy_amd/libcdr_exp.so
run() {  # name, env...
  env "${@:2}" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/fa_$1 -o run --output-format csv -- python3 bench.py --config 3 --n-total ${NTOT:-12500000} --steps 30 --warmup 2 --no-cpu-baseline > gpurun_out/fa_$1.log 2>&1 || { echo FAIL $1; tail -5 gpurun_out/fa_$1.log; return 1; }
  echo "== $1"; python3 tools/kstats.py gpurun_out/fa_$1/run_kernel_stats.csv screen32d fixup finalize
}
run base X=1 && run nofb CDR_FIX_ABL=2 && run noflush CDR_FIX_ABL=4 && run none CDR_FIX_ABL=7 && echo ALL_OK
