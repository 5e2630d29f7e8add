set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for abl in 4 2; do
CDR_BIG_ABL=$abl timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bbl$abl -o r --output-format csv -- python3 bench.py --config 5 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bbl$abl.log 2>&1 || exit 1
echo abl=$abl; python3 tools/kstats.py gpurun_out/bbl$abl/r_kernel_stats.csv | grep -E "big"
done
