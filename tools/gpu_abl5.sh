set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for abl in 0 1 2 4; do
CDR_BIG_ABL=$abl timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abl$abl -o r --output-format csv -- python3 tools/lloyd_loop.py 50000000 64 1024 3 > gpurun_out/abl$abl.log 2>&1 || exit 1
echo abl=$abl; grep -a fallback gpurun_out/abl$abl.log; python3 tools/kstats.py gpurun_out/abl$abl/r_kernel_stats.csv | grep -E "big"
done
