# PMC passes of the default DELTA screens: config 3 (screen32h LDS ring) and config 2 (screen32h1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_lloyd.sh 100000000 16 64 c3l || exit 5
python3 tools/pmc_summary.py gpurun_out/pmc_c3l --want screen32d,fixup32 > gpurun_out/pmc_c3l.txt; cat gpurun_out/pmc_c3l.txt
bash tools/pmc_lloyd.sh 10000000 8 16 c2h || exit 6
python3 tools/pmc_summary.py gpurun_out/pmc_c2h --want screen32d,fixup32 > gpurun_out/pmc_c2h.txt; cat gpurun_out/pmc_c2h.txt
echo ALL_OK
