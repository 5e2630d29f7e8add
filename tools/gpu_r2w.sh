# PMC passes: config-5 L1 (screen_big_sp) and config-3 screen32d traffic.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_big.sh c5sp || exit 7
python3 tools/pmc_summary.py gpurun_out/pmc_c5sp --want screen_big_sp,cand_big,fixup_big,update_big > gpurun_out/pmc_c5sp.txt; cat gpurun_out/pmc_c5sp.txt
bash tools/pmc_lloyd.sh 100000000 16 64 c3 || exit 5
python3 tools/pmc_summary.py gpurun_out/pmc_c3 --want screen32d,fixup32,screen32 > gpurun_out/pmc_c3.txt; cat gpurun_out/pmc_c3.txt
echo ALL_OK
