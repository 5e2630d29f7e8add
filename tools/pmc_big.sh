# rocprofv3 PMC passes over the config-5 screen (tools/lloyd_loop.py 50M x 64, k=1024).
#   bash tools/pmc_big.sh TAG   -> gpurun_out/pmc_TAG/p{1..3}
set -o pipefail
TAG=${1:-c5}
O=gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
A="50000000 64 1024 2"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES -d $O/p1 -o p1 --output-format csv -- python3 tools/lloyd_loop.py $A > $O/p1.log 2>&1 || exit 11
timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $O/p2 -o p2 --output-format csv -- python3 tools/lloyd_loop.py $A > $O/p2.log 2>&1 || exit 12
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU_MFMA_F16 SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT GRBM_COUNT -d $O/p3 -o p3 --output-format csv -- python3 tools/lloyd_loop.py $A > $O/p3.log 2>&1 || exit 13
echo PMC_OK $TAG
