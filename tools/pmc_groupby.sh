# rocprofv3 PMC passes over the config-4 group-by (bench.py --config 4).
#   bash tools/pmc_groupby.sh TAG   -> gpurun_out/pmc_TAG/p{1..4}
set -o pipefail
TAG=${1:-c4}
O=gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
A="bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d $O/p1 -o p1 --output-format csv -- python3 $A > $O/p1.log 2>&1 || exit 11
timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/p2 -o p2 --output-format csv -- python3 $A > $O/p2.log 2>&1 || exit 12
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o p3 --output-format csv -- python3 $A > $O/p3.log 2>&1 || exit 13
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o p4 --output-format csv -- python3 $A > $O/p4.log 2>&1 || exit 14
echo PMC_OK $TAG
