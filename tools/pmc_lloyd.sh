# rocprofv3 PMC passes (one counter group per run) over tools/lloyd_loop.py.
#   bash tools/pmc_lloyd.sh N D K TAG   -> gpurun_out/pmc_TAG/p{1..4}
set -o pipefail
N=${1:-100000000}; D=${2:-16}; K=${3:-64}; TAG=${4:-c3}
O=gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES -d $O/p1 -o p1 --output-format csv -- python3 tools/${DRV:-lloyd_loop}.py $N $D $K ${STEPS:-3} > $O/p1.log 2>&1 || exit 11
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $O/p2 -o p2 --output-format csv -- python3 tools/${DRV:-lloyd_loop}.py $N $D $K ${STEPS:-3} > $O/p2.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o p3 --output-format csv -- python3 tools/${DRV:-lloyd_loop}.py $N $D $K ${STEPS:-3} > $O/p3.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o p4 --output-format csv -- python3 tools/${DRV:-lloyd_loop}.py $N $D $K ${STEPS:-3} > $O/p4.log 2>&1 || exit 14
echo PMC_OK $TAG
