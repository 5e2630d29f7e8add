set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
P="python3 tools/lloyd_loop.py 100000000 16 64 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc/p1 -o p1 --output-format csv -- $P > gpurun_out/pmc/p1.log 2>&1 || exit 11
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d gpurun_out/pmc/p2 -o p2 --output-format csv -- $P > gpurun_out/pmc/p2.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/p3 -o p3 --output-format csv -- $P > gpurun_out/pmc/p3.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/p4 -o p4 --output-format csv -- $P > gpurun_out/pmc/p4.log 2>&1 || exit 14
echo PMC_OK
