# PMC passes over the config-4 group-by (bucket and scatter kernels).
set -o pipefail
mkdir -p gpurun_out/pmc_c4
export TMPDIR=/tmp
A="bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/pmc_c4/p1 -o p1 --output-format csv -- python3 $A > gpurun_out/pmc_c4/p1.log 2>&1 || exit 11
timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/pmc_c4/p2 -o p2 --output-format csv -- python3 $A > gpurun_out/pmc_c4/p2.log 2>&1 || exit 12
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c4/p3 -o p3 --output-format csv -- python3 $A > gpurun_out/pmc_c4/p3.log 2>&1 || exit 13
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c4/p4 -o p4 --output-format csv -- python3 $A > gpurun_out/pmc_c4/p4.log 2>&1 || exit 14
python3 tools/pmc_summary.py gpurun_out/pmc_c4 --want gb_ > gpurun_out/pmc_c4.txt; tail -40 gpurun_out/pmc_c4.txt
echo ALL_OK
