# PMC pass over the config-4 group-by kernels (one counter set per run).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc4a -o run --output-format csv -- python3 -u bench.py --config 4 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc4a.log 2>&1 || { echo PMC_A_FAIL; tail -20 gpurun_out/pmc4a.log; exit 2; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc4b -o run --output-format csv -- python3 -u bench.py --config 4 --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc4b.log 2>&1 || { echo PMC_B_FAIL; tail -20 gpurun_out/pmc4b.log; exit 3; }
python3 tools/pmc_summary.py gpurun_out/pmc4a gpurun_out/pmc4b --want gb_ > gpurun_out/pmc4_summary.txt
cat gpurun_out/pmc4_summary.txt
echo ALL_OK
