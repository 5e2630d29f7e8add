set -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 python -u tools/dbg/gb_cap.py 300000 4 60 > gpurun_out/dbg_wave_big.log 2>&1; echo "wave big rc=$?"
cat gpurun_out/dbg_wave_big.log
