# RCCL path at world size 1, config 5, config 4 and the ingest leg.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --rccl --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench3_rccl.json 2> gpurun_out/bench3_rccl.err || { echo RCCL_FAIL; tail -20 gpurun_out/bench3_rccl.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/bench3_rccl.json'));print('rccl',d['ms_per_step'],d['roofline']['kernel_ms'],d['n_gpus'])"
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo BENCH5_FAIL; tail -20 gpurun_out/bench5.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/bench5.json'));print('c5',d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['seed_s'])"
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo BENCH4_FAIL; tail -20 gpurun_out/bench4.err; exit 4; }
python3 -c "import json;d=json.load(open('gpurun_out/bench4.json'));print('c4',d['ms_per_step'],d['roofline']['frac'],d['value'])"
echo ALL_OK
