set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline --rccl --n-total 12500000 > gpurun_out/pd2.json 2> gpurun_out/pd2.err; echo "torchrun rc=$?"; wc -c gpurun_out/pd2.json; cat gpurun_out/pd2.json | cut -c1-300; grep -v amdgpu.ids gpurun_out/pd2.err | tail -20
