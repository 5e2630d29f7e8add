# Per-rank step cost at the 2/4/8-GPU shard sizes on one GPU, and the RCCL
# code path of bench.py at world size 1 (torchrun, --dist).
set -o pipefail
mkdir -p gpurun_out
for n in 50000000 25000000 12500000; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --n-total $n > gpurun_out/probe_$n.json 2> gpurun_out/probe_$n.err || { echo FAIL $n; tail -20 gpurun_out/probe_$n.err; exit 1; }
  python3 -c "import json,sys; r=json.load(open('gpurun_out/probe_$n.json')); print($n, 'ms/step %.4f kernel %.4f step_kernels %.4f seed_s %.3f' % (r['ms_per_step'], r['roofline']['kernel_ms'], r['step_kernels_ms'], r['seed_s']))"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline --rccl --n-total 12500000 > gpurun_out/probe_dist.json 2> gpurun_out/probe_dist.err || { echo DISTFAIL; tail -30 gpurun_out/probe_dist.err; exit 2; }
python3 -c "import json,sys; r=json.load(open('gpurun_out/probe_dist.json')); print('dist 12.5M', 'ms/step %.4f kernel %.4f step_kernels %.4f seed_s %.3f' % (r['ms_per_step'], r['roofline']['kernel_ms'], r['step_kernels_ms'], r['seed_s']))"
