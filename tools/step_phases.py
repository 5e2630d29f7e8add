"""Host-side phase timing of one sharded Lloyd step (world size 1, RCCL path).
    WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 \
        python tools/step_phases.py [n]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clustering-driven-replication-strategy_amd"), REPO]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
import numpy as np  # noqa: E402

import _cdr  # noqa: E402
from cdr_dist import Comm, ShardedLloyd, seed_sharded  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
d, k = 16, 64
dev = torch.device("cuda", 0)
ctx = _cdr.Context(0)
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
ctx.generate_points(n, 0, n, d, k, 0x5EED)
comm = Comm(dist, dev)
C = seed_sharded(ctx, comm, 0, n, k, random_state=42)
L = ShardedLloyd(ctx, comm, n, 0)
buf = torch.empty(k * (d + 1), dtype=torch.int64, device=dev)
for _ in range(5):
    C, _ = L.step(C, L.row)
torch.cuda.synchronize()
T = np.zeros(6)
steps = 50
for _ in range(steps):
    t0 = time.perf_counter()
    ctx.lloyd_step_device(C, buf.data_ptr())
    t1 = time.perf_counter()
    dist.all_reduce(buf)
    t2 = time.perf_counter()
    acc = buf.view(k, d + 1).cpu().numpy()
    t3 = time.perf_counter()
    counts = acc[:, d]
    sums = np.ldexp(acc[:, :d].astype(np.float64), -L.S)
    new = sums / counts[:, None].astype(np.float64)
    for j in np.flatnonzero(counts == 0):
        new[j] = L.row(np.random.randint(0, n))
    shift = np.linalg.norm(new - C)
    C = new
    t4 = time.perf_counter()
    T += [t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0, 0]
T /= steps
print("us per step: enqueue_step %.1f allreduce_enqueue %.1f wait+D2H %.1f numpy %.1f total %.1f"
      % tuple(T[:5] * 1e6))
ctx.profile_reset(True)
for _ in range(steps):
    C, _ = L.step(C, L.row)
p = ctx.profile_read()
print("device: screen %.1f us, step kernels %.1f us" % (p["screen_ms"] / p["steps"] * 1e3,
                                                         p["step_ms"] / p["steps"] * 1e3))
dist.destroy_process_group()
