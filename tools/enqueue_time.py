"""Host enqueue cost of the device-resident Lloyd loop against its GPU time
(dev tool): is a step bound by the host's launches (where capturing the step
chain in a hipGraph would pay) or by the GPU?  Times cdr_lloyd_enqueue_steps
(m steps: assign, all-reduce, finalize) to its return and to the end of the
GPU work, without and with a native RCCL communicator (world 1, whose
ncclAllReduce goes through RCCL's full launch path).
    python tools/enqueue_time.py [n] [m] [reps]"""
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clustering-driven-replication-strategy_amd"), REPO]

import torch  # noqa: E402  (first: libcdr then binds to torch's HIP runtime)
import torch.distributed as tdist  # noqa: E402

import _cdr  # noqa: E402
from cdr_dist import Comm, DeviceLloyd, bind_stream, seed_sharded  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 40
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
d, k = 16, 64

with socket.socket() as sk:
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                  MASTER_PORT=str(port))
torch.cuda.set_device(0)
tdist.init_process_group("nccl", device_id=torch.device("cuda", 0))
device = torch.device("cuda", 0)

for native in (False, True):
    ctx = _cdr.Context(0)
    bind_stream(ctx, device)
    ctx.generate_points(n, 0, n, d, k, 0x5EED)
    comm = Comm(tdist if native else None, device if native else None)
    if native and not comm.attach_native(ctx):
        raise SystemExit("no native communicator")
    C0 = seed_sharded(ctx, comm, 0, n, k, random_state=42)
    run = DeviceLloyd(ctx, C0, -1.0, lambda g: ctx.get_rows([g])[0], n, comm if native else None)
    run.advance(6)
    ctx.synchronize()
    for rep in range(reps):
        t0 = time.perf_counter()
        ctx.lloyd_enqueue_steps(m)
        t1 = time.perf_counter()
        ctx.synchronize()
        t2 = time.perf_counter()
        print(f"native_rccl={int(native)} rep {rep}: enqueue {(t1 - t0) / m * 1e6:.1f} us/step, "
              f"GPU done {(t2 - t0) / m * 1e6:.1f} us/step over {m} steps", flush=True)
    run.finish()
    ctx.close()
tdist.destroy_process_group()
