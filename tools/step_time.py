"""Wall time per device-loop step with and without the HIP-event profile
(dev tool): k-means++ seeds on the device, `warm` untimed steps, then
`steps` timed steps per mode, the loop restarted from the same seeds.
    python tools/step_time.py [n] [d] [k] [steps] [warm]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# CDR_PKG: another build of the package (A/B of two library versions on one box)
PKG = os.environ.get("CDR_PKG") or os.path.join(REPO, "clustering-driven-replication-strategy_amd")
sys.path[:0] = [PKG, REPO]
import _cdr  # noqa: E402
from cdr_dist import Comm, DeviceLloyd, seed_sharded  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
k = int(sys.argv[3]) if len(sys.argv) > 3 else 64
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
warm = int(sys.argv[5]) if len(sys.argv) > 5 else 5
ctx = _cdr.Context(0)
ctx.generate_points(n, 0, n, d, k, 0x5EED)
C0 = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
for rep in range(2):
    for every in (0, 4, 1):
        np.random.seed(0)
        run = DeviceLloyd(ctx, C0, -1.0, lambda g: ctx.get_rows([g])[0], n)
        run.advance(warm)
        ctx.synchronize()
        ctx.profile_reset(every > 0, every=max(every, 1))
        t0 = time.perf_counter()
        run.advance(steps, chunk=steps, chunk_max=steps)
        ctx.synchronize()
        el = time.perf_counter() - t0
        prof = ctx.profile_read()
        ctx.profile_reset(False)
        run.finish()
        ps = max(prof["steps"], 1)
        print(f"rep {rep} events every {every}: {el / steps * 1e3:.4f} ms/step wall; "
              f"screen {prof['screen_ms'] / ps * 1e3:.1f} us, step kernels {prof['step_ms'] / ps * 1e3:.1f} us "
              f"over {prof['steps']} profiled steps", flush=True)
