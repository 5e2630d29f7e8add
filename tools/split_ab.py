"""Per-step kernel times of the device loop at a BASELINE config (dev tool):
seeds, `warm` steps, then `steps` steps profiled one at a time: screen ms
(both kernels of the split bounded screen), the first kernel's ms, the whole
step's kernels, and the points re-read.
    python tools/split_ab.py [n] [d] [k] [warm] [steps]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clustering-driven-replication-strategy_amd"), REPO]
import _cdr  # noqa: E402
from cdr_dist import Comm, DeviceLloyd, seed_sharded  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
k = int(sys.argv[3]) if len(sys.argv) > 3 else 64
warm = int(sys.argv[4]) if len(sys.argv) > 4 else 5
steps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
ctx = _cdr.Context(0)
ctx.generate_points(n, 0, n, d, k, 0x5EED)
C = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
np.random.seed(0)
run = DeviceLloyd(ctx, C, -1.0, lambda g: ctx.get_rows([g])[0], n)
run.advance(warm)
rows = []
for s in range(steps):
    ctx.profile_reset(True)
    run.advance(1, chunk=1, chunk_max=1)
    p = ctx.profile_read()
    q = ctx.profile_read_sub()
    rows.append((warm + s + 1, p["screen_ms"] * 1e3, q["first_ms"] * 1e3 if q["steps"] else 0.0,
                 p["step_ms"] * 1e3, p["tight_points"]))
    ctx.profile_reset(False)
ctx.profile_reset(True)
ctx.synchronize()
t0 = time.perf_counter()
run.advance(steps, chunk=steps, chunk_max=steps)
ctx.synchronize()
wall = (time.perf_counter() - t0) / steps * 1e3
p = ctx.profile_read()
q = ctx.profile_read_sub()
ctx.profile_reset(False)
print("kernel", ctx.profile_kernel())
print("step  screen_us  first_us  step_us  reread")
for r in rows:
    print(f"{r[0]:4d} {r[1]:9.1f} {r[2]:9.1f} {r[3]:8.1f} {r[4]:9d}")
a = np.array([r[1:4] for r in rows])
print("mean (one-at-a-time)", np.round(a.mean(axis=0), 1))
print(f"batched {steps} more steps: screen {p['screen_ms'] / max(p['steps'], 1) * 1e3:.1f} us, "
      f"first {q['first_ms'] / max(q['steps'], 1) * 1e3:.1f} us, step kernels "
      f"{p['step_ms'] / max(p['steps'], 1) * 1e3:.1f} us, wall {wall * 1e3:.1f} us/step")
run.finish()
