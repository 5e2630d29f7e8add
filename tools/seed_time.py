"""Time k-means++ seeding (config-3 sized by default) for kernel tuning; runs
it `reps` times (the first run also pays the one-time allocations and the
fp16 / row-major copies) and prints a checksum of the centres so variants can
be compared bit for bit.
    python tools/seed_time.py [n] [d] [k] [reps]
CDR_PKG: another build of the package (A/B of two library versions on one box)."""
import hashlib
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.environ.get("CDR_PKG") or os.path.join(REPO, "clustering-driven-replication-strategy_amd")
sys.path[:0] = [PKG, REPO]
import _cdr  # noqa: E402
from cdr_dist import Comm, seed_sharded  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
k = int(sys.argv[3]) if len(sys.argv) > 3 else 64
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
ctx = _cdr.Context(0)
ctx.generate_points(n, 0, n, d, k, 0x5EED)
ctx.synchronize()
for rep in range(reps):
    t = time.perf_counter()
    C = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
    dt = time.perf_counter() - t
    h = hashlib.sha256(np.ascontiguousarray(C).tobytes()).hexdigest()[:16]
    print(f"seed n={n} d={d} k={k} run {rep}: {dt:.4f} s centres {h}", flush=True)
