"""Time k-means++ seeding (config-3 sized by default) for kernel tuning; runs
it twice (the first run also builds the fp16 copy) and prints a checksum of
the centres so variants can be compared bit for bit.
    python tools/seed_time.py [n] [d] [k]"""
import hashlib
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clustering-driven-replication-strategy_amd"), REPO]
import _cdr  # noqa: E402
from cdr_dist import Comm, seed_sharded  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
k = int(sys.argv[3]) if len(sys.argv) > 3 else 64
ctx = _cdr.Context(0)
ctx.generate_points(n, 0, n, d, k, 0x5EED)
ctx.synchronize()
for rep in range(2):
    t = time.perf_counter()
    C = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
    dt = time.perf_counter() - t
    h = hashlib.sha256(np.ascontiguousarray(C).tobytes()).hexdigest()[:16]
    print(f"seed n={n} d={d} k={k} run {rep}: {dt:.4f} s centres {h}", flush=True)
