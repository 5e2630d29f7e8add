"""Time k-means++ seeding steps (config-3 sized by default) for kernel tuning.
    CDR_SEED_STATS=1 python tools/seed_time.py [n] [d] [k]"""
import os
import sys
import time

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
t = time.perf_counter()
C = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
print(f"seed n={n} d={d} k={k}: {time.perf_counter() - t:.4f} s", flush=True)
