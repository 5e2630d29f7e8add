"""Minimal Lloyd-step driver for rocprofv3 runs (no seeding, fixed centroids).
    python tools/lloyd_loop.py [n] [d] [k] [steps]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clustering-driven-replication-strategy_amd"), REPO]
import _cdr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
k = int(sys.argv[3]) if len(sys.argv) > 3 else 64
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
ctx = _cdr.Context(0)
ctx.generate_points(n, 0, n, d, k, 0x5EED)
C = ctx.get_rows(np.sort(np.random.default_rng(0).choice(n, k, replace=False)))
for _ in range(steps):
    out = ctx.lloyd_step(C)
print("fallback", ctx.fallback_count(), "count sum", int(out[:, d].sum()))
