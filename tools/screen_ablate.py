"""In-process A/B timing of the screen kernel with parts switched off
(interleaved rounds, HIP-event timings).  Diagnostic tool, not a test.
Needs the experiments build:  make -C .../csrc OUT=../libcdr_exp.so
OBJDIR=../build_exp EXTRA=-DCDR_EXPERIMENTS  and  CDR_LIB=<that .so>."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clustering-driven-replication-strategy_amd"), REPO]
import _cdr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
k = int(sys.argv[3]) if len(sys.argv) > 3 else 64
masks = [int(m) for m in (sys.argv[4].split(",") if len(sys.argv) > 4 else "0,1,2,3,4,8,15".split(","))]
ctx = _cdr.Context(0)
ctx.generate_points(n, 0, n, d, k, 0x5EED)
if os.environ.get("ABLATE_RANDOM_C"):
    rng = np.random.default_rng(0)
    C = ctx.get_rows(np.sort(rng.choice(n, k, replace=False)))
else:  # the bench's centroids: k-means++ then a few Lloyd steps
    from cdr_dist import Comm, ShardedLloyd, seed_sharded

    C = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
    lloyd = ShardedLloyd(ctx, Comm(), n, 0)
    np.random.seed(0)
    C = lloyd.run_host(C, 4, tol=-1.0)
for _ in range(2):
    ctx.lloyd_step(C)
res = {m: [] for m in masks}
steps = {m: [] for m in masks}
for rnd in range(5):
    for m in masks:
        ctx._lib.cdr_debug_screen_ablate(ctx._h, m)
        ctx.profile_reset(True)
        for _ in range(3):
            ctx.lloyd_step(C)
        p = ctx.profile_read()
        res[m].append(p["screen_ms"] / p["steps"])
        steps[m].append(p["step_ms"] / p["steps"])
ctx._lib.cdr_debug_screen_ablate(ctx._h, 0)
alg = n * (4 * d + 4)
for m in masks:
    med = float(np.median(res[m]))
    print(f"ablate={m:2d} screen median {med:.3f} ms (min {min(res[m]):.3f})  "
          f"GB/s(alg) {alg / med / 1e6:.0f}  step median {np.median(steps[m]):.3f} ms")
ctx.profile_reset(True)
ctx.lloyd_step(C)
print("fallback points", ctx.fallback_count(), "step", ctx.profile_read())
