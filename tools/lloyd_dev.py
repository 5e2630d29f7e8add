"""Device-loop Lloyd driver for rocprofv3 runs: k-means++ seeds on the device,
then `steps` device-loop steps (the bench's path, cdr_dist.DeviceLloyd).
    python tools/lloyd_dev.py [n] [d] [k] [steps]"""
import os
import sys

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
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 8
ctx = _cdr.Context(0)
ctx.generate_points(n, 0, n, d, k, 0x5EED)
C = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
np.random.seed(0)
run = DeviceLloyd(ctx, C, -1.0, lambda g: ctx.get_rows([g])[0], n)
run.advance(steps)
C, st = run.finish()
print("kernel", ctx.profile_kernel(), "steps", st["steps"], "inertia", st["inertia"])
