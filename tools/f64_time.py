"""Wall time of the device-resident F64 Lloyd steps (dev tool; bench.py's F64
leg without the bench around it): blobs from the device generator, min-max
normalised on the host (src/main.py:81), loaded in F64 mode, then `steps`
steps of cdr_lloyd_f64_run after `warm` untimed ones, `reps` times.
    python tools/f64_time.py [n] [d] [k] [steps] [warm] [reps]
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 5
k = int(sys.argv[3]) if len(sys.argv) > 3 else 16
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
warm = int(sys.argv[5]) if len(sys.argv) > 5 else 2
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3

g = _cdr.Context(0)
g.generate_points(n, 0, n, d, k, 0x5EED)
X = g.get_rows(np.arange(n, dtype=np.int64))
g.close()
mn, mx = X.min(axis=0), X.max(axis=0)
X = (X - mn) / (mx - mn)
ctx = _cdr.Context(0)
ctx.load_points(X)
assert ctx.info()["mode"] == _cdr.MODE_F64
C0 = X[np.sort(np.random.default_rng(42).choice(n, k, replace=False))].copy()
del X
for rep in range(reps):
    C, applied, _, _, _ = ctx.lloyd_f64_run(C0, warm, -1.0)
    ctx.synchronize()
    t = time.perf_counter()
    C, applied, _, _, _ = ctx.lloyd_f64_run(C, steps, -1.0)
    ctx.synchronize()
    dt = time.perf_counter() - t
    h = hashlib.sha256(np.ascontiguousarray(C).tobytes()).hexdigest()[:16]
    print(f"f64 n={n} d={d} k={k} rep {rep}: {dt / steps * 1e3:.4f} ms/step over {applied} steps, "
          f"centres {h}", flush=True)
ctx.close()
