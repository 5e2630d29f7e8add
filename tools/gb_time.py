"""Wall time of the config-4 group-by step (dev tool; bench.py's config-4 leg
without the bench around it): the device access simulator's log for nf files,
then `steps` resident group-by steps after `warm` untimed ones, `reps` times.
    python tools/gb_time.py [n_events] [steps] [warm] [reps]
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

n_ev = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 2
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
sys.path.insert(0, REPO)
import bench  # noqa: E402

nf_cfg, duration, nclients, _ = bench.FEATURES_CFG
nf = max(1, int(n_ev / bench.EVENTS_PER_FILE))
ctx = _cdr.Context(0)
ne = ctx.features_simulate(nf, duration, nclients, seed=0x5EED, file_begin=0)
for rep in range(reps):
    for _ in range(warm):
        ctx.features_aggregate_resident(to_host=False)
    ctx.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        ctx.features_aggregate_resident(to_host=False)
    ctx.synchronize()
    dt = (time.perf_counter() - t) / steps
    rows = ctx.features_aggregate_resident(to_host=True)
    h = hashlib.sha256(np.ascontiguousarray(rows[0]).tobytes()).hexdigest()[:16]
    print(f"groupby events={ne} files={nf} rep {rep}: {dt * 1e3:.4f} ms/step, rows {h}", flush=True)
ctx.close()
