"""In-process timing of the bounded screen (screen32b) with parts switched off
(CDR_BOUNDS_DBG bits, experiments build only: 2 no fused fixup, 4 listed
points not decided, 8 no k-way screen, 16 stream only).  Results are garbage
while a bit is set; diagnostic tool, not a test.
    CDR_LIB=.../libcdr_exp.so python tools/bounds_ablate.py [n] [d] [k] [masks]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clustering-driven-replication-strategy_amd"), REPO]
import _cdr  # noqa: E402
from cdr_dist import Comm, DeviceLloyd, seed_sharded  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
k = int(sys.argv[3]) if len(sys.argv) > 3 else 64
# a mask "F<n>" sets CDR_FIX_ABL=n instead (the fused fixup's parts: 1 no moves,
# 2 no fallback, 4 no flush) with every bound part on
masks = sys.argv[4].split(",") if len(sys.argv) > 4 else "0,2,4,8,16,6".split(",")
ctx = _cdr.Context(0)
ctx.generate_points(n, 0, n, d, k, 0x5EED)
C = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
np.random.seed(0)
run = DeviceLloyd(ctx, C, -1.0, lambda g: ctx.get_rows([g])[0], n)
run.advance(6)
res = {m: [] for m in masks}
first = {}
for rnd in range(3):
    for m in masks:
        fix = m.startswith("F")
        os.environ["CDR_BOUNDS_DBG"] = "0" if fix else m
        os.environ["CDR_FIX_ABL"] = m[1:] if fix else "0"
        ctx.profile_reset(True)
        run.advance(4, chunk=4, chunk_max=4)
        p = ctx.profile_read()
        q = ctx.profile_read_sub()
        res[m].append(p["screen_ms"] / max(p["steps"], 1))
        first.setdefault(m, []).append(q["first_ms"] / max(q["steps"], 1))
        if not m.startswith("F") and int(m) & 128:  # candidates of the exact pass (high word)
            print(f"mask {m}: steps {p['steps']} tight {p['tight_points'] & 0xFFFFFFFF} "
                  f"candidates {p['tight_points'] >> 32} profile {p}")
        ctx.profile_reset(False)
os.environ["CDR_BOUNDS_DBG"] = "0"
os.environ["CDR_FIX_ABL"] = "0"
for m in masks:
    print(f"mask {m:>4}: screen32b {np.median(res[m]) * 1e3:8.1f} us  first kernel "
          f"{np.median(first[m]) * 1e3:6.1f} us (rounds {[round(x * 1e3, 1) for x in res[m]]})")
run.finish()
