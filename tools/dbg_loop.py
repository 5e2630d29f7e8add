import sys, os
sys.path[:0] = ["clustering-driven-replication-strategy_amd", "."]
import numpy as np
import _cdr
from cdr_dist import device_lloyd
from oracle import kmeans_oracle as ko, synth
ctx = _cdr.Context(0)
n, d, k = 120000, 16, 24
X = synth.generate(n, 0, n, d, k, 4242)
ctx.load_points(X)
C0 = X[:k].copy()
C0[3] = 1.0e4
for it in (1, 2, 3, 4):
    np.random.seed(11)
    C, st = device_lloyd(ctx, C0.copy(), it, 1e-4, lambda g: X[g], n)
    np.random.seed(11)
    Cr, lr, used = ko.lloyd(X, C0, it, 1e-4)
    lab = ctx.labels()
    print(it, st, "C eq", np.array_equal(C, Cr), "lab eq", np.array_equal(lab, lr),
          "nbad", int((lab != lr).sum()), "maxdiff", float(np.abs(C - Cr).max()), flush=True)
# host-plan single step directly
ctx.load_points(X)
acc = ctx.lloyd_step(C0)
lr = ko.assign(X, C0)
print("legacy step labels eq", np.array_equal(ctx.labels(), lr), ctx.profile_kernel(), flush=True)
_, exp = ko.lloyd_partials(X, C0, ctx.info()["scale_bits"])
print("legacy sums eq", np.array_equal(acc, exp))
