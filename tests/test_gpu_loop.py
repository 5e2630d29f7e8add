"""GPU parity of the device-resident Lloyd loop (csrc/loop.hip) and of the
BASELINE configurations at their full sizes.

The loop replaces the host's per-step means / reseed / shift
(src/kmeans_plusplus.py:31-48) by device kernels; these tests check that it
takes the reference's decisions: bit-identical centroids and labels against
the pinned oracle, the empty-cluster reseed and the fp16-range host take-over
included, and the north_star inertia within 1e-5 (checked at 1e-9)."""
import os

import numpy as np
import pytest

from oracle import kmeans_oracle as ko
from oracle import synth

pytestmark = pytest.mark.gpu


def _loop(ctx, C0, max_iter, tol, X=None, n=None):
    from cdr_dist import device_lloyd

    reseed = (lambda g: X[g]) if X is not None else (lambda g: ctx.get_rows([g])[0])
    return device_lloyd(ctx, np.array(C0, dtype=np.float64), max_iter, tol, reseed,
                        n if n is not None else X.shape[0])


@pytest.mark.parametrize("n,d,k", [(200000, 16, 64), (90000, 8, 16), (50000, 5, 7),
                                   (40000, 24, 33), (20000, 64, 300), (30000, 40, 700),
                                   (12000, 9, 1100)])
def test_loop_matches_oracle_fixed_steps(ctx, n, d, k):
    """tol disabled: max_iter steps; screen32 shapes and the large-k shapes
    (screen_big) use device-built plans, the others (e.g. d = 24, k = 33) the
    host-plan path through the same loop."""
    X = synth.generate(n, 0, n, d, k, 31 * n + d)
    ctx.load_points(X)
    rng = np.random.default_rng(k)
    C0 = X[np.sort(rng.choice(n, k, replace=False))]
    np.random.seed(5)
    C, st = _loop(ctx, C0, 4, -1.0, X)
    np.random.seed(5)
    C_ref, lab_ref, used, _ = ko.lloyd(X, C0, 4, -1.0)
    assert st["steps"] == 4
    np.testing.assert_array_equal(ctx.labels(), lab_ref)
    np.testing.assert_array_equal(C, C_ref)
    want = ko.inertia(X, used, lab_ref)
    assert abs(st["inertia"] - want) <= 1e-9 * want, (st["inertia"], want)


def test_loop_empty_cluster_far_centroid_and_convergence(ctx):
    """One centroid far outside the fp16 screen range: the device plan stops
    the loop (host-plan step), the cluster is empty (the host draws
    np.random.randint and reseeds it, :43), then the loop runs to tol."""
    n, d, k = 120000, 16, 24
    X = synth.generate(n, 0, n, d, k, 4242)
    ctx.load_points(X)
    C0 = X[:k].copy()
    C0[3] = 1.0e4
    np.random.seed(11)
    C, st = _loop(ctx, C0, 400, 1e-4, X)
    np.random.seed(11)
    C_ref, lab_ref, used, steps = ko.lloyd(X, C0, 400, 1e-4)
    np.testing.assert_array_equal(C, C_ref)
    np.testing.assert_array_equal(ctx.labels(), lab_ref)
    assert st["steps"] == steps < 400  # stopped by tol at the reference's step


def test_loop_float32_points_round_means(ctx):
    """X float32: the centroids keep X's dtype (np.empty_like), as the
    drop-in's host loop always did."""
    import kmeans_plusplus as kp

    n, d, k = 30000, 8, 12
    X = synth.generate(n, 0, n, d, k, 77).astype(np.float32)
    np.random.seed(1)
    C, lab = kp.kmeans(X, k, random_state=3, max_iter=6, context=ctx)
    assert C.dtype == np.float32
    X64 = X.astype(np.float64)
    # the drop-in seeds in fp64 on float32 data: rows of X
    Cr = ko.kmeans_plusplus_init(X64, k, random_state=3).astype(np.float32)
    np.random.seed(1)
    for _ in range(6):
        labr = ko.assign(X64, Cr.astype(np.float64))
        new = np.empty_like(Cr)
        for j in range(k):
            m = labr == j
            new[j] = X64[m].mean(axis=0) if m.any() else X[np.random.randint(0, n)]
        shift = np.linalg.norm(new - Cr)
        Cr = new
        if shift < 1e-4:
            break
    np.testing.assert_array_equal(C, Cr)
    np.testing.assert_array_equal(lab, labr)


def _config_common(ctx, n, d, k, steps, sample, seed=0x5EED):
    from cdr_dist import Comm, seed_sharded

    ctx.generate_points(n, 0, n, d, k, seed)
    C0 = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
    np.random.seed(0)
    C_prev, _ = _loop(ctx, C0, steps - 1, -1.0, n=n)
    C, st = _loop(ctx, C_prev, 1, -1.0, n=n)  # the last assignment used C_prev
    lab = ctx.labels()
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(n, sample, replace=False))
    np.testing.assert_array_equal(lab[idx], ko.assign(ctx.get_rows(idx), C_prev))
    return C_prev, C, st, lab


def test_config3_full_size(ctx):
    """BASELINE config 3: 100M x 16, k = 64 (device generator, k-means++
    seeding, device loop).  Labels of a 50k sample = the oracle; the int64
    sums of two sampled clusters = a NumPy recompute; counts sum to n; the
    means the loop moved to = the host's division of those sums; one shard =
    two shards."""
    import _cdr
    from cdr_dist import shard_rows

    n, d, k = 100_000_000, 16, 64
    C_prev, C, st, lab = _config_common(ctx, n, d, k, 3, 50_000)
    acc = ctx.lloyd_step(C_prev)  # the same assignment again: its sums
    np.testing.assert_array_equal(ctx.labels(), lab)
    assert acc[:, d].sum() == n
    np.testing.assert_array_equal(np.bincount(lab, minlength=k), acc[:, d])
    S = ctx.info()["scale_bits"]
    np.testing.assert_array_equal(C, np.ldexp(acc[:, :d].astype(np.float64), -S) /
                                  acc[:, d:].astype(np.float64))
    for j in np.random.default_rng(1).choice(k, 2, replace=False):
        rows = ctx.get_rows(np.flatnonzero(lab == j))
        np.testing.assert_array_equal(np.ldexp(rows, S).astype(np.int64).sum(axis=0),
                                      acc[j, :d])
    b = _cdr.Context(ctx.device)
    try:
        parts = []
        for r in range(2):
            begin, m = shard_rows(n, 2, r)
            b.generate_points(n, begin, m, d, k, 0x5EED)
            parts.append((b.lloyd_step(C_prev), b.labels()))
        np.testing.assert_array_equal(parts[0][0] + parts[1][0], acc)
        np.testing.assert_array_equal(np.concatenate([parts[0][1], parts[1][1]]), lab)
    finally:
        b.close()


def test_config3_every_label_exact(ctx, monkeypatch):
    """all 100M labels of a DELTA step on the default screen
    (pruned screen32p + queued k-way MFMA screen + fixup32) equal the exact
    fp64 NumPy-order assignment of the same centroids (assign_exact_all on
    every point, CDR_EXACT_ASSIGN), and so do the int64 sums."""
    n, d, k = 100_000_000, 16, 64
    C_prev, C, st, lab = _config_common(ctx, n, d, k, 3, 2_000)
    acc = ctx.lloyd_step(C_prev)  # host-plan DELTA step on the same centroids
    np.testing.assert_array_equal(ctx.labels(), lab)
    monkeypatch.setenv("CDR_EXACT_ASSIGN", "1")
    acc_x = ctx.lloyd_step(C_prev)
    monkeypatch.delenv("CDR_EXACT_ASSIGN")
    lab_x = ctx.labels()
    assert (lab_x != lab).sum() == 0
    np.testing.assert_array_equal(acc_x, acc)


def test_config5_full_size_and_scoring(ctx):
    """BASELINE config 5: 50M x 64, k = 1024 (screen_big MFMA path) + replica
    scoring per cluster: labels of a 10k sample = the oracle, sums of two
    sampled clusters = a NumPy recompute, medians of two sampled clusters =
    np.median, and classify_labels = classify on the same medians."""
    import warnings

    from scoring import ClusterClassifier

    n, d, k = 50_000_000, 64, 1024
    C_prev, C, st, lab = _config_common(ctx, n, d, k, 2, 10_000)
    assert ctx.profile_kernel().startswith("screen_big")
    acc = ctx.lloyd_step(C_prev)
    assert acc[:, d].sum() == n
    S = ctx.info()["scale_bits"]
    med = ctx.medians_by_label(k)
    for j in np.random.default_rng(2).choice(np.flatnonzero(acc[:, d] > 0), 2, replace=False):
        rows = ctx.get_rows(np.flatnonzero(lab == j))
        np.testing.assert_array_equal(np.ldexp(rows, S).astype(np.int64).sum(axis=0),
                                      acc[j, :d])
        np.testing.assert_array_equal(med[j], np.median(rows, axis=0))
    names = [f"f{i}" for i in range(d)]
    gm = {nm: 0.5 for nm in names}
    w = {c: {nm: 1.0 for nm in names} for c in ("Hot", "Shared", "Moderate", "Archival")}
    dirs = {"Hot": {nm: 1 for nm in names}, "Shared": {nm: 1 for nm in names},
            "Moderate": {nm: 0 for nm in names}, "Archival": {nm: -1 for nm in names}}
    clf = ClusterClassifier(gm, w, dirs, {"Hot": 3, "Shared": 2, "Moderate": 1, "Archival": 4},
                            context=ctx)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        got = clf.classify_labels(k, names)
    want = {f"C{j}": clf.classify_cluster({nm: np.float64(med[j, i]) for i, nm in enumerate(names)})
            for j in range(k)}
    assert got == want


@pytest.mark.parametrize("n,d,k", [(300_000, 16, 64), (60_000, 64, 300), (40_000, 24, 33)])
def test_sharded_device_loop_two_contexts(n, d, k):
    """The multi-GPU step of bench.py / cdr_dist.DeviceLloyd (csrc/loop.hip with
    a device all-reduce buffer: enqueue_assign -> SUM -> enqueue_finalize)
    emulated with two contexts on one GPU and a device-tensor sum in place of
    RCCL: centroids and labels equal the single-context loop's (screen32,
    large-k DELTA and host-plan shapes)."""
    import torch

    import _cdr
    from cdr_dist import Comm, device_lloyd, seed_sharded

    X = synth.generate(n, 0, n, d, k, 7 * n + d)
    steps = 5
    full = _cdr.Context(0)
    try:
        full.load_points(X)
        # k-means++ centres (as bench.py): no cluster empties in these steps,
        # so no host reseed is involved
        C0 = np.asarray(seed_sharded(full, Comm(), 0, n, k, random_state=42), dtype=np.float64)
        np.random.seed(1)
        C_ref, st_ref = device_lloyd(full, C0, steps, -1.0, lambda g: X[g], n)
        lab_ref = full.labels()
    finally:
        full.close()
    assert st_ref["steps"] == steps and st_ref["running"], st_ref
    cut = (n // 2) // 8192 * 8192
    ctxs = [_cdr.Context(0), _cdr.Context(0)]
    try:
        ctxs[0].load_points(X[:cut])
        ctxs[1].load_points(X[cut:])
        ref = C0[0].copy()
        x2 = ctxs[0].points_sqdev(ref) + ctxs[1].points_sqdev(ref)
        bufs = [torch.zeros(k * (d + 1), dtype=torch.int64, device="cuda") for _ in ctxs]
        for c in ctxs:
            c.lloyd_begin(C0, -1.0, ref, x2)
        for _ in range(steps):
            for c, b in zip(ctxs, bufs):
                c.lloyd_enqueue_assign(b.data_ptr())
            for c in ctxs:
                c.synchronize()
            tot = bufs[0] + bufs[1]
            for b in bufs:
                b.copy_(tot)
            torch.cuda.synchronize()
            for c, b in zip(ctxs, bufs):
                c.lloyd_enqueue_finalize(b.data_ptr())
        sts = [c.lloyd_status() for c in ctxs]
        Cs = [c.lloyd_read()[0] for c in ctxs]
        labs = np.concatenate([c.labels() for c in ctxs])
        for c in ctxs:
            c.lloyd_end()
    finally:
        for c in ctxs:
            c.close()
    assert all(s["steps"] == steps and s["running"] for s in sts), sts
    np.testing.assert_array_equal(Cs[0], C_ref)
    np.testing.assert_array_equal(Cs[1], C_ref)
    np.testing.assert_array_equal(labs, lab_ref)
    assert abs(sts[0]["inertia"] - st_ref["inertia"]) <= 1e-9 * st_ref["inertia"]


def _two_context_loop(parts, C0, steps, unify, n_total):
    """enqueue_assign -> device-tensor SUM -> enqueue_finalize on one context
    per shard (the multi-GPU step emulated on one GPU); returns the contexts'
    statuses, centroids and labels."""
    import torch

    import _cdr
    from cdr_dist import unify_points

    k, d = C0.shape
    ctxs = [_cdr.Context(0) for _ in parts]
    try:
        for c, X in zip(ctxs, parts):
            c.load_points(X)
        if unify:  # cdr_dist.unify_points with the MIN / MAX all-reduce done here
            sts = [c.points_stats() for c in ctxs]
            dd = (sts[0].size - 3) // 2
            g = np.concatenate([np.minimum(*[s[:dd] for s in sts]),
                                np.maximum(*[s[dd:] for s in sts])])
            for c in ctxs:
                c.points_restat(g, n_total)
        ref = C0[0].copy()
        x2 = sum(c.points_sqdev(ref) for c in ctxs)
        bufs = [torch.zeros(k * (d + 1), dtype=torch.int64, device="cuda") for _ in ctxs]
        for c in ctxs:
            c.lloyd_begin(C0, -1.0, ref, x2)
        for _ in range(steps):
            for c, b in zip(ctxs, bufs):
                c.lloyd_enqueue_assign(b.data_ptr())
            for c in ctxs:
                c.synchronize()
            tot = sum(bufs[1:], bufs[0].clone())
            for b in bufs:
                b.copy_(tot)
            torch.cuda.synchronize()
            for c, b in zip(ctxs, bufs):
                c.lloyd_enqueue_finalize(b.data_ptr())
        sts = [c.lloyd_status() for c in ctxs]
        Cs = [c.lloyd_read()[0] for c in ctxs]
        labs = np.concatenate([c.labels() for c in ctxs])
        for c in ctxs:
            c.lloyd_end()
    finally:
        for c in ctxs:
            c.close()
    return sts, Cs, labs


def test_unified_transform_two_shards_of_different_ranges(ctx):
    """each shard used to take its screen transform
    (mu, sigma) from its own ranges, so the fp16 range guard of the device
    plan could stop one rank's loop and not the other's.  Shard 0 holds
    points in [0, 2^-10), shard 1 in [0, 1): with per-shard transforms the
    centroids from shard 1 are out of shard 0's fp16 range (its loop stops
    for the host plan at once); with cdr_dist.unify_points both use the
    global transform, run every step, and equal the single-context loop."""
    from cdr_dist import device_lloyd, seed_sharded, Comm

    n, d, k = 2 * 65536, 16, 32
    X = synth.generate(n, 0, n, d, k, 99)
    X[: n // 2] = np.ldexp(np.floor(np.ldexp(X[: n // 2], 14)), -24)  # same 2^-24 grid
    ctx.load_points(X)
    C0 = np.asarray(seed_sharded(ctx, Comm(), 0, n, k, random_state=42), dtype=np.float64)
    np.random.seed(1)
    C_ref, st_ref = device_lloyd(ctx, C0, 5, -1.0, lambda g: X[g], n)
    lab_ref = ctx.labels()
    assert st_ref["steps"] == 5 and st_ref["running"], st_ref
    parts = [X[: n // 2], X[n // 2:]]
    sts, _, _ = _two_context_loop(parts, C0, 1, False, n)
    # the divergence being fixed: shard 0's own transform stops its loop for
    # the host plan at once (shard 1, summing sums of two scales, is garbage)
    assert not sts[0]["running"] and sts[0]["reason"] == ctx.LL_HOST_PLAN, sts
    sts, Cs, labs = _two_context_loop(parts, C0, 5, True, n)
    assert all(s["steps"] == 5 and s["running"] for s in sts), sts
    np.testing.assert_array_equal(Cs[0], C_ref)
    np.testing.assert_array_equal(Cs[1], C_ref)
    np.testing.assert_array_equal(labs, lab_ref)


def test_native_rccl_step_world1(ctx):
    """The loop's all-reduce issued from C (csrc/comm.hip): a one-rank RCCL
    communicator on the context, cdr_lloyd_enqueue_steps runs assign ->
    ncclAllReduce -> finalize per step; results equal the loop without it."""
    import _cdr
    from cdr_dist import device_lloyd

    n, d, k = 300_000, 16, 64
    X = synth.generate(n, 0, n, d, k, 1234)
    rng = np.random.default_rng(3)
    C0 = X[np.sort(rng.choice(n, k, replace=False))]
    ctx.load_points(X)
    np.random.seed(2)
    C_ref, st_ref = device_lloyd(ctx, C0, 6, -1.0, lambda g: X[g], n)
    lab_ref = ctx.labels()
    b = _cdr.Context(ctx.device)
    try:
        b.load_points(X)
        b.comm_init(_cdr.comm_unique_id(), 1, 0)
        np.random.seed(2)
        C, st = device_lloyd(b, C0, 6, -1.0, lambda g: X[g], n)
        np.testing.assert_array_equal(C, C_ref)
        np.testing.assert_array_equal(b.labels(), lab_ref)
        assert st["steps"] == st_ref["steps"] == 6
        assert st["inertia"] == st_ref["inertia"]
        b.comm_destroy()
    finally:
        b.close()
