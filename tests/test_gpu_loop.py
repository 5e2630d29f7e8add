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
    """X float32: the reference's float32 arithmetic (float32 seeding, norms
    and sequential float32 means; the centroids keep X's dtype) — the oracle
    on the same float32 X, bit for bit."""
    import kmeans_plusplus as kp

    n, d, k = 30000, 8, 12
    X = synth.generate(n, 0, n, d, k, 77).astype(np.float32)
    np.random.seed(1)
    C, lab = kp.kmeans(X, k, random_state=3, max_iter=6, context=ctx)
    assert C.dtype == np.float32
    np.random.seed(1)
    Cr, labr = ko.kmeans(X, k, random_state=3, max_iter=6)
    assert Cr.dtype == np.float32
    np.testing.assert_array_equal(C, Cr)
    np.testing.assert_array_equal(lab, labr)


@pytest.mark.parametrize("n,d,k", [(40000, 1, 5), (30000, 3, 70), (20000, 20, 9)])
def test_float32_serial_shapes_vs_oracle(ctx, n, d, k):
    """The float32 path's shapes outside the parallel sequential sums (d = 1:
    NumPy's blocked pairwise mean; k > 64: the serial kernel) and d > 16
    (the generic distance kernel), against the oracle on float32 X."""
    import kmeans_plusplus as kp

    X = synth.generate(n, 0, n, d, min(k, 40), 91 + d).astype(np.float32)
    np.random.seed(4)
    C, lab = kp.kmeans(X, k, random_state=8, max_iter=4, context=ctx)
    np.random.seed(4)
    Cr, labr = ko.kmeans(X, k, random_state=8, max_iter=4)
    np.testing.assert_array_equal(lab, labr)
    np.testing.assert_array_equal(C, Cr)


def _config_common(ctx, n, d, k, steps, sample, seed=0x5EED):
    """k-means++ seeds, then `steps` steps of ONE device loop (so the last
    steps are DELTA steps on the default screen, the bench's timed kernel);
    returns the centroids the last assignment used, the loop's final
    centroids, status, labels and the last screen kernel's name."""
    from cdr_dist import Comm, DeviceLloyd, seed_sharded

    ctx.generate_points(n, 0, n, d, k, seed)
    C0 = seed_sharded(ctx, Comm(), 0, n, k, random_state=42)
    np.random.seed(0)
    run = DeviceLloyd(ctx, np.array(C0, dtype=np.float64), -1.0,
                      lambda g: ctx.get_rows([g])[0], n)
    try:
        assert run.advance(steps - 1) == steps - 1
        C_prev = ctx.lloyd_read()[0]
        assert run.advance(1) == 1
        kernel = ctx.profile_kernel()
        C, st = run.finish()
    except BaseException:
        ctx.lloyd_end()
        raise
    lab = ctx.labels()
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(n, sample, replace=False))
    np.testing.assert_array_equal(lab[idx], ko.assign(ctx.get_rows(idx), C_prev))
    return C_prev, C, st, lab, kernel


def test_config3_full_size(ctx):
    """BASELINE config 3: 100M x 16, k = 64 (device generator, k-means++
    seeding, device loop).  Labels of a 50k sample = the oracle; the int64
    sums of two sampled clusters = a NumPy recompute; counts sum to n; the
    means the loop moved to = the host's division of those sums; one shard =
    two shards."""
    import _cdr
    from cdr_dist import shard_rows

    n, d, k = 100_000_000, 16, 64
    C_prev, C, st, lab, _ = _config_common(ctx, n, d, k, 3, 50_000)
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


def _every_label_exact(ctx, monkeypatch, n, d, k, steps):
    monkeypatch.setenv("CDR_BOUNDS", "1")
    C_prev, C, st, lab, kernel = _config_common(ctx, n, d, k, steps, 2_000)
    assert kernel.startswith("screen32b"), kernel
    monkeypatch.setenv("CDR_EXACT_ASSIGN", "1")
    acc_x = ctx.lloyd_step(C_prev)
    monkeypatch.delenv("CDR_EXACT_ASSIGN")
    lab_x = ctx.labels()
    assert (lab_x != lab).sum() == 0
    # the loop moved its centroids to the means of its int64 sums: those of
    # the exact labels
    S = ctx.info()["scale_bits"]
    assert acc_x[:, d].sum() == n
    np.testing.assert_array_equal(C, np.ldexp(acc_x[:, :d].astype(np.float64), -S) /
                                  acc_x[:, d:].astype(np.float64))
    return C_prev, lab


def test_config3_every_label_exact(ctx, monkeypatch):
    """all 100M labels of the last of 25 device-loop steps
    (the bounded DELTA screen, the bench's timed kernel, after a full step,
    the bound rebuild and 22 more bounded steps: the driver's last timed step
    at --warmup 5 --steps 20, where the drift bounds have accumulated longest)
    equal the exact fp64 NumPy-order assignment of the same centroids
    (assign_exact_all on every point, CDR_EXACT_ASSIGN), and so do the int64
    sums; a host-plan DELTA step (pruned screen32p + queued k-way MFMA screen
    + fixup32) on the same centroids agrees."""
    n, d, k = 100_000_000, 16, 64
    C_prev, lab = _every_label_exact(ctx, monkeypatch, n, d, k, 25)
    ctx.lloyd_step(C_prev)
    np.testing.assert_array_equal(ctx.labels(), lab)


def test_config3_every_label_exact_split_kernels(ctx, monkeypatch):
    """The same at 12 steps with the split bounded screen (screen32bz streams
    the bound words and lists the failed points, screen32bs decides the
    lists and resolves near ties at once, CDR_S32BS_SPLIT=1)."""
    monkeypatch.setenv("CDR_S32BS_SPLIT", "1")
    _every_label_exact(ctx, monkeypatch, 100_000_000, 16, 64, 12)


def test_config2_every_label_exact(ctx, monkeypatch):
    """BASELINE config 2 (10M x 8, k = 16) at full
    size, 20 device-loop steps (full screen, bound rebuild, 18 bounded DELTA
    steps: the bench's timed kernel, d <= 8 form): every label and the int64
    sums equal the exact fp64 NumPy-order assignment."""
    _every_label_exact(ctx, monkeypatch, 10_000_000, 8, 16, 20)


def test_config5_full_size_and_scoring(ctx):
    """BASELINE config 5: 50M x 64, k = 1024 (screen_big MFMA path) + replica
    scoring per cluster: labels of a 10k sample = the oracle, sums of two
    sampled clusters = a NumPy recompute, medians of two sampled clusters =
    np.median, and classify_labels = classify on the same medians."""
    import warnings

    from scoring import ClusterClassifier

    n, d, k = 50_000_000, 64, 1024
    C_prev, C, st, lab, _ = _config_common(ctx, n, d, k, 2, 10_000)
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


def _grid_uniform(n, d, seed):
    rng = np.random.default_rng(seed)
    return np.floor(rng.random((n, d)) * 2.0 ** 24) * 2.0 ** -24


def _mirrored(n, d, k, seed):
    """Blobs and their reflections x -> 1 - x (exact on the 2^-24 grid), plus
    points at and a few grid steps around the centre 1/2, which is equidistant
    from every mirrored centroid pair: exact and near ties every step."""
    h = synth.generate(n // 2, 0, n // 2, d, k // 2, seed)
    X = np.concatenate([h, 1.0 - h])
    m = n // 50
    rng = np.random.default_rng(seed)
    X[:m] = 0.5 + np.ldexp(rng.integers(-3, 4, (m, d)).astype(np.float64), -24)
    return X


@pytest.mark.parametrize("n,d,k,kind", [(200_000, 16, 64, "blobs"), (150_000, 16, 64, "uniform"),
                                        (150_000, 8, 16, "uniform"), (100_000, 5, 40, "uniform"),
                                        (120_000, 13, 50, "blobs"), (90_000, 3, 7, "uniform"),
                                        (160_000, 16, 64, "mirror"), (100_000, 8, 32, "mirror"),
                                        (160_000, 16, 64, "mirror-queue"),
                                        (150_000, 8, 16, "uniform-queue"),
                                        (160_000, 16, 64, "mirror-split"),
                                        (150_000, 8, 16, "uniform-split")])
def test_bounded_screen_many_steps_vs_oracle(ctx, n, d, k, kind, monkeypatch):
    """screen32b: after the bound rebuild a point keeps its
    label without its coordinates being read when its stored drift bound
    still separates it; 14 device-loop steps on separated blobs, on uniform
    data (every step moves points across slowly moving boundaries) and on
    mirrored data with exact and near ties: labels and centroids equal the
    oracle's every time, and the bounded steps re-read fewer points than
    they kept.  The default kernel decides in registers (screen32bs); the
    "-split" cases run it as two launches (screen32bz lists the failed
    points, screen32bs decides the lists, CDR_S32BS_SPLIT=1), the "-queue"
    cases screen32b (LDS queue + fused fixup, CDR_S32B_SPLIT=0)."""
    monkeypatch.setenv("CDR_BOUNDS", "1")
    queue = kind.endswith("-queue")
    split = kind.endswith("-split")
    monkeypatch.setenv("CDR_S32BS_SPLIT", "1" if split else "0")
    kind = kind.replace("-queue", "").replace("-split", "")
    monkeypatch.setenv("CDR_S32B_SPLIT", "0" if queue else "1")
    if kind == "blobs":
        X = synth.generate(n, 0, n, d, k, 17 * n + d)
    elif kind == "uniform":
        X = _grid_uniform(n, d, n + d)
    else:
        X = _mirrored(n, d, k, n + d)
    ctx.load_points(X)
    rng = np.random.default_rng(k + d)
    if kind == "mirror":
        half = X[n // 50 + rng.choice(n // 2 - n // 50, k // 2, replace=False)]
        C0 = np.concatenate([half, 1.0 - half])
    else:
        C0 = X[np.sort(rng.choice(n, k, replace=False))]
    steps = 14
    ctx.profile_reset(True)
    np.random.seed(3)
    C, st = _loop(ctx, C0, steps, -1.0, X)
    prof = ctx.profile_read()
    ctx.profile_reset(False)
    # (the fused default keeps 2-byte words)
    want = "screen32b<" if queue else ("screen32bs<" if split else "screen32bs16<")
    assert ctx.profile_kernel().startswith(want), ctx.profile_kernel()
    np.random.seed(3)
    C_ref, lab_ref, _, _ = ko.lloyd(X, C0, steps, -1.0)
    np.testing.assert_array_equal(ctx.labels(), lab_ref)
    np.testing.assert_array_equal(C, C_ref)
    # steps 3 .. 14 are bounded: (the rebuild, step 2, re-reads every point)
    bounded = (steps - 1) * n
    assert n <= prof["tight_points"] < (0.5 if kind == "blobs" else 0.9) * bounded, prof


def test_bounded_screen_off_switch_and_resume(ctx, monkeypatch):
    """CDR_BOUNDS=0 (the pruned screen every step) and the default give the
    same run; a loop stopped for the host (empty cluster) resumes with a
    bound rebuild (the host moved the centroids: no drift bound)."""
    n, d, k = 120_000, 16, 24
    monkeypatch.setenv("CDR_BOUNDS", "1")
    X = synth.generate(n, 0, n, d, k, 4243)
    ctx.load_points(X)
    C0 = X[:k].copy()
    C0[5] = 5.0  # far away: empties at once, the host reseeds (:43)
    np.random.seed(12)
    C_a, st_a = _loop(ctx, C0, 12, -1.0, X)
    lab_a = ctx.labels()
    monkeypatch.setenv("CDR_BOUNDS", "0")
    import _cdr

    b = _cdr.Context(ctx.device)
    try:
        b.load_points(X)
        np.random.seed(12)
        C_b, st_b = _loop(b, C0, 12, -1.0, X)
        assert not b.profile_kernel().startswith("screen32b")
        np.testing.assert_array_equal(b.labels(), lab_a)
    finally:
        b.close()
    np.testing.assert_array_equal(C_b, C_a)
    np.random.seed(12)
    C_ref, lab_ref, _, _ = ko.lloyd(X, C0, 12, -1.0)
    np.testing.assert_array_equal(C_a, C_ref)
    np.testing.assert_array_equal(lab_a, lab_ref)
