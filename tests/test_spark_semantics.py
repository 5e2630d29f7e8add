"""Spark value semantics of compute_features that the reference's own inputs
never exercise (src/compute_features.py): null / unparseable timestamps and
manifests that list a path twice or leave it empty.

No Spark in this image and the reference's generators never write these
cases, so the expected values are derived BY HAND from Spark's documented
rules (parity unpinned against Spark itself):
  * to_timestamp of a bad string is null (non-ANSI, :17, :28); count(lit(1))
    still counts the event (:32, :42); groupBy(path, sec) keeps the null sec as
    a group (:44-46); max(ts_epoch) skips nulls (:48), all null -> time.time();
  * an equi-join never matches a null key; a key present m times on the right
    multiplies rows (:37 for the locality counts, :59 for the output rows).
The CPU tests pin the oracle (oracle/features_oracle.compute) to these hand
values and the host-side join expansion; the GPU tests run the product path
(device ingest + group-by + finalize) against both.
"""
import os
import time

import numpy as np
import pytest

from oracle import features_oracle as fo

T0 = 1735689600  # 2025-01-01T00:00:00Z

MANIFEST = """path,creation_ts,primary_node
/a,2025-01-01T00:00:00Z,dn1
/b,2025-01-01T00:00:10Z,dn2
/a,2025-01-01T00:00:20Z,dn2
,2025-01-01T00:00:30Z,dn1
/c,,dn3
"""

LOG = """2025-01-01T00:01:00.500Z,/a,WRITE,dn1,1
2025-01-01T00:01:00.900Z,/a,READ,dn2,1
garbage,/a,READ,dn2,1
,/a,WRITE,dn3,1
2025-13-01T00:00:00Z,/a,READ,dn1,1
2025-01-01T00:01:05Z,/b,READ,dn2,1
2025-01-01T00:01:07Z,/z,READ,dn2,1
2025-01-01T00:02:00Z,,READ,dn1,1
notatime,/b,WRITE,dn1,1
"""

# Hand derivation.  observation_end = 00:02:00 (the null-path event counts for
# the max; the unparseable ones do not) = T0 + 120.
#  /a: 5 events (2 WRITE, 3 READ).  Each meets both /a manifest rows
#      (primaries dn1, dn2): clients dn1 dn2 dn2 dn3 dn1 -> 2 + 2 = 4 local of
#      10.  Seconds: T0+60 holds 2 events, the null second 3 -> concurrency 3.
#  /b: 2 events (1 WRITE, 1 READ), primary dn2: 1 local of 2; seconds T0+65
#      and null, 1 each -> 1.
#  empty path: joins nothing -> zeros, age 0.  /c: no events, null creation
#      -> age 0, locality 1.0.
#  Output rows: manifest order, and each /a row pairs with both /a age rows
#  (creation T0 -> age 120, T0+20 -> 100): /a /a /b /a /a null /c.
EXP_PATHS = ["/a", "/a", "/b", "/a", "/a", None, "/c"]
EXP_COUNTS = np.array([  # access_freq, writes, reads, local, total, concurrency
    [5, 2, 3, 4, 10, 3], [5, 2, 3, 4, 10, 3], [2, 1, 1, 1, 2, 1],
    [5, 2, 3, 4, 10, 3], [5, 2, 3, 4, 10, 3], [0, 0, 0, 0, 0, 0], [0, 0, 0, 0, 0, 0]],
    dtype=np.int64)
EXP_AGE = np.array([120.0, 100.0, 110.0, 120.0, 100.0, 0.0, 0.0])


def _expected_table():
    af = EXP_COUNTS[:, 0].astype(np.float64)
    mean_w = 9 / 7
    wr = EXP_COUNTS[:, 1] / mean_w
    loc = np.array([0.4, 0.4, 0.5, 0.4, 0.4, 1.0, 1.0])
    co = EXP_COUNTS[:, 5].astype(np.float64)

    def mm(v):
        return (v - v.min()) / (v.max() - v.min())
    return np.column_stack([af, EXP_AGE, wr, loc, co, mm(af), mm(EXP_AGE), mm(wr), mm(loc),
                            mm(co)])


@pytest.fixture
def case(tmp_path):
    man = tmp_path / "manifest.csv"
    log = tmp_path / "access.log"
    man.write_text(MANIFEST)
    log.write_text(LOG)
    return str(man), str(log)


def test_oracle_matches_hand_derivation(case):
    paths, table, counts, obs = fo.compute(*case)
    assert obs == T0 + 120
    assert paths == EXP_PATHS
    np.testing.assert_array_equal(counts, EXP_COUNTS)
    np.testing.assert_allclose(table, _expected_table(), rtol=0, atol=1e-15)
    np.testing.assert_array_equal(table[:, 3], [0.4, 0.4, 0.5, 0.4, 0.4, 1.0, 1.0])


def test_oracle_all_null_timestamps_use_now(tmp_path):
    man = tmp_path / "m.csv"
    man.write_text(MANIFEST)
    log = tmp_path / "l.log"
    log.write_text("bad,/a,READ,dn1,1\n,/b,WRITE,dn2,1\n")
    _, table, counts, obs = fo.compute(str(man), str(log), now=T0 + 1000.5)
    assert obs == T0 + 1000.5
    np.testing.assert_array_equal(counts[:, 5], [1, 1, 1, 1, 1, 0, 0])
    np.testing.assert_array_equal(table[:, 1], [1000.5, 980.5, 990.5, 1000.5, 980.5, 0, 0])


def test_counts_from_arrays_null_seconds():
    f = np.array([0, 0, 0, 1, 1, -1], dtype=np.int32)
    op = np.array([1, 2, 2, 1, 0, 1], dtype=np.uint8)
    cl = np.array([0, -1, 0, 1, 1, 0], dtype=np.int32)
    ts = np.array([fo.TS_NULL, fo.TS_NULL, 5_000_000, 7_000_000, 7_100_000, 9_000_000],
                  dtype=np.int64)
    out, mx = fo.counts_from_arrays(f, op, cl, ts, np.array([0, -2], dtype=np.int32), 2)
    np.testing.assert_array_equal(out, [[3, 1, 2, 2, 3, 2], [2, 1, 0, 0, 2, 2]])
    assert mx == 9_000_000
    out, mx = fo.counts_from_arrays(f[:2], op[:2], cl[:2], ts[:2], np.zeros(2, np.int32), 2)
    assert mx is None and out[0, 5] == 2


def test_expand_joins_host_logic():
    """compute_features.expand_joins on device-shaped counts (every event on
    the first manifest row of its path) gives the hand-derived rows."""
    import compute_features as cf

    paths = ["/a", "/b", "/a", "", "/c"]
    primary = ["dn1", "dn2", "dn2", "dn1", "dn3"]
    created = np.array([T0, T0 + 10, T0 + 20, T0 + 30, np.nan])
    # device counts: /a on row 0, local vs row 0's primary (dn1) = 2
    counts = np.array([[5, 2, 3, 2, 5, 3], [2, 1, 1, 1, 2, 1], [0] * 6, [0] * 6, [0] * 6],
                      dtype=np.int64)
    prim, nodes = cf.encode_primary(primary)
    nid = {n: i for i, n in enumerate(nodes)}
    f_ev = np.array([0, 0, 0, 0, 0, 1, 1], dtype=np.int32)
    c_ev = np.array([nid["dn1"], nid["dn2"], nid["dn2"], -3, nid["dn1"], nid["dn2"], nid["dn1"]],
                    dtype=np.int32)
    out_p, out_c, out_t = cf.expand_joins(paths, created, primary, counts, lambda: (f_ev, c_ev))
    assert out_p == ["/a", "/a", "/b", "/a", "/a", "", "/c"]
    np.testing.assert_array_equal(out_c, EXP_COUNTS)
    np.testing.assert_array_equal(out_t, [T0, T0 + 20, T0 + 10, T0, T0 + 20, np.nan, np.nan])


def test_expand_joins_unique_paths_untouched():
    import compute_features as cf

    counts = np.arange(12, dtype=np.int64).reshape(2, 6)
    created = np.array([1.0, 2.0])
    out_p, out_c, out_t = cf.expand_joins(["/x", "/y"], created, ["dn1", None], counts,
                                          lambda: pytest.fail("events read without repeats"))
    assert out_p == ["/x", "/y"] and out_c is counts
    np.testing.assert_array_equal(out_t, created)


# ---- the product path on the device ---------------------------------------
@pytest.mark.gpu
def test_device_pipeline_hand_case(case):
    import compute_features as cf
    from _cdr import Context

    ctx = Context(0)
    try:
        paths, table = cf.compute_features(*case, ctx=ctx)
        assert paths == ["" if p is None else p for p in EXP_PATHS]
        _, exp_table, _, _ = fo.compute(*case)
        np.testing.assert_array_equal(table, exp_table)
        np.testing.assert_allclose(table, _expected_table(), rtol=0, atol=1e-15)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_device_pipeline_all_null_timestamps(tmp_path):
    import compute_features as cf
    from _cdr import Context

    man = tmp_path / "m.csv"
    man.write_text(MANIFEST)
    log = tmp_path / "l.log"
    log.write_text("bad,/a,READ,dn1,1\n,/b,WRITE,dn2,1\n2025-02-30T00:00:00Z,/a,READ,dn2,1\n")
    ctx = Context(0)
    try:
        t0 = time.time()
        _, table = cf.compute_features(str(man), str(log), ctx=ctx)
        t1 = time.time()
    finally:
        ctx.close()
    age = table[:, 1]
    assert t0 - T0 - 1e-3 <= age[0] <= t1 - T0 + 1e-3  # observation_end = time.time()
    _, exp, _, _ = fo.compute(str(man), str(log), now=age[0] + T0)
    np.testing.assert_array_equal(table[:, [0, 2, 3, 4, 5, 7, 8, 9]], exp[:, [0, 2, 3, 4, 5, 7, 8, 9]])
    np.testing.assert_allclose(table[:, [1, 6]], exp[:, [1, 6]], rtol=0, atol=1e-6)
