"""GPU parity of the access-log ingest (csrc/ingest.hip, cdr_ingest_*).

Checker: oracle.features_oracle.encode_log (python csv + the ISO grammar),
itself pinned against the reference simulator's golden log in
tests/test_oracle_ingest.py.  Events must match field for field; the features
computed through the device ingest must match the golden table bit for bit.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import features_oracle as fo

pytestmark = pytest.mark.gpu
PDIR = os.path.join(GOLDEN, "pipeline")


def _manifest():
    import compute_features as cf

    return cf.load_manifest(os.path.join(PDIR, "metadata.csv"))


def _ingest_and_check(ctx, data: bytes, paths, primary):
    import compute_features as cf

    prim, nodes = cf.encode_primary(primary)
    ctx.ingest_manifest(paths, prim, nodes)
    st = ctx.ingest_log(data)
    f, o, c, t = fo.encode_log(data, paths, primary)
    assert st[0] == f.size
    assert st[2] == -1
    gf, go, gc, gt, gp = ctx.features_events_read()
    np.testing.assert_array_equal(gf, f)
    np.testing.assert_array_equal(go, o)
    np.testing.assert_array_equal(gc, c)
    np.testing.assert_array_equal(gt, t)
    np.testing.assert_array_equal(gp, prim)
    bad = np.flatnonzero(t == fo.TS_NULL)
    assert st[3] == bad.size
    assert st[1] == (bad[0] if bad.size else -1)
    return st


def test_golden_log_events(ctx):
    paths, _, primary = _manifest()
    with open(os.path.join(PDIR, "access.log"), "rb") as fh:
        data = fh.read()
    st = _ingest_and_check(ctx, data, paths, primary)
    assert st[0] == 6995 and st[1] == -1


def test_golden_features_through_device_ingest(ctx):
    import compute_features as cf

    paths, table = cf.compute_features(os.path.join(PDIR, "metadata.csv"),
                                       os.path.join(PDIR, "access.log"), ctx=ctx)
    z = np.load(os.path.join(PDIR, "features_oracle.npz"))
    np.testing.assert_array_equal(table, z["table"])
    counts, _ = ctx.features_aggregate_resident()
    _, _, exp_counts, _ = fo.compute(os.path.join(PDIR, "metadata.csv"),
                                     os.path.join(PDIR, "access.log"))
    np.testing.assert_array_equal(counts[:, [0, 1, 3, 4, 5]], exp_counts[:, [0, 1, 3, 4, 5]])


EDGE_LINES = [
    "2025-11-01T12:00:00.165Z,/user/root/synth/synth_1.bin,READ,dn1,1",
    "",
    "2025-11-01T12:00:01Z,/user/root/synth/synth_2.bin,WRITE,dn9,2\r",
    "\r",
    "2025-11-01 12:00:02,/not/in/manifest,READ,dn2",
    "2025-11-01T12:00:03+05:30,/user/root/synth/synth_3.bin",
    "2025-11-01T12:00:04.123456789-0800,/user/root/synth/synth_3.bin,read,,x,extra,fields",
    " 2025-1-2T3:4 ,/user/root/synth/synth_4.bin,WRITE,dn3,",
    "2025-11-01T12:00:05Z,,READ,dn1,5",
    "2024-02-29T23:59:59.5+01,/user/root/synth/synth_5.bin,WRITE,dn2,6",
    "2023-02-29T00:00:00Z,/user/root/synth/synth_6.bin,READ,dn2,7",
    "2025-11-01T24:00:00Z,/user/root/synth/synth_6.bin,READ,dn2,7",
    "2025-11-01T12:00:06Z,/user/root/synth/synth_7.bin,WRITE,DN1,8",
    ",/user/root/synth/synth_8.bin,READ,dn1,9",
    "2025-11-01T12:00:07Z,/user/root/synth/synth_9.bin, READ,dn1,10",
    "2025-11-01T12:00:08Z,/user/root/synth/synth_9.bin,WRITE ,dn1 ,11",
    "0000-02-29,/user/root/synth/synth_10.bin,READ,dn3,12",
    "9999-12-31T23:59:59.999999-23:59,/user/root/synth/synth_10.bin,READ,dn3,13",
    "2025-11-01T12:00:09Z",
    "x",
    "2025-11-01T12:00:10Z,/user/root/synth/synth_11.bin,WRITE,dn1,14",
]


@pytest.mark.parametrize("trailing", ["", "\n", "\r\n", "\n\n"])
def test_edge_log_records_fields_and_timestamps(ctx, trailing):
    paths, _, primary = _manifest()
    data = ("\n".join(EDGE_LINES) + trailing).encode()
    st = _ingest_and_check(ctx, data, paths, primary)
    assert st[3] == 4  # 2023-02-29, hour 24, the empty ts, "x"


def _fuzz_ts(rng, n):
    def digits(k):
        return "".join(str(int(v)) for v in rng.integers(0, 10, k))

    out = []
    for _ in range(n):
        s = " " * int(rng.integers(0, 2)) + digits(int(rng.choice([4, 4, 4, 3, 5])))
        s += "-" + digits(int(rng.choice([1, 2, 2, 3])))
        s += rng.choice(["-", "-", "-", "/"]) + digits(int(rng.choice([1, 2, 2, 3])))
        r = rng.random()
        if r < 0.8:
            s += rng.choice(["T", " ", "T", "t"]) + digits(int(rng.choice([1, 2, 2, 3])))
            if rng.random() < 0.95:
                s += ":" + digits(int(rng.choice([1, 2, 2, 3, 0])))
            if rng.random() < 0.8:
                s += ":" + digits(int(rng.choice([1, 2, 2, 3, 0])))
                if rng.random() < 0.6:
                    s += "." + digits(int(rng.choice([0, 1, 3, 6, 7, 9, 10])))
        s += rng.choice(["", "", "Z", " Z", "+05:30", "-0800", "+01", "+1", "-05:3", "\t", "z"])
        s += " " * int(rng.integers(0, 2))
        out.append(s)
    return out


def test_timestamp_grammar_fuzz(ctx):
    rng = np.random.default_rng(11)
    paths, _, primary = _manifest()
    ts = _fuzz_ts(rng, 40000)
    # plausible values so that a good share of them parse
    for i in range(0, len(ts), 3):
        y, mo, d = 1970 + int(rng.integers(0, 100)), int(rng.integers(1, 13)), int(rng.integers(1, 32))
        ts[i] = f"{y:04d}-{mo:02d}-{d:02d}T{int(rng.integers(0, 25)):02d}:" \
                f"{int(rng.integers(0, 61)):02d}:{int(rng.integers(0, 61)):02d}" \
                + rng.choice(["", ".5", ".123456", ".1234567", "Z", "+02:00"])
    # the kernel's fixed-layout fast path: 24-byte "YYYY-MM-DDTHH:MM:SS.fffZ"
    # strings with random digits (invalid dates and times included) and a
    # mutated separator or digit now and then
    for i in range(1, len(ts), 3):
        s = list(f"{int(rng.integers(0, 10000)):04d}-{int(rng.integers(0, 14)):02d}-"
                 f"{int(rng.integers(0, 33)):02d}T{int(rng.integers(0, 26)):02d}:"
                 f"{int(rng.integers(0, 62)):02d}:{int(rng.integers(0, 62)):02d}."
                 f"{int(rng.integers(0, 1000)):03d}Z")
        if rng.random() < 0.2:
            s[int(rng.integers(0, 24))] = str(rng.choice(list("0-T:.Z zx/+")))
        ts[i] = "".join(s)
    lines = [f"{t},{paths[i % len(paths)]},READ,dn1,{i}" for i, t in enumerate(ts)]
    data = "\n".join(lines).encode()
    st = _ingest_and_check(ctx, data, paths, primary)
    assert 0 < st[3] < st[0]


def test_bad_timestamp_is_null_like_host_path(ctx, tmp_path):
    """An unparseable timestamp is a null event (Spark's non-ANSI
    to_timestamp): device ingest, host tokeniser and the oracle agree."""
    import compute_features as cf

    log = tmp_path / "bad.log"
    lines = list(EDGE_LINES[:1]) + ["", "2025-13-01T00:00:00Z,/user/root/synth/synth_1.bin,READ,dn1,1",
                                    "x,/user/root/synth/synth_1.bin,WRITE,dn2,1"]
    log.write_bytes(("\n".join(lines) + "\n").encode())
    man = os.path.join(PDIR, "metadata.csv")
    paths, _, primary = cf.load_manifest(man)
    st = _ingest_and_check(ctx, log.read_bytes(), paths, primary)
    assert st[0] == 3 and st[3] == 2
    _, table = cf.compute_features(man, str(log), ctx=ctx)
    lt, lp, lo, lc = cf.load_access_log(str(log))
    fidx, opc, client, ts, prim = cf.encode(paths, primary, lt, lp, lo, lc)
    counts, mx = ctx.features_aggregate(fidx, opc, client, ts, prim)
    _, exp_table, exp_counts, obs = fo.compute(man, str(log))
    np.testing.assert_array_equal(counts, exp_counts)
    assert mx / 1e6 == obs
    np.testing.assert_array_equal(table, exp_table)
    assert exp_counts[1, 5] == 2  # synth_1: the two null events are one second group


def test_quoted_log_goes_to_host_tokeniser(ctx, tmp_path):
    import compute_features as cf

    man = os.path.join(PDIR, "metadata.csv")
    with open(os.path.join(PDIR, "access.log"), "rb") as fh:
        data = fh.read().splitlines()
    data[5] = b'2025-11-01T12:00:02.000Z,"/user/root/synth/synth_3.bin",READ,dn1,1'
    log = tmp_path / "quoted.log"
    log.write_bytes(b"\n".join(data) + b"\n")
    paths, _, primary = cf.load_manifest(man)
    prim, nodes = cf.encode_primary(primary)
    ctx.ingest_manifest(paths, prim, nodes)
    st = ctx.ingest_log(log.read_bytes())
    assert st[2] == 5
    _, table = cf.compute_features(man, str(log), ctx=ctx)
    _, exp_table, _, _ = fo.compute(man, str(log))
    np.testing.assert_array_equal(table, exp_table)


def test_large_random_log_long_paths(ctx):
    """Many tiles, staged and unstaged workgroups (paths up to 600 bytes make
    some 256-record spans exceed the 32 KiB LDS stage), blank lines, CRLF."""
    rng = np.random.default_rng(3)
    nf = 3000
    paths = [f"/data/{'d' * int(rng.integers(0, 600 if i % 50 == 0 else 40))}/f{i}.bin"
             for i in range(nf)]
    paths[7] = paths[3]  # duplicate manifest path: the first row wins
    nodes = [f"dn{j}" for j in range(12)]
    primary = [None if rng.random() < 0.05 else nodes[int(rng.integers(0, 12))] for _ in range(nf)]
    ne = 300000
    fi = rng.integers(-1, nf, ne)
    sec = 1_761_998_400 + np.sort(rng.integers(0, 600, ne))
    ms = rng.integers(0, 1000, ne)
    ops = np.array(["READ", "WRITE", "OPEN"])[rng.choice(3, ne, p=[0.6, 0.35, 0.05])]
    cl = rng.integers(0, 14, ne)
    out = []
    for e in range(ne):
        t = np.datetime64(int(sec[e]), "s").astype(str)
        p = paths[fi[e]] if fi[e] >= 0 else "/elsewhere/x"
        c = f"dn{cl[e]}" if cl[e] < 13 else ""
        out.append(f"{t}.{ms[e]:03d}Z,{p},{ops[e]},{c},{e}")
        if rng.random() < 0.01:
            out.append("")
    data = "\n".join(out).replace("\n", "\r\n", 1000).encode()
    st = _ingest_and_check(ctx, data, paths, primary)
    assert st[0] == ne and st[1] == -1
    again = ctx.ingest_reparse()
    np.testing.assert_array_equal(again, st)
    counts, mx = ctx.features_aggregate_resident()
    f, o, c, t = fo.encode_log(data, paths, primary)
    import compute_features as cf

    prim, _ = cf.encode_primary(primary)  # the ids encode_log's clients use
    exp, emx = fo.counts_from_arrays(f, o, c, t, prim, nf)
    np.testing.assert_array_equal(counts, exp)
    assert mx == emx


@pytest.mark.parametrize("data", [b"", b"\n", b"\n\r\n\n", b"\r"])
def test_empty_logs(ctx, data):
    paths, _, primary = _manifest()
    st = _ingest_and_check(ctx, data, paths, primary)
    assert st[0] == 0
    counts, mx = ctx.features_aggregate_resident()
    assert not counts.any() and mx == -(2 ** 63)


def test_bench_log_generator_events(ctx):
    """The config-4 ingest leg's fixed-width log (bench.make_log): every event
    as the checker reads it, then the group-by counts."""
    import bench
    import compute_features as cf

    data, paths, primary = bench.make_log(200000, 20000, 7)
    st = _ingest_and_check(ctx, data, paths, primary)
    assert st[0] == 200000 and st[1] == -1
    counts, mx = ctx.features_aggregate_resident()
    f, o, c, t = fo.encode_log(data, paths, primary)
    prim, _ = cf.encode_primary(primary)
    exp, emx = fo.counts_from_arrays(f, o, c, t, prim, len(paths))
    np.testing.assert_array_equal(counts, exp)
    assert mx == emx
