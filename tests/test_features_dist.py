"""Sharded compute_features (features_dist.py) on CPU:
gloo, world sizes 1-3.  Each rank's device context is replaced by a test
double built on the oracle (the device ingest's restatement encode_log, the
NumPy group-by counts_from_arrays, the finalisation formulas), so this checks
the distributed protocol itself — newline-aligned log slices, the all-to-all
of 16-byte records to the owners of their rows, the MAX of the last
timestamp, the repeated-path records and the SUM / MIN / MAX statistics —
against the single-process oracle (oracle/features_oracle.compute), bit for
bit.  The GPU version of the same run is tests/test_gpu_features_dist.py."""
import os
import socket

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import features_oracle as fo

PDIR = os.path.join(GOLDEN, "pipeline")
REC = np.dtype([("ts", "<i8"), ("file", "<i4"), ("cop", "<i4")])


class OracleFeatures:
    """Test double with the _cdr.Context surface features_dist uses."""

    def __init__(self):
        self._ev = (0, 0)

    def ingest_manifest(self, paths, prim, nodes):
        self.paths = list(paths)
        self.prim_all = np.asarray(prim, dtype=np.int32)
        self.names = [nodes[i] if i >= 0 else None for i in self.prim_all]

    def ingest_log(self, data):
        self.f, self.op, self.cl, self.ts = fo.encode_log(bytes(data), self.paths, self.names)
        self.prim = self.prim_all
        self._ev = (self.f.size, len(self.paths))
        return np.array([self.f.size, -1, -1, 0, 0, 0], dtype=np.int64)

    def features_load_events(self, f, op, cl, ts, prim):
        self.f, self.op, self.cl, self.ts = f, op, cl, ts
        self._ev = (f.size, len(prim))

    def features_exchange_pack(self, bounds, send):
        b = np.asarray(bounds)
        ok = (self.f >= b[0]) & (self.f < b[-1])
        owner = np.searchsorted(b, self.f, side="right") - 1
        real = self.ts[self.ts != fo.TS_NULL]
        mx = int(real.max()) if real.size else fo.TS_NULL
        counts = np.zeros(b.size - 1, dtype=np.int64)
        recs = []
        for r in range(b.size - 1):
            sel = ok & (owner == r)
            counts[r] = sel.sum()
            x = np.zeros(int(counts[r]), dtype=REC)
            x["ts"], x["file"] = self.ts[sel], self.f[sel]
            x["cop"] = (self.cl[sel].astype(np.int64) << 8 | self.op[sel]).astype(np.int32)
            recs.append(x)
        flat = np.concatenate(recs).view(np.uint8) if recs else np.zeros(0, np.uint8)
        send[: flat.size] = flat
        return send, counts, mx

    def features_exchange_unpack(self, recv, n, lo, hi):
        x = np.frombuffer(np.asarray(recv)[: 16 * n].tobytes(), dtype=REC)
        self.ts = x["ts"].copy()
        self.f = (x["file"] - lo).astype(np.int32)
        self.op = (x["cop"] & 0xFF).astype(np.uint8)
        self.cl = (x["cop"] >> 8).astype(np.int32)
        self.prim = self.prim_all[lo:hi]
        self._ev = (int(n), hi - lo)

    def features_aggregate_resident(self):
        return fo.counts_from_arrays(self.f, self.op, self.cl, self.ts, self.prim, self.prim.size)

    def features_events_read(self):
        return self.f, self.op, self.cl, self.ts, self.prim

    @staticmethod
    def _cols(counts, created, obs_end):
        age = np.where(np.isnan(created), 0.0, obs_end - created)
        tot = counts[:, 4]
        loc = np.where(tot > 0, counts[:, 3] / np.maximum(tot, 1), 1.0)
        return age, loc

    def features_finalize_stats(self, counts, created, obs_end):
        if counts.shape[0] == 0:
            big, small = np.iinfo(np.int64).max, np.iinfo(np.int64).min
            return (np.array([0, big, small, big, small, big, small], dtype=np.int64),
                    np.array([np.inf, -np.inf, np.inf, -np.inf]))
        age, loc = self._cols(counts, created, obs_end)
        af, w, co = counts[:, 0], counts[:, 1], counts[:, 5]
        return (np.array([w.sum(), af.min(), af.max(), w.min(), w.max(), co.min(), co.max()],
                         dtype=np.int64),
                np.array([age.min(), age.max(), loc.min(), loc.max()]))

    def features_finalize_apply(self, counts, created, obs_end, ist, dst, n_rows):
        age, loc = self._cols(counts, created, obs_end)
        mean = float(ist[0]) / n_rows or 1.0
        af, co = counts[:, 0], counts[:, 5]
        wr = counts[:, 1] / mean
        wmin, wmax = ist[3] / mean, ist[4] / mean

        def nl(v, a, b):
            return np.zeros(v.size) if a == b else (v - a).astype(np.float64) / float(b - a)

        def nd(v, a, b):
            return np.zeros(v.size) if a == b else (v - a) / (b - a)
        return np.column_stack([af.astype(np.float64), age, wr, loc, co.astype(np.float64),
                                nl(af, ist[1], ist[2]), nd(age, dst[0], dst[1]),
                                nd(wr, wmin, wmax), nd(loc, dst[2], dst[3]),
                                nl(co, ist[5], ist[6])])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, man, log, out_dir):
    import torch.distributed as dist

    from cdr_dist import Comm
    from features_dist import sharded_compute_features

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    paths, table = sharded_compute_features(man, log, OracleFeatures(), Comm(dist, None))
    if rank == 0:
        np.save(os.path.join(out_dir, "table.npy"), table)
        with open(os.path.join(out_dir, "paths.txt"), "w") as fh:
            fh.write("\n".join(paths))
    dist.barrier()
    dist.destroy_process_group()


def _case(tmp_path):
    """The golden pipeline manifest with a repeated path, an empty path and a
    null creation time appended; its log plus events of those rows, a
    null-path event, an unparseable timestamp and a path outside the
    manifest."""
    with open(os.path.join(PDIR, "metadata.csv")) as fh:
        man = fh.read().rstrip("\n").split("\n")
    man += ["/user/root/synth/synth_3.bin,2025-10-06T00:00:00Z,dn2,5,moderate",
            ",2025-10-06T00:00:00Z,dn1,5,moderate",
            "/extra/x.bin,,dn3,5,hot"]
    with open(os.path.join(PDIR, "access.log")) as fh:
        log = fh.read().rstrip("\n").split("\n")
    log += ["2025-11-01T12:09:59.999Z,/user/root/synth/synth_3.bin,READ,dn2,1",
            "2025-11-01T12:10:00.500Z,/extra/x.bin,WRITE,dn3,1",
            "garbage,/extra/x.bin,READ,dn1,1",
            "2025-11-01T12:10:01.000Z,,READ,dn1,1",
            "2025-11-01T12:10:02.000Z,/not/in/manifest,READ,dn1,1"]
    mp_, lp = tmp_path / "manifest.csv", tmp_path / "access.log"
    mp_.write_text("\n".join(man) + "\n")
    lp.write_text("\n".join(log) + "\n")
    return str(mp_), str(lp)


def test_file_bounds_and_log_slices(tmp_path):
    from features_dist import file_bounds, log_slice

    for n in (0, 1, 5, 50, 1001):
        for w in (1, 2, 3, 8):
            b = file_bounds(n, w)
            assert b[0] == 0 and b[-1] == n and np.all(np.diff(b) >= 0)
            assert np.diff(b).max() - np.diff(b).min() <= 1
    data = b"a,1\n\nbb,2\r\nccc,3\nd,4"
    p = tmp_path / "l.log"
    p.write_bytes(data)
    for w in (1, 2, 3, 5, 30):
        parts = [log_slice(str(p), r, w) for r in range(w)]
        assert b"".join(parts) == data
        end = 0
        for x in parts:  # every slice but the log's tail ends at a line end
            end += len(x)
            assert x == b"" or x[-1:] == b"\n" or end == len(data)


def test_quoted_log_slices_keep_records(tmp_path):
    """A quoted field with newlines (and doubled quotes) never straddles two
    ranks' slices: the slices' records are csv.reader's records of the whole
    log, for every world size and wherever the byte cut lands."""
    import csv
    import io

    from features_dist import log_slice

    lines = ["2025-11-01T12:00:00.000Z,/a.bin,READ,dn1,1"]
    lines += ['2025-11-01T12:00:01.000Z,"/b\n\n""q""\n.bin",WRITE,dn2,2'] * 3
    lines += ['2025-11-01T12:00:02.000Z,/c"d.bin,READ,dn3,3', "", "x,\"y\nz\",READ,dn1,4\r"]
    data = ("\n".join(lines) + "\n").encode()
    p = tmp_path / "q.log"
    p.write_bytes(data)
    want = list(csv.reader(io.StringIO(data.decode(), newline="")))
    for w in range(1, 12):
        parts = [log_slice(str(p), r, w, quoted=True) for r in range(w)]
        assert b"".join(parts) == data
        got = [rec for x in parts for rec in csv.reader(io.StringIO(x.decode(), newline=""))]
        assert got == want, w


def _quoted_case(tmp_path):
    """_case with records whose quoted path holds newlines, placed across
    the byte cuts of 2 and 3 ranks."""
    man, log = _case(tmp_path)
    with open(log) as fh:
        lines = fh.read().rstrip("\n").split("\n")
    q = ('2025-11-01T12:05:00.000Z,"/user/root/synth/' + "\n" * 300 + 'synth_7.bin",READ,dn1,9')
    lines = [x for i, line in enumerate(lines) for x in ([line, q] if i % 3 == 2 else [line])]
    with open(log, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    return man, log


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("quoted", [False, True], ids=["plain", "quoted-newlines"])
def test_sharded_features_equal_single_process(tmp_path, world, quoted):
    man, log = (_quoted_case if quoted else _case)(tmp_path)
    if world == 1:
        from cdr_dist import Comm
        from features_dist import sharded_compute_features

        paths, table = sharded_compute_features(man, log, OracleFeatures(), Comm(None))
    else:
        mp = pytest.importorskip("torch.multiprocessing")
        mp.spawn(_worker, args=(world, _free_port(), man, log, str(tmp_path)), nprocs=world,
                 join=True)
        table = np.load(tmp_path / "table.npy")
        paths = (tmp_path / "paths.txt").read_text().split("\n")
    exp_paths, exp_table, _, _ = fo.compute(man, log)
    assert [p or "" for p in exp_paths] == [p or "" for p in paths]
    np.testing.assert_array_equal(table, exp_table)


def _record_start_bytewise(data: bytes, x: int) -> int:
    """The csv.reader record-start scan byte by byte (the form features_dist
    used before its quote-free fast path): the checker of test below."""
    if x <= 0:
        return 0
    if x >= len(data):
        return len(data)
    inq = qpend = False
    fstart = True
    for i, c in enumerate(data):
        if inq:
            if qpend:
                qpend = False
                if c == 34:
                    continue
                inq = False
            elif c == 34:
                qpend = True
                continue
            else:
                continue
        if c == 34 and fstart:
            inq, fstart = True, False
        elif c == 44:
            fstart = True
        elif c == 10:
            fstart = True
            if i + 1 >= x:
                return i + 1
        else:
            fstart = c == 13
    return len(data)


def test_record_start_fast_path_matches_bytewise(tmp_path):
    """quote-free 64 KiB chunks skip the per-byte loop; the
    cut points equal the byte-by-byte scan on logs with sparse and dense
    quoting, quoted newlines, doubled quotes and CRs."""
    import random

    from features_dist import _record_start

    rng = random.Random(5)
    alphabet = [b"a", b"b", b"1", b",", b"\n", b"\r", b'"', b" "]
    for trial in range(6):
        weights = [30, 30, 20, 10, 6, 1, 1 if trial % 2 else 8, 4]
        n = 200_000 if trial < 3 else 3000
        data = b"".join(rng.choices(alphabet, weights=weights, k=n))
        p = tmp_path / f"log{trial}.csv"
        p.write_bytes(data)
        with open(p, "rb") as fh:
            for x in [0, 1, 2, 65535, 65536, 65537, n // 3, n // 2, n - 2, n - 1, n] + \
                     [rng.randrange(n) for _ in range(20)]:
                assert _record_start(fh, x, n) == _record_start_bytewise(data, x), (trial, x)
