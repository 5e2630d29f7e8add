"""compute_features over several ranks: one process per
GPU, the same output as the single-process job (src/compute_features.py).

Partition (DESIGN.md §features sharding):

* rows — rank r owns the contiguous manifest rows [bounds[r], bounds[r+1])
  (``file_bounds``) and every output row that comes from them;
* log — rank r ingests the newline-aligned byte range [r L / W, (r+1) L / W)
  of the access log (``log_slice``; a line belongs to the rank whose range
  holds its first byte), on the device (csrc/ingest.hip) or, for CSV quoting,
  with the host tokeniser; when any slice holds a quote every rank cuts at
  CSV record starts instead, so a quoted newline never splits a record;
* exchange — one all-to-all (RCCL on the GPU path) of 16-byte event records
  sends every event to the owner of its file row (csrc/exchange.hip), so the
  owner's group-by (csrc/groupby.hip) sees all events of its files: the
  integer counters equal the single-process ones;
* collectives — MAX of the last timestamp over all events (:48; events of
  paths outside the manifest included), an all-gather of the repeated-path
  records (a path listed m times is owned by the rank of its first row, whose
  local / total counts every row of it needs, :37-42, :56-59), and SUM / MIN /
  MAX of the finalisation statistics (:62-83) before each rank writes its
  rows' table (``cdr_features_finalize_apply``);
* output — the per-rank tables are gathered to rank 0 in rank order, which
  is manifest order.

Observation end without any parseable timestamp is rank 0's time.time(),
broadcast, so every rank ages its rows from the same instant (:50-51).
"""
from __future__ import annotations

import csv
import io
import os
import time

import numpy as np

import compute_features as cf
from cdr_dist import Comm

TS_NULL = cf.TS_NULL
XREC = 16  # bytes per exchanged event record (csrc/exchange.hip)


def file_bounds(n_files: int, world: int) -> np.ndarray:
    """Contiguous, balanced manifest row ranges: bounds[r] .. bounds[r+1]."""
    return np.array([(n_files * r) // world for r in range(world + 1)], dtype=np.int64)


def _line_start(fh, x: int, size: int) -> int:
    """First line start at or after byte x (x itself when x == 0 or the byte
    before it is a newline)."""
    if x <= 0:
        return 0
    if x >= size:
        return size
    fh.seek(x - 1)
    pos = x - 1
    while True:
        chunk = fh.read(1 << 16)
        if not chunk:
            return size
        i = chunk.find(b"\n")
        if i >= 0:
            return pos + i + 1
        pos += len(chunk)


_Q, _C, _NL = ord('"'), ord(","), ord("\n")


def _record_start(fh, x: int, size: int) -> int:
    """First CSV record start at or after byte x, reading the log from byte 0
    the way csv.reader does (excel dialect, the host path of
    compute_features.load_access_log): a newline inside a quoted field does
    not end the record.  Linear in x; only used for logs that hold quotes."""
    if x <= 0:
        return 0
    if x >= size:
        return size
    fh.seek(0)
    inq = qpend = False  # inside a quoted field / a quote seen inside one
    fstart = True        # at the first byte of a field
    pos = 0
    while True:
        chunk = fh.read(1 << 16)
        if not chunk:
            return size
        if not inq and b'"' not in chunk:
            # no quote: every newline ends a record and only "at a field
            # start" carries over (bytes.find, not a Python loop per byte)
            if pos + len(chunk) >= x:
                i = chunk.find(b"\n", max(0, x - pos - 1))
                if i >= 0:
                    return pos + i + 1
            fstart = chunk[-1] in (_C, _NL, 13)
            pos += len(chunk)
            continue
        for i, c in enumerate(chunk):
            if inq:
                if qpend:
                    qpend = False
                    if c == _Q:  # "" inside quotes: a literal quote
                        continue
                    inq = False  # the quoted part ended; c continues the field
                elif c == _Q:
                    qpend = True
                    continue
                else:
                    continue
            if c == _Q and fstart:
                inq, fstart = True, False
            elif c == _C:
                fstart = True
            elif c == _NL:
                fstart = True
                if pos + i + 1 >= x:
                    return pos + i + 1
            else:
                fstart = c == 13  # after a CR a new record (and field) begins
        pos += len(chunk)


def log_slice(path: str, rank: int, world: int, quoted: bool = False) -> bytes:
    """Rank `rank`'s byte range of the log: cut at newlines, or (quoted: the
    log holds CSV quoting) at record starts, so that a quoted field with a
    newline stays on one rank as csv.reader keeps it in one record."""
    path = cf._strip_scheme(path)
    size = os.path.getsize(path)
    start = _record_start if quoted else _line_start
    with open(path, "rb") as fh:
        a = start(fh, (size * rank) // world, size)
        b = start(fh, (size * (rank + 1)) // world, size)
        fh.seek(a)
        return fh.read(b - a)


def _host_events(data: bytes, paths, primary):
    """The host tokeniser on a slice (CSV quoting): events with global rows."""
    ts, p, op, cl = [], [], [], []
    for rec in csv.reader(io.StringIO(data.decode("utf-8"), newline="")):
        if not rec:
            continue
        rec = rec + [""] * (5 - len(rec))
        ts.append(rec[0] or None)
        p.append(rec[1] or None)
        op.append(rec[2] or None)
        cl.append(rec[3] or None)
    return cf.encode(paths, primary, ts, p, op, cl)


def _dup_rows(paths):
    rows_of = {}
    for i, p in enumerate(paths):
        if p:
            rows_of.setdefault(p, []).append(i)
    return {p: r for p, r in rows_of.items() if len(r) > 1}


def sharded_compute_features(manifest: str, access_log: str, ctx, comm: Comm):
    """Every rank calls this; rank 0 returns (paths, table (rows, 10)) of the
    whole job, the other ranks (None, None)."""
    paths, created, primary = cf.load_manifest(manifest)
    nf, world, rank = len(paths), comm.world, comm.rank
    bounds = file_bounds(nf, world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    prim, nodes = cf.encode_primary(primary)
    # 1) this rank's slice of the log -> resident events (global rows)
    data = log_slice(access_log, rank, world)
    if int(comm.allreduce_i64(np.array([b'"' in data], dtype=np.int64), "max")[0]):
        data = log_slice(access_log, rank, world, quoted=True)
    ctx.ingest_manifest(paths, prim, nodes)
    st = ctx.ingest_log(data)
    if st[2] >= 0:  # CSV syntax the device tokeniser leaves to the host
        f, o, c, t, _ = _host_events(data, paths, primary)
        ctx.features_load_events(f, o, c, t, prim)
    # 2) events to the owners of their rows
    ne_local = int(ctx._ev[0])
    send, handle = comm.exchange_buffer(ne_local * XREC)
    _, counts, mx = ctx.features_exchange_pack(bounds, handle)
    recv, rhandle, recv_bytes = comm.fenced(ctx, comm.all_to_all_bytes, send, counts * XREC)
    n_recv = int(recv_bytes.sum()) // XREC
    ctx.features_exchange_unpack(rhandle, n_recv, lo, hi)
    # 3) the owned rows' counters
    if hi > lo:
        counts_local, _ = ctx.features_aggregate_resident()
    else:
        counts_local = np.zeros((0, 6), dtype=np.int64)
    # 4) observation end over every event of every rank (:48-51)
    gmx = int(comm.allreduce_i64(np.array([mx]), "max")[0])
    if gmx != TS_NULL:
        obs_end = gmx / 1e6
    else:
        obs_end = float(comm.bcast(np.array([time.time()]), 0)[0])
    # 5) repeated paths: the owner of the first row counts local accesses
    #    against every row's primary (:37-42); records all-gathered
    dup = _dup_rows(paths)
    mine = []
    if dup:
        f_ev, _, c_ev, _, _ = ctx.features_events_read() if hi > lo else (np.zeros(0, np.int32),) * 5
        for p, rows in dup.items():
            if lo <= rows[0] < hi:
                cl = c_ev[f_ev == rows[0] - lo]
                local = sum(int(np.count_nonzero((cl >= 0) & (cl == prim[r]))) for r in rows
                            if prim[r] >= 0)
                c = counts_local[rows[0] - lo].copy()
                c[3] = local
                c[4] = c[4] * len(rows)
                mine.append(np.concatenate([[rows[0]], c]))
    recs = {}
    if dup:
        flat = np.concatenate(mine).astype(np.int64) if mine else np.zeros(0, np.int64)
        for part in comm.allgather(flat):
            for rec in part.reshape(-1, 7):
                recs[int(rec[0])] = rec[1:]
    # 6) the output rows of the owned manifest rows (expand_joins, sharded)
    out_c, out_t = [], []
    for i in range(lo, hi):
        p = paths[i]
        if p in dup:
            rows = dup[p]
            for j in rows:
                out_c.append(recs[rows[0]])
                out_t.append(created[j])
        else:
            out_c.append(counts_local[i - lo])
            out_t.append(created[i] if p else np.nan)
    rc = np.array(out_c, dtype=np.int64).reshape(-1, 6)
    rt = np.array(out_t, dtype=np.float64)
    # 7) statistics over all rows, then this rank's table
    ist, dst = ctx.features_finalize_stats(rc, rt, obs_end)
    n_rows = int(comm.allreduce_i64(np.array([rc.shape[0]]), "sum")[0])
    g_sum = comm.allreduce_i64(ist[[0]], "sum")
    g_min = comm.allreduce_i64(ist[[1, 3, 5]], "min")
    g_max = comm.allreduce_i64(ist[[2, 4, 6]], "max")
    gi = np.array([g_sum[0], g_min[0], g_max[0], g_min[1], g_max[1], g_min[2], g_max[2]],
                  dtype=np.int64)
    d_min = comm.allreduce_f64(dst[[0, 2]], "min")
    d_max = comm.allreduce_f64(dst[[1, 3]], "max")
    gd = np.array([d_min[0], d_max[0], d_min[1], d_max[1]], dtype=np.float64)
    table = (ctx.features_finalize_apply(rc, rt, obs_end, gi, gd, n_rows) if rc.shape[0]
             else np.zeros((0, 10)))
    # 8) rank 0 assembles the job's output in manifest order
    parts = comm.allgather(table.reshape(-1))
    if rank != 0:
        return None, None
    full = np.concatenate(parts).reshape(-1, 10)
    out_p = []
    for p in paths:
        out_p.extend([p] * (len(dup[p]) if p in dup else 1))
    return out_p, full
