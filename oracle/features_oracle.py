"""pandas restatement of the reference PySpark job (TEST INFRASTRUCTURE ONLY).

Follows /root/reference/src/compute_features.py:14-94 with Spark 3.5 value
semantics (docker/docker-compose.yml:67 pins apache/spark:3.5.2):

  :16-17  creation_ts_epoch = double(floorDiv(micros, 1e6))
  :28-29  ts_epoch = micros / 1e6 (double)
  :31-35  access_freq, writes, reads per path
  :37-42  local_accesses / total_accesses via the left join on path
  :44-46  max over floor(ts_epoch) of per-(path, sec) counts
  :48-54  observation_end = max(ts_epoch); age = end - creation
  :56-60  manifest-order left joins, nulls -> 0
  :62-68  write_ratio = writes / mean(writes) (0 -> 1.0); locality
  :77-94  min-max normalisation (max == min -> 0.0; longs as double(v-min)/...)

PARITY UNPINNED against Spark itself (no PySpark/Java in this image): the
timestamp parsing is a restatement of Spark's ISO-8601 handling; integer
counts are pinned by an independent group-by.
"""
from __future__ import annotations

import csv
import math

import numpy as np
import pandas as pd


def _ts_us(series: pd.Series) -> pd.Series:
    t = pd.to_datetime(series, format="ISO8601", utc=True, errors="coerce")
    return pd.Series(t.astype("int64") // 1000, index=series.index).where(t.notna())


def compute(manifest_csv: str, log_csv: str):
    man = pd.read_csv(manifest_csv, dtype=str, keep_default_na=False)
    cr_us = _ts_us(man["creation_ts"])
    creation = np.floor(cr_us.to_numpy(dtype=np.float64) / 1e6)
    rows = []
    with open(log_csv, newline="") as fh:
        for rec in csv.reader(fh):
            if rec:
                rows.append((rec + [""] * 5)[:5])
    log = pd.DataFrame(rows, columns=["ts", "path", "op", "client", "pid"])
    us = _ts_us(log["ts"]).astype("int64") if len(log) else pd.Series([], dtype="int64")
    log["sec"] = np.floor(us.to_numpy(dtype=np.int64) / 1e6).astype(np.int64) if len(log) else []
    log["w"] = (log["op"] == "WRITE").astype(np.int64)
    log["r"] = (log["op"] == "READ").astype(np.int64)
    prim = dict(zip(man["path"], man["primary_node"]))
    log["loc"] = [1 if (c != "" and prim.get(p, None) not in (None, "") and c == prim[p]) else 0
                  for p, c in zip(log["path"], log["client"])]
    g = log.groupby("path")
    agg = pd.DataFrame({"access_freq": g.size(), "writes": g["w"].sum(), "reads": g["r"].sum(),
                        "local": g["loc"].sum()})
    conc = log.groupby(["path", "sec"]).size().groupby(level=0).max()
    agg["conc"] = conc
    if len(log):
        obs_end = float(us.max()) / 1e6
    else:
        obs_end = None
    n = len(man)
    af = np.zeros(n, dtype=np.int64)
    wr = np.zeros(n, dtype=np.int64)
    lo = np.zeros(n, dtype=np.int64)
    co = np.zeros(n, dtype=np.int64)
    for i, p in enumerate(man["path"]):
        if p in agg.index:
            a = agg.loc[p]
            af[i], wr[i], lo[i], co[i] = a["access_freq"], a["writes"], a["local"], a["conc"]
    age = np.where(np.isnan(creation), 0.0, (obs_end if obs_end is not None else 0.0) - creation)
    mean_w = float(wr.sum()) / n if n else 0.0
    if mean_w == 0:
        mean_w = 1.0
    write_ratio = wr / mean_w
    locality = np.where(af > 0, lo / np.maximum(af, 1), 1.0)

    def norm_long(v):
        mn, mx = int(v.min()), int(v.max())
        return np.zeros(n) if mx == mn else (v - mn).astype(np.float64) / float(mx - mn)

    def norm_dbl(v):
        mn, mx = float(v.min()), float(v.max())
        return np.zeros(n) if mx == mn else (v - mn) / (mx - mn)

    table = np.column_stack([af.astype(np.float64), age, write_ratio, locality,
                             co.astype(np.float64), norm_long(af), norm_dbl(age),
                             norm_dbl(write_ratio), norm_dbl(locality), norm_long(co)])
    counts = np.column_stack([af, wr, np.zeros(n, dtype=np.int64), lo, af, co])
    return list(man["path"]), table, counts, obs_end


def counts_from_arrays(file_idx, op, client, ts_us, primary, n_files):
    """Independent per-file counters from encoded arrays (for the device K5)."""
    out = np.zeros((n_files, 6), dtype=np.int64)
    ok = (file_idx >= 0) & (file_idx < n_files)
    f = file_idx[ok].astype(np.int64)
    o = op[ok]
    c = client[ok]
    sec = np.floor(ts_us[ok] / 1e6).astype(np.int64)
    np.add.at(out[:, 0], f, 1)
    np.add.at(out[:, 1], f, (o == 1).astype(np.int64))
    np.add.at(out[:, 2], f, (o == 2).astype(np.int64))
    pr = primary[f]
    np.add.at(out[:, 3], f, ((c >= 0) & (pr >= 0) & (c == pr)).astype(np.int64))
    out[:, 4] = out[:, 0]
    if f.size:
        key = f * (1 << 33) + (sec - sec.min())
        uk, cnt = np.unique(key, return_counts=True)
        files = uk // (1 << 33)
        np.maximum.at(out[:, 5], files, cnt)
    mx = int(ts_us.max()) if ts_us.size else None
    return out, mx


def finalize(counts, creation_s, obs_end):
    """K6 restatement from counts (n, 6) and creation seconds (NaN = null)."""
    n = counts.shape[0]
    af, w, lo, tot, co = counts[:, 0], counts[:, 1], counts[:, 3], counts[:, 4], counts[:, 5]
    age = np.where(np.isnan(creation_s), 0.0, obs_end - creation_s)
    mean_w = float(int(w.sum())) / n if n else 0.0
    if mean_w == 0:
        mean_w = 1.0
    wr = w.astype(np.float64) / mean_w
    loc = np.where(tot > 0, lo.astype(np.float64) / np.maximum(tot, 1).astype(np.float64), 1.0)

    def nl(v):
        mn, mx = int(v.min()), int(v.max())
        return np.zeros(n) if mx == mn else (v - mn).astype(np.float64) / float(mx - mn)

    def nd(v):
        mn, mx = float(v.min()), float(v.max())
        return np.zeros(n) if mx == mn else (v - mn) / (mx - mn)

    return np.column_stack([af.astype(np.float64), age, wr, loc, co.astype(np.float64),
                            nl(af), nd(age), nd(wr), nd(loc), nl(co)])


def java_double_check(x: float) -> float:
    """Round trip helper for CSV tests."""
    return float(x) if not math.isnan(x) else x


# ---- access-log read (csrc/ingest.hip's checker) ---------------------------
# The reference reads the log with spark.read.csv + to_timestamp
# (src/compute_features.py:19-29) and joins path against the manifest (:37).
# Restated here with python's csv module (the simulator's format,
# src/access_simulator.py:61-63) and the ISO-8601 grammar the build pins
# (compute_features.parse_ts_us): regex match, calendar validation, UTC unless
# a zone is given, fraction truncated to microseconds.
import re as _re  # noqa: E402
import datetime as _dt  # noqa: E402

_ISO_RE = _re.compile(
    r"^\s*(\d{4})-(\d{1,2})-(\d{1,2})(?:[T ](\d{1,2}):(\d{1,2})(?::(\d{1,2})(?:\.(\d{1,9}))?)?)?"
    r"\s*(Z|[+-]\d{2}(?::?\d{2})?)?\s*$")
TS_NULL = -(2 ** 63)


def iso_to_us(s):
    """ISO-8601 string -> UTC microseconds, or None (Spark null)."""
    if s is None:
        return None
    m = _ISO_RE.match(s)
    if not m:
        return None
    y, mo, d, hh, mi, ss, frac, zone = m.groups()
    hh, mi, ss = int(hh or 0), int(mi or 0), int(ss or 0)
    if hh > 23 or mi > 59 or ss > 59:
        return None
    yy = int(y)
    try:
        # datetime has no year 0 (1 BCE): it is leap like 2000 and ends 366
        # days before 0001-01-01 (day -719162 from the epoch)
        base = _dt.date(yy if yy >= 1 else 2000, int(mo), int(d))
    except ValueError:
        return None
    if yy == 0:
        days = (base - _dt.date(2000, 1, 1)).days - 719162 - 366
    else:
        days = (base - _dt.date(1970, 1, 1)).days
    us = int((frac or "").ljust(6, "0")[:6] or 0)
    off = 0
    if zone and zone != "Z":
        z = zone[1:].replace(":", "")
        off = (-1 if zone[0] == "-" else 1) * (int(z[:2]) * 3600 + int(z[2:4] or 0) * 60)
    return ((days * 86400 + hh * 3600 + mi * 60 + ss) - off) * 1_000_000 + us


def encode_log(log_bytes: bytes, paths, primary):
    """Events of a log as the device ingest encodes them: file row (first
    manifest row of the path, -1), op (1 WRITE, 2 READ, 0), client (node id
    of a primary name in first-appearance order, -1 null, -3 other), ts in
    microseconds (TS_NULL when unparseable)."""
    import io

    row = {}
    for i, p in enumerate(paths):
        if p:
            row.setdefault(p, i)
    node = {}
    for v in primary:
        if v:
            node.setdefault(v, len(node))
    f, o, c, t = [], [], [], []
    for rec in csv.reader(io.StringIO(log_bytes.decode("utf-8"), newline="")):
        if not rec:
            continue
        rec = rec + [""] * (5 - len(rec))
        f.append(row.get(rec[1], -1) if rec[1] else -1)
        o.append(1 if rec[2] == "WRITE" else (2 if rec[2] == "READ" else 0))
        c.append(-1 if not rec[3] else node.get(rec[3], -3))
        u = iso_to_us(rec[0] or None)
        t.append(TS_NULL if u is None else u)
    return (np.array(f, dtype=np.int32), np.array(o, dtype=np.uint8),
            np.array(c, dtype=np.int32), np.array(t, dtype=np.int64))
