"""pandas restatement of the reference PySpark job (TEST INFRASTRUCTURE ONLY).

Follows /root/reference/src/compute_features.py:14-94 with Spark 3.5 value
semantics (docker/docker-compose.yml:67 pins apache/spark:3.5.2), one pandas
step per Spark statement:

  :16-17  creation_ts_epoch = double(floorDiv(micros, 1e6))
  :28-29  ts_epoch = micros / 1e6 (double); unparseable / empty -> null
  :31-35  access_freq, writes, reads per path
  :37-42  local_accesses / total_accesses via the left join on path (an event
          meets every manifest row of its path; null keys match nothing)
  :44-46  max over floor(ts_epoch) of per-(path, sec) counts (null sec = group)
  :48-54  observation_end = max(ts_epoch) skipping nulls (none -> now);
          age = end - creation
  :56-60  manifest-order left joins (m rows of a path x m age rows), nulls -> 0
  :62-68  write_ratio = writes / mean(writes) (0 -> 1.0); locality
  :77-94  min-max normalisation (max == min -> 0.0; longs as double(v-min)/...)

PARITY UNPINNED against Spark itself (no PySpark/Java in this image): the
timestamp parsing is a restatement of Spark's ISO-8601 handling; integer
counts are pinned by an independent group-by (counts_from_arrays); the null
and repeated-path rules are pinned by hand-derived values
(tests/test_spark_semantics.py).
"""
from __future__ import annotations

import csv
import math
import time

import numpy as np
import pandas as pd


def _ts_us(series: pd.Series) -> list:
    """to_timestamp (:17, :28) of each string -> UTC microseconds or None."""
    t = pd.to_datetime(pd.Series(series, dtype=object), format="ISO8601", utc=True,
                       errors="coerce")
    us = t.astype("int64") // 1000
    return [int(u) if ok else None for u, ok in zip(us, t.notna())]


def _keys(paths, tag):
    """Join keys: Spark's equi-join never matches a null key, pandas merges
    NaN with NaN -- so a null path gets a per-row key that matches nothing."""
    return [p if isinstance(p, str) else f"\0{tag}{i}" for i, p in enumerate(paths)]


def _nulls(df: pd.DataFrame) -> pd.DataFrame:
    """spark.read.csv: an empty field is null."""
    df = df.astype(object)
    return df.where(df != "", None)


def compute(manifest_csv: str, log_csv: str, now=None):
    """The reference job, one pandas step per Spark statement.  Returns
    (paths, table (rows, 10), counts (rows, 6): access_freq, writes, reads,
    local_accesses, total_accesses, max_concurrency, observation_end)."""
    man = _nulls(pd.read_csv(manifest_csv, dtype=str, keep_default_na=False))
    cr = _ts_us(man["creation_ts"])                                        # :16-17
    man["creation_ts_epoch"] = [np.nan if u is None else float(u // 1_000_000) for u in cr]
    rows = []
    with open(log_csv, newline="") as fh:                                  # :19-26
        for rec in csv.reader(fh):
            if rec:
                rows.append((rec + [""] * 5)[:5])
    log = _nulls(pd.DataFrame(rows, columns=["ts_iso", "path", "op", "client_node", "pid"],
                              dtype=object))
    log["ts_epoch"] = [np.nan if u is None else u / 1e6 for u in _ts_us(log["ts_iso"])]  # :28-29
    log["w"] = (log["op"] == "WRITE").astype(np.int64)                     # :31-35
    log["r"] = (log["op"] == "READ").astype(np.int64)
    freq = log.groupby("path").agg(access_freq=("w", "size"), writes=("w", "sum"),
                                   reads=("r", "sum"))
    lk = log.assign(key=_keys(log["path"], "l"))                           # :37
    mk = pd.DataFrame({"key": _keys(man["path"], "m"), "primary_node": man["primary_node"]})
    awp = lk.merge(mk, on="key", how="left")
    awp["is_local"] = [1 if isinstance(c, str) and isinstance(p, str) and c == p else 0
                       for c, p in zip(awp["client_node"], awp["primary_node"])]  # :38-39
    loc = awp.groupby("path").agg(local_accesses=("is_local", "sum"),      # :40-42
                                  total_accesses=("is_local", "size"))
    log["sec"] = np.floor(log["ts_epoch"].astype(np.float64))              # :44-46
    conc = (log.groupby(["path", "sec"], dropna=False).size().groupby(level=0).max()
            .rename("max_concurrency").to_frame())
    mx = log["ts_epoch"].astype(np.float64).max() if len(log) else np.nan  # :48-51
    obs_end = float(mx) if not np.isnan(mx) else (time.time() if now is None else now)
    age = pd.DataFrame({"key": _keys(man["path"], "a"),                    # :53-54
                        "age_seconds": float(obs_end) - man["creation_ts_epoch"].astype(np.float64)})

    def keyed(df):
        df = df.reset_index()
        return df.assign(key=df["path"]).drop(columns="path")

    j = pd.DataFrame({"key": _keys(man["path"], "j"), "path": man["path"]})  # :56-59
    j = (j.merge(keyed(freq), on="key", how="left").merge(keyed(loc), on="key", how="left")
         .merge(keyed(conc), on="key", how="left").merge(age, on="key", how="left"))
    longs = ["access_freq", "writes", "reads", "local_accesses", "total_accesses",
             "max_concurrency"]
    for cname in longs:                                                    # :60
        j[cname] = j[cname].fillna(0).astype(np.int64)
    j["age_seconds"] = j["age_seconds"].fillna(0.0).astype(np.float64)
    n = len(j)
    mean_w = float(j["writes"].sum()) / n if n else 0.0                    # :62-65
    if mean_w == 0:
        mean_w = 1.0
    af, co = j["access_freq"].to_numpy(), j["max_concurrency"].to_numpy()
    lo, tot = j["local_accesses"].to_numpy(), j["total_accesses"].to_numpy()
    age_s = j["age_seconds"].to_numpy()
    write_ratio = j["writes"].to_numpy() / mean_w                          # :66
    locality = np.where(tot > 0, lo / np.maximum(tot, 1), 1.0)             # :68

    def norm_long(v):                                                      # :77-94
        if n == 0:
            return np.zeros(0)
        mn, mx_ = int(v.min()), int(v.max())
        return np.zeros(n) if mx_ == mn else (v - mn).astype(np.float64) / float(mx_ - mn)

    def norm_dbl(v):
        if n == 0:
            return np.zeros(0)
        mn, mx_ = float(v.min()), float(v.max())
        return np.zeros(n) if mx_ == mn else (v - mn) / (mx_ - mn)

    table = np.column_stack([af.astype(np.float64), age_s, write_ratio, locality,
                             co.astype(np.float64), norm_long(af), norm_dbl(age_s),
                             norm_dbl(write_ratio), norm_dbl(locality), norm_long(co)])
    counts = j[longs].to_numpy(dtype=np.int64).reshape(-1, 6)
    return list(j["path"]), table.reshape(-1, 10), counts, obs_end


def counts_from_arrays(file_idx, op, client, ts_us, primary, n_files):
    """Independent per-file counters from encoded arrays (for the device K5);
    ts TS_NULL is a null timestamp (its own second group, not in the max)."""
    out = np.zeros((n_files, 6), dtype=np.int64)
    ok = (file_idx >= 0) & (file_idx < n_files)
    f = file_idx[ok].astype(np.int64)
    o = op[ok]
    c = client[ok]
    t = ts_us[ok]
    null = t == TS_NULL
    np.add.at(out[:, 0], f, 1)
    np.add.at(out[:, 1], f, (o == 1).astype(np.int64))
    np.add.at(out[:, 2], f, (o == 2).astype(np.int64))
    pr = primary[f]
    np.add.at(out[:, 3], f, ((c >= 0) & (pr >= 0) & (c == pr)).astype(np.int64))
    out[:, 4] = out[:, 0]
    if f.size:
        sec = np.floor(np.where(null, 0, t) / 1e6).astype(np.int64)
        sec[null] = np.iinfo(np.int64).max  # the null second: one more group per file
        order = np.lexsort((sec, f))
        fs, ss = f[order], sec[order]
        start = np.ones(fs.size, dtype=bool)
        start[1:] = (fs[1:] != fs[:-1]) | (ss[1:] != ss[:-1])
        idx = np.flatnonzero(start)
        cnt = np.diff(np.append(idx, fs.size))
        np.maximum.at(out[:, 5], fs[idx], cnt)
    real = ts_us[ts_us != TS_NULL]
    mx = int(real.max()) if real.size else None
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
