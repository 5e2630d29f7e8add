"""Per-file feature extraction on MI355X (drop-in for ``src/compute_features.py``).

Same CLI as the reference's PySpark job, so ``run_pipeline.sh:206-215`` and
``Makefile:45-60`` drive it unchanged (``spark-submit`` -> ``python``)::

    python compute_features.py --manifest M --access_log L --out OUT

and the same output: a directory ``OUT`` holding one ``part-00000-*.csv`` with a
header and the columns ``path, access_freq, age_seconds, write_ratio,
locality, concurrency, access_freq_norm, age_norm, write_ratio_norm,
locality_norm, concurrency_norm`` (src/compute_features.py:70-96), which
``src/main.py:155-168`` globs.

Host side (plumbing): the manifest CSV and its dictionaries.  Device side
(libcdr): the access-log read of :19-29 and the path join of :37
(``cdr_ingest_log``: tokenising, ISO-8601 timestamps -> microseconds, hash
lookups of paths and client nodes, csrc/ingest.hip), the group-by counters of
:31-46 (``cdr_features_aggregate_resident``) and the finalisation / min-max
normalisation of :48-94 (``cdr_features_finalize``).  A log with CSV quoting
(or NUL bytes, lone CRs, non-ASCII timestamps), which the reference's
simulator never writes, is tokenised on the host by ``load_access_log`` and
aggregated on the device the same way.

Spark semantics kept (Spark 3.5, docker/docker-compose.yml:67):
  * ``to_timestamp`` of ISO strings -> microseconds; ``cast(ts as double)`` =
    micros / 1e6; ``floor`` of that is the concurrency second;
  * ``unix_timestamp(to_timestamp(creation_ts))`` = floor(micros / 1e6) as double;
  * ``avg(writes)`` = double(sum) / count; ``long / long`` divides as doubles;
  * rows in manifest order (Spark's order is unspecified; main.py's seed
    depends on row order, so the build pins the manifest order);
  * an unparseable or empty timestamp is null (non-ANSI ``to_timestamp``): the
    event still counts (:31-42), the nulls of a file form one more second
    group (:44-46), and ``max(ts_epoch)`` ignores them (:48; all null ->
    ``time.time()``, :50-51);
  * a path listed twice in the manifest is joined as Spark joins it: every
    event meets every manifest row of its path in the locality join (:37-42),
    and the age join (:56-59) pairs every manifest row of the path with every
    row of it again, so m rows give m * m output rows (manifest row order,
    then age-row order); an empty path is null and joins nothing (age 0).
    The reference's generators never write either case: parity unpinned.
  * doubles written like Java's ``Double.toString`` (decimal in [1e-3, 1e7),
    otherwise ``d.dddE<exp>``), longs as integers.  The digits are those of
    the JDK that runs Spark: apache/spark:3.5.2 ships a pre-19 JDK, whose
    ``FloatingDecimal`` does not always print the shortest digits
    (``java_double_legacy``, the default).  ``CDR_JAVA_DOUBLE=19`` selects the
    JDK 19+ shortest-digit layout (``java_double``).
"""
from __future__ import annotations

import argparse
import csv
import math
import os
import re
import struct
import time
import uuid
from decimal import Decimal

import numpy as np

from _cdr import Context, default_context

OUT_COLUMNS = ["path", "access_freq", "age_seconds", "write_ratio", "locality", "concurrency",
               "access_freq_norm", "age_norm", "write_ratio_norm", "locality_norm",
               "concurrency_norm"]
LONG_COLUMNS = {"access_freq", "concurrency"}
TS_NULL = -(2 ** 63)  # a null timestamp in the device events (include/cdr.h)

_ISO = re.compile(
    r"^\s*(\d{4})-(\d{1,2})-(\d{1,2})(?:[T ](\d{1,2}):(\d{1,2})(?::(\d{1,2})(?:\.(\d{1,9}))?)?)?"
    r"\s*(Z|[+-]\d{2}(?::?\d{2})?)?\s*$")


def _strip_scheme(path: str) -> str:
    return path[len("file://"):] if path.startswith("file://") else path


def parse_ts_us(s) -> int | None:
    """Spark ``to_timestamp`` of an ISO-8601 string -> microseconds (UTC when
    no zone is given; fraction truncated to microseconds).  None = null."""
    if s is None:
        return None
    m = _ISO.match(str(s))
    if not m:
        return None
    y, mo, d, hh, mi, ss, frac, zone = m.groups()
    try:
        days = _days_from_civil(int(y), int(mo), int(d))
    except ValueError:
        return None
    hh, mi, ss = int(hh or 0), int(mi or 0), int(ss or 0)
    if hh > 23 or mi > 59 or ss > 59:
        return None
    us = int((frac or "").ljust(6, "0")[:6] or 0)
    off = 0
    if zone and zone != "Z":
        sign = -1 if zone[0] == "-" else 1
        z = zone[1:].replace(":", "")
        off = sign * (int(z[:2]) * 3600 + int(z[2:4] or 0) * 60)
    return ((days * 86400 + hh * 3600 + mi * 60 + ss) - off) * 1_000_000 + us


def _days_from_civil(y: int, m: int, d: int) -> int:
    if not (1 <= m <= 12):
        raise ValueError
    mdays = [31, 29 if (y % 4 == 0 and (y % 100 != 0 or y % 400 == 0)) else 28, 31, 30, 31,
             30, 31, 31, 30, 31, 30, 31]
    if not (1 <= d <= mdays[m - 1]):
        raise ValueError
    y2 = y - (m <= 2)
    era = (y2 if y2 >= 0 else y2 - 399) // 400
    yoe = y2 - era * 400
    doy = (153 * (m + (-3 if m > 2 else 9)) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def java_double(x: float) -> str:
    """``Double.toString`` of JDK 19+: the shortest round-trip digits."""
    x = float(x)
    if x != x:
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    t = Decimal(repr(abs(x))).as_tuple()
    digits = "".join(map(str, t.digits)).rstrip("0") or "0"
    exp10 = len(t.digits) + t.exponent - 1  # position of the leading digit
    if len(digits) == 1 and abs(x) < 2.2250738585072014e-308:
        # JDK 19+ Double.toString: when the shortest decimal has one digit,
        # two-digit decimals that round to x compete and the closest to x
        # wins (only subnormals near 4.9E-324 have one): Double.MIN_VALUE
        # prints as 4.9E-324, not 5.0E-324
        exact = Decimal(abs(x))
        best, bd = None, abs(Decimal(digits + "E" + str(exp10)) - exact)
        for lead in (exp10, exp10 - 1):  # two-digit decimals of this decade or the one below
            for c in range(10, 100):
                cand = Decimal(f"{c}E{lead - 1}")
                if float(cand) == abs(x) and abs(cand - exact) < bd:
                    best, bd = (str(c), lead), abs(cand - exact)
        if best is not None:
            digits, exp10 = best[0].rstrip("0"), best[1]
    if 1e-3 <= abs(x) < 1e7:
        if exp10 >= 0:
            ip = digits[: exp10 + 1].ljust(exp10 + 1, "0")
            fp = digits[exp10 + 1:] or "0"
        else:
            ip = "0"
            fp = "0" * (-exp10 - 1) + digits
        return f"{sign}{ip}.{fp}"
    mant = digits[0] + "." + (digits[1:] or "0")
    return f"{sign}{mant}E{exp10}"


# ---- pre-JDK-19 Double.toString -------------------------------------------
# Restated from the published algorithm of OpenJDK's
# jdk.internal.math.FloatingDecimal.BinaryToASCIIBuffer (JDK 8 to 18; the JDK is
# not part of the reference, which reaches it through Spark's CSV writer,
# src/compute_features.py:96): Steele & White digit generation with a symmetric
# half-ulp stopping test, a decimal-exponent estimate from a linear fit of
# log10, a direct path for integers below 2^63 that keeps all their digits up
# to a power-of-two-derived rounding position, and at least two digits in
# E-notation.  Pinned by the outputs JDK bug 4511638 lists (tests/test_host_logic.py).

_N5_BITS = [(5 ** i).bit_length() for i in range(27)]  # bit length of 5^i
_POW2_DEC_DIGITS = [len(str(1 << p)) - 1 for p in range(64)]  # floor(log10(2^p))


def _wrap(v: int, bits: int) -> int:
    """Two's-complement wrap (the int / long arithmetic of the fast paths)."""
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def _legacy_digits(bin_exp: int, fract: int, n_sig: int):
    """Digits and decimal exponent (value = 0.d1d2... x 10^exp) of
    fract * 2^(bin_exp - 52), fract normalised to 53 bits."""
    tail = (fract & -fract).bit_length() - 1
    n_fract = 53 - tail  # significant bits
    n_tiny = max(0, n_fract - bin_exp - 1)  # bits right of the binary point
    if n_tiny == 0 and -21 <= bin_exp <= 62:
        # an integer: all its digits, rounded (half up) at 10^i where 2^p
        # has i + 1 digits and p = bin_exp - n_sig - 1
        p = bin_exp - n_sig - 1
        drop = _POW2_DEC_DIGITS[p] if bin_exp > n_sig and 1 < p < 64 else 0
        v = fract << (bin_exp - 52) if bin_exp >= 52 else fract >> (52 - bin_exp)
        if drop:
            v, rem = divmod(v, 10 ** drop)
            v += rem >= (10 ** drop) >> 1
        txt = str(v)
        return [int(c) for c in txt.rstrip("0")], drop + len(txt)
    mant = struct.unpack("<d", struct.pack("<Q", 0x3FF0000000000000 | (fract & ((1 << 52) - 1))))[0]
    dec = math.floor((mant - 1.5) * 0.289529654 + 0.176091259 + bin_exp * 0.301029995663981)
    b5 = max(0, -dec)
    b2 = b5 + n_tiny + bin_exp
    s5 = max(0, dec)
    s2 = s5 + n_tiny
    m5, m2 = b5, b2 - n_sig
    fract >>= tail
    b2 -= n_fract - 1
    common = min(b2, s2)
    b2, s2, m2 = b2 - common, s2 - common, m2 - common
    if n_fract == 1:  # a power of two: the gap below is half as wide
        m2 -= 1
    if m2 < 0:
        b2, s2, m2 = b2 - m2, s2 - m2, 0
    b_bits = n_fract + b2 + (_N5_BITS[b5] if b5 < 27 else 3 * b5)
    ts_bits = s2 + 1 + (_N5_BITS[s5 + 1] if s5 + 1 < 27 else 3 * (s5 + 1))
    digits = []
    if b_bits < 64 and ts_bits < 64:
        # int (both < 32 bits) or long arithmetic; m may overflow as in Java
        w = 32 if b_bits < 32 and ts_bits < 32 else 64
        b = _wrap((fract * 5 ** b5) << b2, w)
        s = _wrap(5 ** s5 << s2, w)
        m = _wrap(5 ** m5 << m2, w)
        ts = _wrap(s * 10, w)
        q, b, m = b // s, _wrap(10 * (b % s), w), _wrap(m * 10, w)
        low, high = b < m, _wrap(b + m, w) > ts
        if q == 0 and not high:
            dec -= 1
        else:
            digits.append(q)
        if dec < -3 or dec >= 8:
            low = high = False
        while not low and not high:
            q, b, m = b // s, _wrap(10 * (b % s), w), _wrap(m * 10, w)
            if m > 0:
                low, high = b < m, _wrap(b + m, w) > ts
            else:
                low = high = True
            digits.append(q)
        tie = _wrap(_wrap(b << 1, w) - ts, w)
    else:
        s = 5 ** s5 << s2
        m = 5 ** (m5 + 1) << (m2 + 1)
        ts = 10 * s
        q, r = divmod((fract * 5 ** b5) << b2, s)
        b = 10 * r
        low, high = b < m, ts <= b + m
        if q == 0 and not high:
            dec -= 1
        else:
            digits.append(q)
        if dec < -3 or dec >= 8:
            low = high = False
        while not low and not high:
            q, r = divmod(b, s)
            b, m = 10 * r, m * 10
            low, high = b < m, ts <= b + m
            digits.append(q)
        tie = (2 * b > ts) - (2 * b < ts) if high and low else 0
    exp = dec + 1
    if high and (not low or tie > 0 or (tie == 0 and digits[-1] & 1)):
        i = len(digits) - 1
        while digits[i] == 9 and i > 0:
            digits[i] = 0
            i -= 1
        if digits[i] == 9:  # 9...9 -> 10...0
            digits[0] = 1
            exp += 1
        else:
            digits[i] += 1
    return digits, exp


def java_double_legacy(x: float) -> str:
    """``Double.toString`` of a JDK 8-18 (the JVM of apache/spark:3.5.2,
    docker/docker-compose.yml:67), e.g. 2e23 -> ``1.9999999999999998E23``."""
    x = float(x)
    if x != x:
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    bits = struct.unpack("<Q", struct.pack("<d", x))[0]
    sign = "-" if bits >> 63 else ""
    fract, be = bits & ((1 << 52) - 1), (bits >> 52) & 0x7FF
    if be == 0:
        if fract == 0:
            return sign + "0.0"
        shift = 53 - fract.bit_length()
        fract, be, n_sig = fract << shift, 1 - shift, fract.bit_length()
    else:
        fract, n_sig = fract | (1 << 52), 53
    digits, exp = _legacy_digits(be - 1023, fract, n_sig)
    d = "".join(map(str, digits))
    if 0 < exp < 8:
        if len(d) <= exp:
            return f"{sign}{d.ljust(exp, '0')}.0"
        return f"{sign}{d[:exp]}.{d[exp:]}"
    if -3 < exp <= 0:
        return f"{sign}0.{'0' * -exp}{d}"
    return f"{sign}{d[0]}.{d[1:] or '0'}E{exp - 1}"


def _double_formatter():
    mode = os.environ.get("CDR_JAVA_DOUBLE", "legacy")
    if mode not in ("legacy", "19"):
        raise ValueError(f"CDR_JAVA_DOUBLE={mode!r}: expected 'legacy' or '19'")
    return java_double if mode == "19" else java_double_legacy


def load_manifest(path: str):
    """Manifest CSV (header; path, creation_ts, primary_node, ...) -> columns."""
    with open(_strip_scheme(path), newline="") as fh:
        rows = list(csv.DictReader(fh))
    paths = [r.get("path") for r in rows]
    created = np.array([np.nan if (u := parse_ts_us(r.get("creation_ts"))) is None
                        else float(u // 1_000_000) for r in rows], dtype=np.float64)
    primary = [r.get("primary_node") or None for r in rows]
    return paths, created, primary


def load_access_log(path: str):
    """Header-less ``ts,path,op,client,pid`` CSV (src/access_simulator.py:61-63)."""
    ts, p, op, cl = [], [], [], []
    with open(_strip_scheme(path), newline="") as fh:
        for rec in csv.reader(fh):
            if not rec:
                continue
            rec = rec + [""] * (5 - len(rec))
            ts.append(rec[0] or None)
            p.append(rec[1] or None)
            op.append(rec[2] or None)
            cl.append(rec[3] or None)
    return ts, p, op, cl


def encode(paths, primary, log_ts, log_path, log_op, log_client):
    """Dictionary-encode strings for the device."""
    index = {}
    for i, pth in enumerate(paths):
        index.setdefault(pth, i)
    nodes = {}

    def node_id(name):
        return nodes.setdefault(name, len(nodes))

    prim = np.array([-2 if v is None else node_id(v) for v in primary], dtype=np.int32)
    n = len(log_ts)
    file_idx = np.empty(n, dtype=np.int32)
    opc = np.empty(n, dtype=np.uint8)
    client = np.empty(n, dtype=np.int32)
    ts_us = np.empty(n, dtype=np.int64)
    for i in range(n):
        file_idx[i] = index.get(log_path[i], -1) if log_path[i] is not None else -1
        o = log_op[i]
        opc[i] = 1 if o == "WRITE" else (2 if o == "READ" else 0)
        c = log_client[i]
        client[i] = -1 if c is None else node_id(c)
        u = parse_ts_us(log_ts[i])
        ts_us[i] = TS_NULL if u is None else u  # Spark: null timestamp
    return file_idx, opc, client, ts_us, prim


def encode_primary(primary):
    """Node ids of the primaries (first-appearance order, -2 = null) and the
    node names in id order: the ids ``encode`` gives them."""
    nodes = {}
    prim = np.array([-2 if v is None else nodes.setdefault(v, len(nodes)) for v in primary],
                    dtype=np.int32)
    return prim, list(nodes)


def ingest_events(ctx: Context, paths, primary, access_log: str) -> int:
    """Access log -> resident device events of ``ctx``; returns the count."""
    prim, nodes = encode_primary(primary)
    ctx.ingest_manifest(paths, prim, nodes)
    with open(_strip_scheme(access_log), "rb") as fh:
        data = fh.read()
    st = ctx.ingest_log(data)
    if st[2] >= 0:
        return -1  # csv syntax the device tokeniser leaves to the host
    return int(st[0])  # (unparseable timestamps are null events, st[3] of them)


def expand_joins(paths, created, primary, counts, events):
    """Spark's join multiplicity for the manifest (src/compute_features.py:37,
    :56-59).  ``counts`` (n, 6) has every event of a path on its first
    manifest row (the device dictionary's row); ``events`` () -> (file, client)
    arrays of the events, read only when a path repeats.  Returns the output
    rows: (paths, counts, creation seconds), one row per manifest row, m * m
    rows for a path listed m times; an empty (null) path joins nothing."""
    rows_of = {}
    for i, p in enumerate(paths):
        if p:
            rows_of.setdefault(p, []).append(i)
    created = np.where([bool(p) for p in paths], created, np.nan) if len(paths) else created
    dup = {p: r for p, r in rows_of.items() if len(r) > 1}
    if not dup:
        return list(paths), counts, created
    f_ev, c_ev = events()
    prim, _ = encode_primary(primary)
    local = {}
    for p, rows in dup.items():
        cl = c_ev[f_ev == rows[0]]
        local[p] = sum(int(np.count_nonzero((cl >= 0) & (cl == prim[r]))) for r in rows
                       if prim[r] >= 0)
    out_p, out_c, out_t = [], [], []
    for i, p in enumerate(paths):
        if p not in dup:
            out_p.append(p)
            out_c.append(counts[i])
            out_t.append(created[i])
            continue
        rows = dup[p]
        c = counts[rows[0]].copy()
        c[3] = local[p]              # every event meets every manifest row (:37)
        c[4] = c[4] * len(rows)
        for j in rows:               # the age join pairs row i with every row j (:56-59)
            out_p.append(p)
            out_c.append(c)
            out_t.append(created[j])
    return out_p, np.array(out_c, dtype=np.int64).reshape(-1, 6), np.array(out_t)


def compute_features(manifest: str, access_log: str, ctx: Context | None = None):
    """Returns (paths, table) with table (rows, 10) float64 in OUT_COLUMNS order
    (one row per manifest row; see expand_joins for repeated paths)."""
    ctx = ctx if ctx is not None else default_context()
    paths, created, primary = load_manifest(manifest)
    n_events = ingest_events(ctx, paths, primary, access_log) if paths else -1
    if n_events >= 0:
        counts, max_ts_us = ctx.features_aggregate_resident()

        def events():
            f, _, cl, _, _ = ctx.features_events_read()
            return f, cl
    else:
        lt, lp, lo, lc = load_access_log(access_log)
        file_idx, opc, client, ts_us, prim = encode(paths, primary, lt, lp, lo, lc)
        counts, max_ts_us = ctx.features_aggregate(file_idx, opc, client, ts_us, prim)

        def events():
            return file_idx, client
    if max_ts_us != TS_NULL:
        observation_end = max_ts_us / 1e6  # max(cast(ts as double)) :48
    else:
        observation_end = time.time()  # no events or every timestamp null :50-51
    paths, counts, created = expand_joins(paths, created, primary, counts, events)
    table = ctx.features_finalize(counts, created, observation_end)
    return paths, table


def write_spark_csv(out_dir: str, paths, table, fmt=None) -> str:
    """One part file with a header, like ``coalesce(1).write.csv`` (:96).
    ``fmt`` formats the doubles (default: ``CDR_JAVA_DOUBLE``, see above)."""
    fmt = fmt or _double_formatter()
    out_dir = _strip_scheme(out_dir)
    if os.path.isdir(out_dir):  # mode("overwrite")
        for name in os.listdir(out_dir):
            os.remove(os.path.join(out_dir, name))
    os.makedirs(out_dir, exist_ok=True)
    part = os.path.join(out_dir, f"part-00000-{uuid.uuid4()}-c000.csv")
    with open(part, "w", newline="") as fh:
        w = csv.writer(fh, lineterminator="\n")
        w.writerow(OUT_COLUMNS)
        for i, pth in enumerate(paths):
            row = [pth]
            for j, col in enumerate(OUT_COLUMNS[1:]):
                v = table[i, j]
                row.append(str(int(v)) if col in LONG_COLUMNS else fmt(v))
            w.writerow(row)
    open(os.path.join(out_dir, "_SUCCESS"), "w").close()
    return part


def main(argv=None):
    """Single process, or one rank per GPU under torch.distributed.run
    (WORLD_SIZE > 1: features_dist.sharded_compute_features over RCCL; rank 0
    writes the CSV)."""
    parser = argparse.ArgumentParser()
    parser.add_argument("--manifest", required=True)
    parser.add_argument("--access_log", required=True)
    parser.add_argument("--out", default="features_out")
    args = parser.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch
        import torch.distributed as dist

        from cdr_dist import Comm, bind_stream
        from features_dist import sharded_compute_features

        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        ctx = Context(local)
        bind_stream(ctx, torch.device("cuda", local))
        paths, table = sharded_compute_features(args.manifest, args.access_log, ctx,
                                                Comm(dist, torch.device("cuda", local)))
        if dist.get_rank() == 0:
            write_spark_csv(args.out, paths, table)
            print("Wrote features to", args.out)
        ctx.close()
        dist.destroy_process_group()
        return
    paths, table = compute_features(args.manifest, args.access_log)
    write_spark_csv(args.out, paths, table)
    print("Wrote features to", args.out)


if __name__ == "__main__":
    main()
