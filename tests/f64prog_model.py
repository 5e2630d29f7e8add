"""Python model of the sharded F64 sums (include/cdr.h cdr_f64s_*,
csrc/f64sum.hip f64s_program / f64s_compose) for the CPU tests: a shard's
part of every (cluster, feature) sequence as a program of RUN transfers
(member blocks predicted in one binade, no crossing inside) and ELEM values
(every other member), composed in rank order from the exact start.  Test
infrastructure only (the devices build the real programs); it lets the
sharded protocol be checked on gloo ranks against NumPy's sequential sums
without a GPU."""
import math

import numpy as np

F64_ITEM = np.dtype([("a", "<i8"), ("b", "<i8"), ("e", "<i4"), ("kind", "<i4")])
RUN, ELEM, CONST = 1, 2, 3
KFB = 256  # rows per block
TOP = 1 << 53


def binade(c):
    if not (c > 0.0) or c < 2.0 ** -1022 or math.isinf(c) or math.isnan(c):
        return None
    return math.frexp(c)[1] - 1


def _bits(x):
    return int(np.float64(x).view(np.int64))


def _val(bits):
    return float(np.int64(bits).view(np.float64))


def block_transfer(vals, e):
    """(d0, d1, p): grid steps the block's sequential additions add inside
    binade e for an even / odd entry and the exit parities, or None when an
    addend is negative or leaves the binade (xfer_pre's invalid flag)."""
    out = []
    for m in (1 << 52, (1 << 52) + 1):  # even / odd entries at the binade's bottom
        s = math.ldexp(float(m), e - 52)
        for x in vals:
            if not (x >= 0.0) or math.isinf(x):
                return None
            s = s + x
        if binade(s) != e:
            return None
        g = int(math.ldexp(s, 52 - e))
        out.append((g - m, g & 1))
    return out[0][0], out[1][0], out[0][1] | (out[1][1] << 1)


def compose(a, b):
    """xc_compose: a then b."""
    a0, a1 = a[2] & 1, (a[2] >> 1) & 1
    d0 = a[0] + (b[1] if a0 else b[0])
    d1 = a[1] + (b[1] if a1 else b[0])
    p = ((b[2] >> a0) & 1) | (((b[2] >> a1) & 1) << 1)
    return d0, d1, p


def shard_program(col, labels, j, offset, cap):
    """Items of shard r > 0 for sequence (j, column col): RUNs of member
    blocks whose predicted start binade (offset + the shard's approximate
    prefix) equals their predicted end binade and whose transfer is usable,
    ELEMs for the other members."""
    n = col.size
    nb = -(-n // KFB)
    blocks = []
    for b in range(nb):
        m = labels[b * KFB:(b + 1) * KFB] == j
        blocks.append(col[b * KFB:(b + 1) * KFB][m])
    approx = [float(np.sum(v)) for v in blocks]
    starts = offset + np.concatenate([[0.0], np.cumsum(approx)[:-1]]) if nb else np.zeros(0)
    end_all = offset + float(np.sum(approx))
    items, run = [], None

    def flush():
        nonlocal run
        if run is not None:
            items.append((run[0], run[1], run[3], RUN))
            run = None

    for b in range(nb):
        v = blocks[b]
        if v.size == 0:
            continue
        e = binade(starts[b])
        e_end = binade(starts[b + 1] if b + 1 < nb else end_all)
        x = block_transfer(v, e) if e is not None else None
        if x is not None and e_end == e:
            if run is not None and run[3] == e:
                c = compose(run[:3], x)
                run = (c[0], c[1], c[2], e)
            else:
                flush()
                run = (x[0], x[1], x[2], e)
        else:
            flush()
            items.extend((_bits(val), 0, 0, ELEM) for val in v)
    flush()
    if len(items) > cap:
        return None
    return items


def compose_programs(progs):
    """progs: per rank, a list of items (or None: overflow); returns (s,
    ok) — the exact sequential sum when every RUN's transfer test holds."""
    s, any_, ok = 0.0, False, True
    for items in progs:
        if items is None:
            return s, False
        for a, b, e, kind in items:
            if kind == RUN:
                if not (any_ and s > 0.0) or binade(s) != e:
                    return s, False
                g = int(math.ldexp(s, 52 - e))
                g2 = g + (b if g & 1 else a)
                if g2 >= TOP:
                    return s, False
                s = math.ldexp(float(g2), e - 52)
            elif kind == ELEM:
                v = _val(a)
                s = s + v if any_ else v
                any_ = True
            elif kind == CONST:
                s, any_ = _val(a), e != 0
    return s, ok
