"""Python model of a shard's cumsum program (include/cdr.h cdr_seed_item,
csrc/seed.hip seg_block_kernel) for the CPU tests: runs of elements whose
guessed running value stays in one binade become RUN transfers, every other
element a CROSS.  Test infrastructure only (the device builds the real
programs); it lets the host evaluator and the sharded protocol be checked
against np.cumsum without a GPU."""
import math

import numpy as np

SEED_ITEM = np.dtype([("d0", "<i8"), ("d1", "<i8"), ("p", "<f8"), ("e", "<i4"),
                      ("kind", "<i4")])
RUN, CROSS, CONST, FINE, MARK, END, SKIP, BAD = range(8)


def binade(c: float):
    """Exponent e with 2^e <= c < 2^(e+1) for positive normal c, else None."""
    if not (c > 0.0) or c < 2.0 ** -1022 or math.isinf(c) or c >= 2.0 ** 1023:
        return None
    return math.frexp(c)[1] - 1


def near(c: float) -> bool:
    """Within 2^-24 of a binade edge (csrc/seed.hip gnear)."""
    m = int(np.float64(c).view(np.uint64)) & ((1 << 52) - 1)
    return m < (1 << 28) or m > (1 << 52) - (1 << 28)


def run_transfer(vals, e: int):
    """(d0, d1): grid steps (2^(e-52)) the sequential sum of vals adds to a
    running value in binade e that entered with an even / odd step count —
    measured by adding from the bottom of the binade, which is exact while
    the sum stays inside it (None: it does not)."""
    out = []
    for q in (0, 1):
        n0 = (1 << 52) + q
        c = math.ldexp(n0, e - 52)
        for v in vals:
            c = c + float(v)
        if c >= 2.0 ** (e + 1):
            return None
        out.append(int(c / math.ldexp(1.0, e - 52)) - n0)
    return out


def build_program(p, c_guess: float) -> np.ndarray:
    items = []
    run, e_run = [], None

    def flush():
        nonlocal run, e_run
        if run:
            t = run_transfer(run, e_run)
            items.append((t[0], t[1], 0.0, e_run, RUN) if t else (0, 0, 0.0, 0, BAD))
        run, e_run = [], None

    c = c_guess
    for v in np.asarray(p, dtype=np.float64):
        ca = c + v
        eb, ea = binade(c), binade(ca)
        if eb is None or eb != ea or near(c) or near(ca):
            flush()
            items.append((0, 0, float(v), 0, CROSS))
        else:
            if e_run is not None and e_run != eb:
                flush()
            e_run = eb
            run.append(v)
        c = ca
    flush()
    items.append((0, 0, 0.0, 0, END))
    return np.array(items, dtype=SEED_ITEM)
