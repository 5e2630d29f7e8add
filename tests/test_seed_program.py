"""Cumsum programs (include/cdr.h cdr_seed_program_eval): the host evaluator
that sharded seeding uses to compose the shards' exact np.cumsum carries
(src/kmeans_plusplus.py:19) instead of a rank-ordered chain.  Programs here
come from tests/seedprog_model.py (the device builds them in
csrc/seed.hip); the GPU side is tests/test_gpu_kmeans.py."""
import numpy as np
import pytest

from seedprog_model import BAD, CONST, CROSS, END, FINE, RUN, SEED_ITEM, SKIP, build_program


@pytest.fixture(scope="module")
def ev():
    import _cdr

    _cdr.load_library()
    return _cdr.seed_program_eval


def _exact(p, c_in):
    return float(np.cumsum(np.concatenate([[c_in], p]))[-1])


def _cases(seed=0):
    rng = np.random.default_rng(seed)
    for n in (1, 7, 300, 5000):
        for kind in ("exp", "heavy", "zeros", "ties"):
            if kind == "exp":
                d = rng.exponential(1.0, n)
            elif kind == "heavy":
                d = rng.pareto(1.2, n)
            elif kind == "zeros":
                d = rng.exponential(1.0, n) * (rng.random(n) < 0.3)
                d[-1] = 0.5  # a positive total
            else:  # dyadic values: exact ties in the running sum's rounding
                d = np.ldexp(rng.integers(1, 9, n).astype(np.float64), -rng.integers(0, 60, n))
            yield d


def test_program_from_exact_start_is_exact(ev):
    for d in _cases():
        total = float(d.sum()) * 1.25
        p = d / total
        for c_in in (0.0, 0.37, 0.5, 1e-300):
            prog = build_program(p, c_in)
            c, ok = ev(prog, c_in)
            assert ok
            assert c == _exact(p, c_in)


def test_wrong_guess_fails_or_is_exact(ev):
    """A program built from a guessed start either fails its own checks or
    gives exactly np.cumsum's carry."""
    rng = np.random.default_rng(3)
    n_fail = 0
    for d in _cases(1):
        p = d / float(d.sum())
        for c_in in (0.49999999, 0.25, 0.75):
            for guess in (c_in, c_in * (1 + 1e-12), c_in * 0.5, c_in * 1.5, 0.0):
                c, ok = ev(build_program(p, guess), c_in)
                if ok:
                    assert c == _exact(p, c_in)
                else:
                    n_fail += 1
    assert n_fail > 0  # the far-off guesses are caught


def test_shards_compose(ev):
    """Three shards: each program built from the approximate prefix, composed
    in order from 0.0 = np.cumsum over all rows."""
    rng = np.random.default_rng(5)
    d = rng.exponential(1.0, 30000) ** 3
    p = d / float(d.sum())
    cuts = [0, 11000, 21000, 30000]
    c = 0.0
    for a, b in zip(cuts[:-1], cuts[1:]):
        guess = float(p[:a].sum())
        c, ok = ev(build_program(p[a:b], guess), c)
        assert ok
    assert c == _exact(p, 0.0)


def test_item_kinds(ev):
    it = np.zeros(4, dtype=SEED_ITEM)
    it[0]["kind"], it[0]["p"] = CONST, 0.75
    it[1]["kind"] = SKIP
    it[2]["kind"], it[2]["p"] = CROSS, 0.125
    it[3]["kind"] = END
    assert ev(it, 123.0) == (0.875, True)
    # RUN: binade [0.5, 1): grid 2^-53; N = 0.75 * 2^53 is even -> d0
    run = np.zeros(1, dtype=SEED_ITEM)
    run[0]["kind"], run[0]["e"], run[0]["d0"], run[0]["d1"] = RUN, -1, 4, 5
    assert ev(run, 0.75) == (0.75 + 4 * 2.0 ** -53, True)
    assert ev(run, 0.75 + 2.0 ** -53) == (0.75 + 6 * 2.0 ** -53, True)
    assert ev(run, 0.25)[1] is False  # other binade
    assert ev(run, 1.0 - 2.0 ** -53)[1] is False  # leaves the binade
    for k in (BAD, FINE):
        bad = np.zeros(1, dtype=SEED_ITEM)
        bad[0]["kind"] = k
        assert ev(bad, 0.5)[1] is False
    assert ev(np.zeros(0, dtype=SEED_ITEM), 0.3) == (0.3, True)
