"""CPU check of the hi-only screen's certificate (csrc/screen32.hip, screen32d
HO) in exact-enough fp64 arithmetic.

The kernel screens h = fp16(xhat) instead of xhat and certifies a point when
    v_s > v_b (1 + 2^-16) + thr0 + 2 dn (sqrt(G_s) + sqrt(G_b)),
    dn = 2^-11 (1 + 2^-9) ||h|| + 2^-23,  G = v - D + ||h||^2 + thr0.
Here the screen values are formed exactly from h (E = 0, so thr0 is only the
slack) and every certified point must have the true argmin of
||chat_j||^2 - 2 chat_j.xhat (the decision values of the reference's argmin)
at the screen's best, with a positive margin to every other centroid."""
import numpy as np


def _certify(xh, ch, D, thr0):
    h = xh.astype(np.float16).astype(np.float64)
    cc = (ch ** 2).sum(axis=1)
    S = D + cc[None, :] - 2.0 * h @ ch.T  # the screen values of the point h
    order = np.argsort(S, axis=1, kind="stable")
    b, s = order[:, 0], order[:, 1]
    rows = np.arange(len(xh))
    vb, vs = S[rows, b], S[rows, s]
    hh = (h ** 2).sum(axis=1)
    dn = 2.0 ** -11 * (1 + 2.0 ** -9) * np.sqrt(hh) + 2.0 ** -23
    Gs = np.maximum(vs - D + hh + thr0, 0.0)
    Gb = np.maximum(vb * (1 + 2.0 ** -16) - D + hh + thr0, 0.0)
    cert = vs > vb * (1 + 2.0 ** -16) + thr0 + 2 * dn * (np.sqrt(Gs) + np.sqrt(Gb))
    T = cc[None, :] - 2.0 * xh @ ch.T  # decision values of xhat
    Tb = T[rows, b]
    T_other = T.copy()
    T_other[rows, b] = np.inf
    margin = T_other.min(axis=1) - Tb
    return cert, margin


def _near_ties(rng, n, d, k, scale):
    ch = rng.uniform(-scale, scale, (k, d))
    a = rng.integers(0, k, n)
    b = (a + 1 + rng.integers(0, k - 1, n)) % k
    eps = rng.choice([0.0, 2.0 ** -14, -2.0 ** -14, 2.0 ** -11, -2.0 ** -11, 2.0 ** -8, 0.05], n)
    xh = 0.5 * (ch[a] + ch[b]) + eps[:, None] * (ch[b] - ch[a])
    xh += rng.normal(0.0, scale * 2.0 ** -12, xh.shape)  # off the exact bisector
    return xh, ch


def test_certified_points_keep_the_exact_argmin():
    rng = np.random.default_rng(7)
    for d, k, scale in [(16, 64, 256.0), (11, 64, 300.0), (16, 17, 40.0), (9, 5, 1000.0)]:
        xh, ch = _near_ties(rng, 40000, d, k, scale)
        D = float((xh ** 2).sum(axis=1).max()) * 1.01 + 1.0
        thr0 = D * 2.0 ** -40
        cert, margin = _certify(xh, ch, D, thr0)
        assert np.all(margin[cert] > 0), (d, k, float(margin[cert].min()))
        # not vacuous: the clear points (eps = 0.05 and random data) certify
        assert cert.mean() > 0.1, (d, k, cert.mean())


def test_random_points_mostly_certify():
    rng = np.random.default_rng(3)
    d, k = 16, 64
    ch = rng.uniform(-300, 300, (k, d))
    xh = ch[rng.integers(0, k, 50000)] + rng.normal(0, 40, (50000, d))
    D = float((xh ** 2).sum(axis=1).max()) * 1.01 + 1.0
    cert, margin = _certify(xh, ch, D, D * 2.0 ** -40)
    assert np.all(margin[cert] > 0)
    assert cert.mean() > 0.97, cert.mean()
