"""Sharded medians (cdr_dist.sharded_medians) on CPU: gloo,
world sizes 1-3, each rank's device context replaced by a NumPy double of
the radix-select protocol (group -> global counts -> per pass: local digit
histograms, SUM all-reduce, digit selection), against np.median of every
cluster's column (src/scoring.py:50-54)."""
import os

import numpy as np
import pytest

from test_features_dist import _free_port


def _okey(v):
    b = np.asarray(v, dtype=np.float64).view(np.uint64)
    neg = (b >> np.uint64(63)) == 1
    return np.where(neg, ~b, b | np.uint64(1 << 63))


def _from_okey(k):
    k = np.uint64(k)
    b = (k & np.uint64(0x7FFFFFFFFFFFFFFF)) if (k >> np.uint64(63)) else ~k
    return float(np.array([b], dtype=np.uint64).view(np.float64)[0])


class NumpyMedians:
    """Test double with the _cdr.Context median-pass surface (fp64 keys)."""

    def __init__(self, X, labels):
        self.X, self.lab = X, labels

    def medians_group(self, k):
        self.k = k
        return np.bincount(self.lab, minlength=k).astype(np.int64)

    def medians_begin(self, counts):
        self.m = np.asarray(counts)
        d = self.X.shape[1]
        self.pref = np.zeros((self.k, d, 2), dtype=np.uint64)
        self.rank = np.stack([(self.m - 1) // 2, self.m // 2], axis=1)[:, None, :].repeat(d, 1)
        return 8, self.k * d * 512

    def medians_pass_hist(self, p, hist):
        sh = (7 - p) * 8
        mask = np.uint64(0) if sh + 8 >= 64 else np.uint64(((1 << 64) - 1) << (sh + 8) & ((1 << 64) - 1))
        h = np.zeros((self.k, self.X.shape[1], 2, 256), dtype=np.uint32)
        keys = _okey(self.X)
        dig = ((keys >> np.uint64(sh)) & np.uint64(0xFF)).astype(np.int64)
        for j in range(self.k):
            rows = self.lab == j
            for f in range(self.X.shape[1]):
                kk, dd = keys[rows, f], dig[rows, f]
                p0, p1 = self.pref[j, f]
                h[j, f, 0] = np.bincount(dd[(kk & mask) == p0], minlength=256)
                if p1 != p0:
                    h[j, f, 1] = np.bincount(dd[(kk & mask) == p1], minlength=256)
        hist[:] = h.reshape(-1)

    def medians_pass_select(self, p, hist):
        sh = (7 - p) * 8
        h = hist.reshape(self.k, self.X.shape[1], 2, 256)
        for j in range(self.k):
            if self.m[j] <= 0:
                continue
            for f in range(self.X.shape[1]):
                p0, p1 = self.pref[j, f]
                two = p0 != p1
                for w in range(2):
                    c = np.cumsum(h[j, f, 1 if (w and two) else 0].astype(np.int64))
                    r = self.rank[j, f, w]
                    g = int(np.searchsorted(c, r, side="right"))
                    self.rank[j, f, w] = r - (c[g - 1] if g else 0)
                    self.pref[j, f, w] = (p0, p1)[w] | np.uint64(g << sh)

    def medians_by_label(self, k):
        passes, words = self.medians_begin(self.medians_group(k))
        h = np.zeros(words, dtype=np.uint32)
        for q in range(passes):
            self.medians_pass_hist(q, h)
            self.medians_pass_select(q, h)
        return self.medians_finish()

    def medians_finish(self):
        out = np.full((self.k, self.X.shape[1]), np.nan)
        for j in range(self.k):
            if self.m[j] <= 0:
                continue
            for f in range(self.X.shape[1]):
                a = _from_okey(self.pref[j, f, 0])
                out[j, f] = (0.0 + a) / 1.0 if self.m[j] & 1 else \
                    ((0.0 + a) + _from_okey(self.pref[j, f, 1])) / 2.0
        return out


def _data():
    rng = np.random.default_rng(3)
    X = rng.normal(0, 2, (3001, 3))
    X[::5, 1] = 0.25
    X[::9, 2] = -0.0
    lab = rng.integers(0, 6, X.shape[0])
    lab[lab == 4] = 5  # cluster 4 empty
    return X, lab


def _exp(X, lab, k):
    out = np.full((k, X.shape[1]), np.nan)
    for j in range(k):
        if (lab == j).any():
            out[j] = np.median(X[lab == j], axis=0)
    return out


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from cdr_dist import Comm, sharded_medians

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, lab = _data()
    lo, hi = (X.shape[0] * rank) // world, (X.shape[0] * (rank + 1)) // world
    med = sharded_medians(NumpyMedians(X[lo:hi], lab[lo:hi]), Comm(dist, None), 6)
    np.save(os.path.join(out_dir, f"m{rank}.npy"), med)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_medians_equal_numpy(tmp_path, world):
    X, lab = _data()
    exp = _exp(X, lab, 6)
    if world == 1:
        from cdr_dist import Comm, sharded_medians

        got = [sharded_medians(NumpyMedians(X, lab), Comm(None), 6)]
    else:
        mp = pytest.importorskip("torch.multiprocessing")
        mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
        got = [np.load(tmp_path / f"m{r}.npy") for r in range(world)]
    for g in got:
        np.testing.assert_array_equal(g, exp)
