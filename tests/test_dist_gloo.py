"""Multi-rank protocol of cdr_dist (sharded seeding + Lloyd) on CPU, gloo,
world_size 2.  Each rank's device shard is replaced by a test double built on
the pinned oracle, so this checks the collective logic — 8192-row sharding,
block-sum all-gather, the rank-ordered exact scan chain, the owner broadcast
and the int64 all-reduce — against the single-process reference semantics."""
import os
import socket

import numpy as np
import pytest

from oracle import kmeans_oracle as ko
from oracle import synth

N_TOTAL, D, K = 3 * 8192 + 1234, 4, 6


class OracleShard:
    """Test double with the _cdr.Context surface cdr_dist uses."""

    def __init__(self, X):
        self.X = X
        self.dmin = None
        self.cum = None
        self._labels = None

    def info(self):
        return {"n": self.X.shape[0], "d": self.X.shape[1], "mode": 1, "scale_bits": 24}

    def get_rows(self, idx):
        return self.X[np.atleast_1d(idx)]

    def seed_reset(self):
        self.dmin = np.full(self.X.shape[0], np.inf)

    def seed_update(self, c):
        self.dmin = np.minimum(self.dmin, np.sqrt(ko.sqdist_rows(self.X, c)) ** 2)

    def seed_block_sums(self):
        return np.array([ko.pairwise_sum_1d(self.dmin[s:s + 8192])
                         for s in range(0, self.dmin.size, 8192)])

    def seed_scan(self, total, c_in):
        self.cum = np.cumsum(np.concatenate([[c_in], self.dmin / total]))[1:]
        return float(self.cum[-1])

    def seed_search(self, c_last, u):
        i = int(np.searchsorted(self.cum / c_last, u, side="right"))
        return i if i < self.cum.size else -1

    def lloyd_step(self, C):
        self._labels, out = ko.lloyd_partials(self.X, C, 24)
        return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from cdr_dist import Comm, ShardedLloyd, seed_sharded, shard_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    begin, n_local = shard_rows(N_TOTAL, world, rank)
    shard = OracleShard(synth.generate(N_TOTAL, begin, n_local, D, K, 9))
    comm = Comm(dist, None)
    C = seed_sharded(shard, comm, begin, N_TOTAL, K, random_state=42)
    np.random.seed(0)
    C = ShardedLloyd(shard, comm, N_TOTAL, begin).run(C, max_iter=4, tol=-1.0)
    if rank == 0:
        np.save(os.path.join(out_dir, "C.npy"), C)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_rows_blocks():
    from cdr_dist import shard_rows

    for n in (1, 8191, 8192, 8193, 5 * 8192 + 7, 100_000_000):
        for w in (1, 2, 3, 8):
            parts = [shard_rows(n, w, r) for r in range(w)]
            assert sum(p[1] for p in parts) == n
            b = 0
            for r, (begin, m) in enumerate(parts):
                assert begin == b
                b += m
                assert begin % 8192 == 0 or m == 0
                assert m % 8192 == 0 or begin + m == n  # only the last block is partial


def test_two_ranks_match_single_process(tmp_path):
    mp = pytest.importorskip("torch.multiprocessing")
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    X = synth.generate(N_TOTAL, 0, N_TOTAL, D, K, 9)
    np.random.seed(0)
    C_ref, _ = ko.kmeans(X, K, random_state=42, max_iter=4, tol=-1.0)
    np.testing.assert_array_equal(np.load(tmp_path / "C.npy"), C_ref)
