"""Points sharded over ranks: one process per GPU, torch.distributed over RCCL.

The reference k-means is single-process (src/kmeans_plusplus.py); this module
runs the same algorithm on a row-sharded data set with results identical to
the single-process run:

* Sharding — contiguous row ranges in multiples of 8192 rows (NumPy's
  reduction chunk), so every rank's seeding blocks are global blocks and the
  blocked pairwise ``dist_sq.sum()`` is unchanged; only the last rank may own
  a partial block.
* Seeding (kmeans_plusplus.py:13-20) per step: all-gather of the per-block
  pairwise sums (every rank then adds them left to right — the exact global
  total), a rank-ordered chain of exact ``cumsum`` scans (each rank starts
  from its predecessor's running value), an all-gather of the local
  ``searchsorted`` hits and a broadcast of the chosen row by its owner.
* Lloyd (:33-48) per step: the fused device step writes k x (d+1) int64
  fixed-point sums/counts; one SUM all-reduce (integer, hence exact and
  order-free) over RCCL; every rank then forms the identical means.  With
  the device-resident loop (``device_lloyd``, csrc/loop.hip) the means, the
  shift and the convergence test run on the device after the all-reduce, and
  with a libcdr communicator (``Comm.attach_native``, csrc/comm.hip) a chunk
  of steps — assign, ncclAllReduce, finalize each — is enqueued by one C
  call; the host only polls every few steps and takes over exactly when the
  reference's host logic is needed (empty cluster: np.random.randint on every
  rank in j order, the row broadcast by its owner; a shift too close to tol:
  np.linalg.norm).  ``unify_points`` gives every shard the same storage mode,
  scale and screen transform, so these decisions agree on every rank.

``Comm`` hides the backend: NCCL (=RCCL on ROCm) keeps the all-reduced
tensor on the GPU; gloo (the CPU test backend) uses host tensors.
"""
from __future__ import annotations

import numpy as np

SEED_BLOCK = 8192


def shard_rows(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """(row_begin, n_local) of `rank`: whole 8192-row blocks, remainder last."""
    nb = -(-n_total // SEED_BLOCK) if n_total > 0 else 0
    base, extra = divmod(nb, world)
    b0 = rank * base + min(rank, extra)
    nbr = base + (1 if rank < extra else 0)
    begin = min(b0 * SEED_BLOCK, n_total)
    end = min((b0 + nbr) * SEED_BLOCK, n_total)
    return begin, end - begin


def bind_stream(ctx, device):
    """Put ctx and torch on ONE HIP stream, so Comm.fenced needs no host
    synchronisation around the collectives on the context's buffers.  The
    legacy default stream's handle is 0, which cdr_set_stream reads as "the
    context's own stream" (every fenced collective then paid two
    host syncs); in that case a torch stream is created and made current."""
    import torch

    cur = torch.cuda.current_stream(device)
    if not cur.cuda_stream:
        cur = torch.cuda.Stream(device)
        torch.cuda.set_stream(cur)
    ctx.set_stream(cur.cuda_stream)
    return cur


class Comm:
    """Thin collective layer over torch.distributed (or a single process)."""

    def __init__(self, dist=None, device=None):
        self.dist = dist
        self.rank = dist.get_rank() if dist else 0
        self.world = dist.get_world_size() if dist else 1
        self.device = device  # torch.device for NCCL, None for gloo / single
        self.seed_bad = 0  # this rank's seeding consistency flag (seed_sharded)

    def attach_native(self, ctx) -> bool:
        """Give ``ctx`` its own RCCL communicator over the same ranks
        (csrc/comm.hip), so that the device loop issues each step's
        all-reduce from C (cdr_lloyd_enqueue_steps).  Only under NCCL (RCCL)
        with device tensors; collective: every rank calls it."""
        if self.device is None or not self.dist or not hasattr(ctx, "comm_init"):
            return False
        import torch

        import _cdr

        # every rank checks that librccl loads (dlopen / dlsym only) and the
        # ranks agree (MIN) before any of them enters the collective init: one
        # rank that cannot load it must not leave the others waiting in
        # ncclCommInitRank.  Only rank 0 creates the unique id (each
        # ncclGetUniqueId starts a bootstrap listener).
        try:
            ok = 1 if _cdr.comm_available() else 0
        except Exception:  # noqa: BLE001 - any failure means "no native comm"
            ok = 0
        uid = np.zeros(128, dtype=np.uint8)
        if ok and self.rank == 0:
            try:
                uid = np.frombuffer(_cdr.comm_unique_id(), dtype=np.uint8).copy()
            except Exception:  # noqa: BLE001
                ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device=self.device)
        self.dist.all_reduce(flag, op=self.dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            return False
        t = torch.from_numpy(uid).to(self.device)
        self.dist.broadcast(t, 0)
        ctx.comm_init(t.cpu().numpy().tobytes(), self.world, self.rank)
        return True

    def has_native(self, ctx) -> bool:
        """ctx holds a libcdr communicator over exactly these ranks (asked of
        the C side: a Python-side record by id() could outlive the context)."""
        return hasattr(ctx, "comm_ranks") and ctx.comm_ranks()[0] == self.world

    def fenced(self, ctx, fn, *args):
        """Run the collective fn(*args) on device buffers that ctx's kernels
        write before it and read after it.  torch.distributed runs it on
        torch's current stream; when ctx enqueues on another stream (its own,
        unless ctx.set_stream(torch's current stream) was called), wait for
        ctx's queued kernels before the collective and for the collective
        before ctx's next kernels (otherwise the two streams race
        and the results are silently wrong).  Host buffers (gloo) need none."""
        if self.device is None or not self.dist:
            return fn(*args)
        import torch

        cur = torch.cuda.current_stream(self.device)
        sh = getattr(ctx, "stream_handle", None)
        same = sh is not None and sh() == cur.cuda_stream
        if not same:
            ctx.synchronize()
        r = fn(*args)
        if not same:
            cur.synchronize()
        return r

    def _t(self, arr):
        import torch

        t = torch.from_numpy(np.ascontiguousarray(arr))
        return t.to(self.device) if self.device is not None else t

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def allreduce_sum_i64(self, arr: np.ndarray) -> np.ndarray:
        if not self.dist:
            return arr
        t = self._t(arr.astype(np.int64))
        self.dist.all_reduce(t)
        return t.cpu().numpy()

    def allgather(self, arr: np.ndarray) -> list[np.ndarray]:
        """Variable-length 1-D all-gather (rank order)."""
        if not self.dist:
            return [arr]
        import torch

        n = self._t(np.array([arr.size], dtype=np.int64))
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(sizes, n)
        sizes = [int(s.item()) for s in sizes]
        m = max(sizes) if sizes else 0
        buf = np.zeros(max(m, 1), dtype=arr.dtype)
        buf[: arr.size] = arr
        t = self._t(buf)
        outs = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(outs, t)
        return [o.cpu().numpy()[:s] for o, s in zip(outs, sizes)]

    def allreduce_sum_f64(self, v: float) -> float:
        if not self.dist:
            return v
        t = self._t(np.array([v], dtype=np.float64))
        self.dist.all_reduce(t)
        return float(t.cpu().numpy()[0])

    def allreduce_i64(self, arr: np.ndarray, op: str = "sum") -> np.ndarray:
        """Element-wise SUM / MIN / MAX of an int64 vector over the ranks."""
        if not self.dist:
            return np.asarray(arr, dtype=np.int64)
        t = self._t(np.asarray(arr, dtype=np.int64))
        red = {"sum": self.dist.ReduceOp.SUM, "min": self.dist.ReduceOp.MIN,
               "max": self.dist.ReduceOp.MAX}[op]
        self.dist.all_reduce(t, op=red)
        return t.cpu().numpy()

    def allreduce_f64(self, arr: np.ndarray, op: str = "sum") -> np.ndarray:
        if not self.dist:
            return np.asarray(arr, dtype=np.float64)
        t = self._t(np.asarray(arr, dtype=np.float64))
        red = {"sum": self.dist.ReduceOp.SUM, "min": self.dist.ReduceOp.MIN,
               "max": self.dist.ReduceOp.MAX}[op]
        self.dist.all_reduce(t, op=red)
        return t.cpu().numpy()

    def exchange_buffer(self, nbytes: int):
        """(buffer, pointer-or-array) for the feature exchange: a device
        uint8 tensor under NCCL (RCCL all-to-all), a host array otherwise."""
        nbytes = max(int(nbytes), 1)
        if self.device is not None and self.dist:
            import torch

            t = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            return t, t.data_ptr()
        a = np.zeros(nbytes, dtype=np.uint8)
        return a, a

    def all_to_all_bytes(self, send, send_bytes: np.ndarray):
        """Variable all-to-all: send_bytes[r] bytes of `send` (the regions in
        rank order) go to rank r.  Returns (recv buffer, pointer-or-array,
        received bytes per source rank)."""
        send_bytes = np.asarray(send_bytes, dtype=np.int64)
        if not self.dist:
            return send, send, send_bytes
        import torch

        sb = self._t(send_bytes)
        rb = torch.empty_like(sb)
        self.dist.all_to_all_single(rb, sb)
        recv_bytes = rb.cpu().numpy()
        recv, handle = self.exchange_buffer(int(recv_bytes.sum()))
        if self.device is not None:
            sendt = send
            recvt = recv
        else:
            sendt = torch.from_numpy(send)
            recvt = torch.from_numpy(recv)
        total_send = int(send_bytes.sum())
        self.dist.all_to_all_single(recvt[: int(recv_bytes.sum())], sendt[:total_send],
                                    output_split_sizes=[int(x) for x in recv_bytes],
                                    input_split_sizes=[int(x) for x in send_bytes])
        return recv, handle, recv_bytes

    def lloyd_buffer(self, n: int):
        """(buffer, pointer) of the per-step (k, d+1) int64 all-reduce: a
        device tensor under NCCL (RCCL), a host array otherwise."""
        if self.device is not None and self.dist:
            import torch

            t = torch.empty(n, dtype=torch.int64, device=self.device)
            return t, t.data_ptr()
        a = np.zeros(n, dtype=np.int64)
        return a, a

    def allreduce_inplace(self, buf) -> None:
        if not self.dist:
            return
        if self.device is not None:
            self.dist.all_reduce(buf)
        else:
            import torch

            t = torch.from_numpy(buf)
            self.dist.all_reduce(t)

    def buffer(self, nbytes: int):
        """(buffer, handle) of `nbytes` for a device protocol's exchanges: a
        device uint8 tensor and its pointer under NCCL (RCCL), a host uint8
        array (the handle itself) otherwise."""
        return self.exchange_buffer(nbytes)

    def allgather_slots(self, buf, m: int) -> None:
        """In-place all-gather of m-byte slots: rank r's slot is bytes
        [r m, (r + 1) m) of buf; afterwards every rank holds every slot."""
        if not self.dist:
            return
        import torch

        t = buf if self.device is not None else torch.from_numpy(buf)
        src = t[self.rank * m:(self.rank + 1) * m].clone()
        self.dist.all_gather([t[r * m:(r + 1) * m] for r in range(self.world)], src)

    def allreduce_sum_f64_inplace(self, buf) -> None:
        """SUM all-reduce of a byte buffer holding float64 values, in place."""
        if not self.dist:
            return
        import torch

        t = buf if self.device is not None else torch.from_numpy(buf)
        self.dist.all_reduce(t.view(torch.float64))

    def bcast_buffer(self, buf, src: int) -> None:
        """In-place broadcast of a byte buffer (device tensor or host array)
        from rank src."""
        if not self.dist:
            return
        import torch

        t = buf if self.device is not None else torch.from_numpy(buf)
        self.dist.broadcast(t, src)

    def bcast(self, arr: np.ndarray, src: int) -> np.ndarray:
        if not self.dist:
            return arr
        t = self._t(np.ascontiguousarray(arr))
        self.dist.broadcast(t, src)
        return t.cpu().numpy()


_SIGN = np.uint64(1 << 63)


def unify_points(ctx, comm: Comm | None, n_total: int) -> None:
    """One storage mode, fixed-point scale and screen transform for every
    shard (include/cdr.h cdr_points_restat): the int64 sums of the all-reduce
    must share one scale, and the device loop's stop decisions (the fp16
    screen-range guard) must be the same on every rank.  Statistics are
    combined with MIN (per-feature minima) and MAX (everything else) over the
    ranks; collective: every rank calls it after loading its shard."""
    st = ctx.points_stats()
    if comm is not None and comm.world > 1:
        d = (st.size - 3) // 2
        s = (st ^ _SIGN).view(np.int64)  # unsigned order -> signed order
        lo = comm.allreduce_i64(s[:d], "min")
        hi = comm.allreduce_i64(s[d:], "max")
        st = np.concatenate([lo, hi]).view(np.uint64) ^ _SIGN
    ctx.points_restat(st, n_total)


def ensure_unified(ctx, comm: Comm | None, n_total: int) -> None:
    """Collective guard of the sharded paths: if any rank's
    context was not unified over n_total rows (``Context.restat_n``), every
    rank runs unify_points; then the ranks check that they agree on the
    storage mode and the fixed-point scale, and raise together if not."""
    if comm is None or comm.world == 1 or not hasattr(ctx, "points_restat"):
        return
    need = int(getattr(ctx, "restat_n", None) != n_total)
    if int(comm.allreduce_i64(np.array([need]), "max")[0]):
        unify_points(ctx, comm, n_total)
    inf = ctx.info()
    v = np.array([inf["mode"], inf["scale_bits"], inf["d"]], dtype=np.int64)
    if not np.array_equal(comm.allreduce_i64(v, "min"), comm.allreduce_i64(v, "max")):
        raise RuntimeError("sharded points disagree on storage mode / scale after unify_points")


def _fetch_row(ctx, comm: Comm, owner: int, local_idx: int, d: int) -> np.ndarray:
    row = ctx.get_rows([local_idx])[0] if comm.rank == owner else np.zeros(d)
    return comm.bcast(np.asarray(row, dtype=np.float64), owner)


def row_fetcher(ctx, comm: Comm, row_begin: int, d: int):
    """gidx -> X[gidx] over the shards (collective: every rank calls it)."""
    offs = np.concatenate(comm.allgather(np.array([row_begin], dtype=np.int64)))

    def row(gidx: int) -> np.ndarray:
        owner = _owner_of(offs, gidx)
        return _fetch_row(ctx, comm, owner, gidx - int(offs[owner]), d)

    return row


def _is_device_context(ctx) -> bool:
    """ctx is libcdr's GPU context (not a host-side model of one)."""
    return type(ctx).__module__ == "_cdr" and type(ctx).__name__ == "Context"


def _owner_of(offsets: np.ndarray, gidx: int) -> int:
    return int(np.searchsorted(offsets, gidx, side="right") - 1)


SEED_PROGRAM_CAP = 4096  # items per rank in the all-gathered cumsum programs


def _program_record(prog) -> np.ndarray:
    """A rank's program padded to SEED_PROGRAM_CAP items, as int64 words for
    the all-gather: item 0 holds the count in d0 (-1: no usable program)."""
    from _cdr import SEED_ITEM

    rec = np.zeros(SEED_PROGRAM_CAP + 1, dtype=SEED_ITEM)
    if prog is None or prog.size > SEED_PROGRAM_CAP:
        rec[0]["d0"] = -1
    else:
        rec[0]["d0"] = prog.size
        rec[1:1 + prog.size] = prog
    return rec.view(np.int64)


def shard_scan(ctx, comm: Comm, parts, total: float):
    """np.cumsum(dist_sq / total) over the sharded rows (kmeans_plusplus.py:19):
    returns the running value after the last shard (c_last); afterwards every
    rank's ctx can answer seed_search.

    Every rank builds its shard's cumsum program in parallel from a guess of
    the running value at its first row (the earlier shards' block sums /
    total; include/cdr.h cdr_seed_scan_begin).  The first rank's start is
    exactly 0, so it scans outright and publishes a constant.  The programs
    are all-gathered and every rank composes them in rank order on the host
    (cdr_seed_program_eval), which gives each rank its exact start; a guess
    that does not hold for the exact start is detected there, and then the
    rank-ordered chain of exact scans runs instead (same result)."""
    world, rank = comm.world, comm.rank
    if world == 1:
        return ctx.seed_scan(total, 0.0)
    if hasattr(ctx, "seed_scan_begin"):
        from _cdr import SEED_CONST, SEED_ITEM, seed_program_eval

        if rank == 0:
            prog = np.zeros(1, dtype=SEED_ITEM)
            prog[0]["kind"] = SEED_CONST
            prog[0]["p"] = ctx.seed_scan(total, 0.0)
        else:
            before = sum(int(p.size) for p in parts[:rank])
            guess = float(np.sum(np.concatenate(parts)[:before])) / total
            ni, nf = ctx.seed_scan_begin(total, guess)
            prog = ctx.seed_scan_items(ni) if 0 <= ni <= SEED_PROGRAM_CAP and nf == 0 else None
        recs = comm.allgather(_program_record(prog))
        c, c_mine, ok = 0.0, 0.0, True
        for r, words in enumerate(recs):
            rec = np.ascontiguousarray(words, dtype=np.int64).view(SEED_ITEM)
            cnt = int(rec[0]["d0"])
            if cnt < 0:
                ok = False
                break
            if r == rank:
                c_mine = c
            c, good = seed_program_eval(rec[1:1 + cnt], c)
            if not good:
                ok = False
                break
        if ok:
            if rank > 0:
                mine = ctx.seed_scan_end(c_mine)
                # checked by every rank together with the draw's hits (a raise
                # on one rank alone would leave the others in a collective)
                comm.seed_bad = int(mine != seed_program_eval(prog, c_mine)[0])
            return c
    c = 0.0
    for r in range(world):  # rank-ordered chain of exact scans
        mine = ctx.seed_scan(total, c) if rank == r else 0.0
        c = float(comm.bcast(np.array([mine], dtype=np.float64), r)[0])
    return c


def device_seed_layout_ok(offsets, n_total: int, world: int) -> bool:
    """Whether the ranks' row layout fits the device-resident protocol
    (csrc/seed.hip seed_shard_begin): shards in rank order from row 0, every
    start on an 8192-row block, and no shard over ceil(blocks / world) blocks
    (the [nranks][nbmax] block-sum slots).  Decided from the all-gathered
    offsets, so every rank takes the same branch: a layout the device
    protocol cannot hold runs the host protocol on all ranks instead of
    raising on some of them while the others wait in a collective."""
    off = [int(o) for o in np.asarray(offsets, dtype=np.int64).ravel()]
    if len(off) != world or off[0] != 0:
        return False
    ends = off[1:] + [int(n_total)]
    nbmax = -(-(-(-int(n_total) // 8192)) // world)
    for b, e in zip(off, ends):
        if e < b or (b % 8192 != 0 and e > b) or -(-(e - b) // 8192) > nbmax:
            return False
    return True


def seed_sharded(ctx, comm: Comm, row_begin: int, n_total: int, k: int, random_state=None,
                 host_seq_sum=None) -> np.ndarray:
    """kmeans_plusplus_init over the sharded rows (float64 centroids)."""
    if host_seq_sum is None:
        from _cdr import host_seq_sum
    ensure_unified(ctx, comm, n_total)
    offsets = np.array([b for b in comm.allgather(np.array([row_begin], dtype=np.int64))],
                       dtype=np.int64).ravel()
    rng = np.random.default_rng(random_state)
    first = int(rng.integers(0, n_total))
    # rng.choice draws one uniform per step (:19): all k - 1 taken up front
    u = rng.random(k - 1) if k > 1 else np.zeros(0)
    if comm.world == 1 and k > 1 and hasattr(ctx, "seed_run"):
        # one shard: every step on the device (cdr_seed_run)
        picks = ctx.seed_run(first, k, u)
        return np.asarray(ctx.get_rows(picks), dtype=np.float64)
    if comm.world > 1 and k > 1 and hasattr(ctx, "seed_shard_begin") and \
            device_seed_layout_ok(offsets, n_total, comm.world):
        # sharded and device-resident: three collectives per step, no host
        # round trip (include/cdr.h cdr_seed_shard_*); status 1 (a program
        # that cannot be composed, seen by every rank) -> the host protocol
        _, cents, status = seed_device_sharded(ctx, comm, row_begin, n_total, first, k, u)
        if status == 2:
            raise ValueError("Probabilities contain NaN")
        if status == 0:
            return cents
        comm.seed_fallbacks = getattr(comm, "seed_fallbacks", 0) + 1
    return seed_host_protocol(ctx, comm, offsets, n_total, first, k, u, host_seq_sum)


def seed_host_protocol(ctx, comm: Comm, offsets, n_total: int, first: int, k: int, u,
                       host_seq_sum) -> np.ndarray:
    """The sharded seeding steps (:13-20) with the host in every step: the
    block sums all-gathered and added left to right, the cumsum programs
    composed on every rank (shard_scan), the hits all-gathered, the picked row
    broadcast by its owner.  Runs when the device protocol cannot (its layout,
    or status 1 seen by every rank); collective."""
    d = ctx.info()["d"]
    C = np.empty((k, d), dtype=np.float64)
    owner = _owner_of(offsets, first)
    C[0] = _fetch_row(ctx, comm, owner, first - int(offsets[owner]), d)
    if k > 1:
        ctx.seed_reset()
    for i in range(1, k):
        ctx.seed_update(C[i - 1])
        parts = comm.allgather(ctx.seed_block_sums())
        total = host_seq_sum(np.concatenate(parts))
        if not (total > 0.0) or total == np.inf:
            raise ValueError("Probabilities contain NaN")
        comm.seed_bad = 0
        c = shard_scan(ctx, comm, parts, total)
        got = np.stack(comm.allgather(np.array([ctx.seed_search(c, u[i - 1]), comm.seed_bad],
                                               dtype=np.int64)))
        if got[:, 1].any():
            raise RuntimeError("a shard's cumsum program and its exact scan disagree")
        hits = got[:, 0]
        owner = int(np.flatnonzero(hits >= 0)[0])
        C[i] = _fetch_row(ctx, comm, owner, int(hits[owner]), d)
    return C


def seed_device_sharded(ctx, comm: Comm, row_begin: int, n_total: int, first: int, k: int, u):
    """kmeans_plusplus_init's steps (:13-20) on sharded rows with every step on
    the devices: with a libcdr communicator the whole run is enqueued by one C
    call (cdr_seed_run_sharded: ncclAllGather / ncclAllReduce between the
    kernels); otherwise the same phases are driven from here with the
    collectives of ``comm`` on device (RCCL) or host (gloo) buffers.  Returns
    (picks, centres (k, d), status) — status 0 ok, 1 run the host protocol,
    2 "Probabilities contain NaN"."""
    if comm.has_native(ctx) and hasattr(ctx, "seed_run_sharded"):
        return ctx.seed_run_sharded(row_begin, n_total, first, k, u)
    d = ctx.info()["d"]
    red_b = 8 * (d + 4)
    red, hred = comm.buffer(red_b)
    sizes = ctx.seed_shard_begin(row_begin, n_total, comm.world, comm.rank, first, k, u, hred)
    comm.fenced(ctx, comm.allreduce_sum_f64_inplace, red)
    bs, hbs = comm.buffer(comm.world * int(sizes[0]))
    pg, hpg = comm.buffer(comm.world * int(sizes[1]))
    for _ in range(1, k):
        ctx.seed_shard_phase(0, hred, hbs)
        comm.fenced(ctx, comm.allgather_slots, bs, int(sizes[0]))
        ctx.seed_shard_phase(1, hbs, hpg)
        comm.fenced(ctx, comm.allgather_slots, pg, int(sizes[1]))
        ctx.seed_shard_phase(2, hpg, hred)
        comm.fenced(ctx, comm.allreduce_sum_f64_inplace, red)
    return ctx.seed_shard_end(hred)


LL_CHUNK_MAX = 64  # steps enqueued between two status polls (doubling from 2)


class DeviceLloyd:
    """Lloyd iterations (src/kmeans_plusplus.py:31-48) on the device-resident
    loop of one context (csrc/loop.hip), optionally sharded over ``comm``.

    ``reseed_row(gidx)`` returns X[gidx] for the reference's empty-cluster
    reseed (:43); under ``comm`` every rank calls it (the owner broadcasts)."""

    def __init__(self, ctx, C, tol: float, reseed_row, n_total: int, comm: Comm | None = None,
                 dtype=np.float64):
        self.ctx, self.tol, self.reseed_row, self.n_total = ctx, tol, reseed_row, n_total
        self.comm, self.dtype = comm, np.dtype(dtype)
        ensure_unified(ctx, comm, n_total)
        self.k, self.d = C.shape
        ref = np.array(C[0], dtype=np.float64)  # a data row: x - ref is exact
        x2 = ctx.points_sqdev(ref)
        if comm is not None:
            x2 = comm.allreduce_sum_f64(x2)
        ctx.lloyd_begin(C, tol, ref, x2, round32=self.dtype == np.float32)
        self.buf, self.ptr = None, None
        # steps enqueued from C (one call per chunk): a single shard, or a
        # context with its own RCCL communicator (Comm.attach_native)
        self.native = hasattr(ctx, "lloyd_enqueue_steps") and (
            comm is None or comm.world == 1 or comm.has_native(ctx))
        if not self.native and comm is not None and comm.world > 1:
            self.buf, self.ptr = comm.lloyd_buffer(self.k * (self.d + 1))
        self.steps = 0
        self.converged = False
        self.status = None

    def enqueue(self, m: int) -> None:
        if self.native:
            self.ctx.lloyd_enqueue_steps(m)
            return
        for _ in range(m):
            self.ctx.lloyd_enqueue_assign(self.ptr)
            if self.buf is not None:
                self.comm.fenced(self.ctx, self.comm.allreduce_inplace, self.buf)
            self.ctx.lloyd_enqueue_finalize(self.ptr)

    def advance(self, max_steps: int, chunk: int = 2, chunk_max: int = LL_CHUNK_MAX) -> int:
        """Run up to max_steps more steps (fewer on convergence); returns the
        number of steps the reference would have taken."""
        start = self.steps
        target = start + max_steps
        while self.steps < target and not self.converged:
            self.enqueue(min(chunk, target - self.steps))
            chunk = min(2 * chunk, chunk_max)
            st = self.status = self.ctx.lloyd_status()
            self.steps = st["steps"]
            if st["running"]:
                continue
            if st["reason"] == self.ctx.LL_CONVERGED:
                self.converged = True
                break
            if st["reason"] == self.ctx.LL_HOST_PLAN:
                self.ctx.lloyd_resume(host_plan_once=True)
                continue
            # empty cluster or a shift too close to tol: the reference's host
            # logic for this one step (kmeans_plusplus.py:37-48)
            C_cur, means, counts = self.ctx.lloyd_read()
            new = np.empty((self.k, self.d), dtype=self.dtype)
            new[...] = means
            for j in np.flatnonzero(counts == 0):  # j order, as the reference draws
                new[j] = self.reseed_row(np.random.randint(0, self.n_total))
            shift = np.linalg.norm(new - C_cur.astype(self.dtype))
            self.ctx.lloyd_resume(new, add_steps=1)
            self.steps += 1
            if shift < self.tol:
                self.converged = True
        return self.steps - start

    def finish(self):
        """(centroids as dtype, status of the last step); ends the loop."""
        try:
            C = self.ctx.lloyd_read()[0].astype(self.dtype)
            st = self.ctx.lloyd_status()
        finally:
            self.ctx.lloyd_end()
        return C, st


def device_lloyd(ctx, C, max_iter: int, tol: float, reseed_row, n_total: int,
                 comm: Comm | None = None, dtype=np.float64):
    """max_iter Lloyd steps (fewer on convergence) on the device loop:
    (centroids as ``dtype``, status dict of the last step: steps, shift,
    inertia)."""
    run = DeviceLloyd(ctx, C, tol, reseed_row, n_total, comm, dtype)
    try:
        run.advance(max_iter)
    except BaseException:
        ctx.lloyd_end()
        raise
    return run.finish()


def f64_sharded_sums(ctx, comm: Comm, C: np.ndarray):
    """The exact sequential cluster sums of an F64 Lloyd step over rows sharded
    in rank order (src/kmeans_plusplus.py:33-41: labels from C, then
    X[labels == j] summed row after row, as NumPy's mean does), every rank
    getting (sums (k, d), counts (k,)).  Two all-gathers per step: the
    shards' approximate totals, then their programs (include/cdr.h
    cdr_f64s_*), composed in rank order on every rank; when a program's
    guess does not hold (every rank sees it), the exact rank chain: each
    shard walks from the exact entry in turn, broadcasting its exit."""
    k, d = C.shape
    kd = k * d
    tot, htot = comm.buffer(comm.world * 8 * (kd + k))
    sizes = ctx.f64s_begin(C, comm.world, comm.rank, htot)
    comm.fenced(ctx, comm.allgather_slots, tot, int(sizes[0]))
    prog, hprog = comm.buffer(comm.world * int(sizes[1]))
    ctx.f64s_build(htot, hprog)
    comm.fenced(ctx, comm.allgather_slots, prog, int(sizes[1]))
    sums, counts, status = ctx.f64s_finish(htot, hprog)
    if status:
        comm.f64_chains = getattr(comm, "f64_chains", 0) + 1
        chain, hchain = comm.buffer(16 * kd)
        if comm.device is not None:
            import torch

            chain.zero_()
            # the zeroing runs on torch's current stream; rank 0's f64s_chain
            # reads chain[0, 2kd) as its exact entry on the context's stream
            # (without this fence it could walk from the
            # uninitialised buffer)
            if getattr(ctx, "stream_handle", lambda: None)() != \
                    torch.cuda.current_stream(comm.device).cuda_stream:
                torch.cuda.current_stream(comm.device).synchronize()
        else:
            chain[:] = 0
        for r in range(comm.world):
            if comm.rank == r:
                ctx.f64s_chain(hchain)
            comm.fenced(ctx, comm.bcast_buffer, chain, r)
        if comm.device is not None:
            import torch

            sums = chain.view(torch.float64)[:kd].cpu().numpy().reshape(k, d)
        else:
            sums = chain.view(np.float64)[:kd].copy().reshape(k, d)
    return sums, counts


class ShardedLloyd:
    """Lloyd iterations over sharded points: F32X (grid) points with one
    int64 all-reduce per step (or the device-resident loop); F64 points with
    the exact sharded sequential sums (f64_sharded_sums) and the host
    forming the means, as src/kmeans_plusplus.py:37-48 does."""

    def __init__(self, ctx, comm: Comm, n_total: int, row_begin: int):
        ensure_unified(ctx, comm, n_total)
        info = ctx.info()
        if info["mode"] not in (1, 2):
            raise NotImplementedError("sharded Lloyd needs loaded points")
        self.ctx, self.comm = ctx, comm
        self.n_total, self.row_begin = n_total, row_begin
        self.d, self.S = info["d"], info["scale_bits"]
        self.f64 = info["mode"] == 2
        self._dev_buf = None
        if self.f64 and comm.dist and comm.device is None and _is_device_context(ctx):
            # the F64 programs are all-gathered in device buffers that the
            # context's kernels read and write; gloo hands host arrays
            # (this used to fail with an obscure ctypes TypeError)
            raise NotImplementedError(
                "sharded F64 Lloyd on a GPU context needs a device communicator "
                "(torch.distributed with the nccl backend); gloo is not supported")

    def partials(self, C: np.ndarray) -> np.ndarray:
        k = C.shape[0]
        if self.comm.device is not None and self.comm.dist:
            import torch

            if self._dev_buf is None or self._dev_buf.numel() != k * (self.d + 1):
                self._dev_buf = torch.empty(k * (self.d + 1), dtype=torch.int64,
                                            device=self.comm.device)
            self.ctx.lloyd_step_device(C, self._dev_buf.data_ptr())
            self.comm.dist.all_reduce(self._dev_buf)
            return self._dev_buf.view(k, self.d + 1).cpu().numpy()
        return self.comm.allreduce_sum_i64(self.ctx.lloyd_step(C))

    def step(self, C: np.ndarray, reseed_row) -> tuple[np.ndarray, float]:
        """One iteration; returns (new centroids, shift)."""
        k, d = C.shape
        if self.f64:
            sums, counts = f64_sharded_sums(self.ctx, self.comm, np.asarray(C, dtype=np.float64))
        else:
            acc = self.partials(C)
            counts = acc[:, d]
            sums = np.ldexp(acc[:, :d].astype(np.float64), -self.S)
        with np.errstate(invalid="ignore", divide="ignore"):
            new = sums / counts[:, None].astype(np.float64)
        for j in np.flatnonzero(counts == 0):  # j order, as the reference draws
            new[j] = reseed_row(np.random.randint(0, self.n_total))
        shift = np.linalg.norm(new - C)
        return new, shift

    def row(self, gidx: int) -> np.ndarray:
        offs = np.concatenate(self.comm.allgather(np.array([self.row_begin], dtype=np.int64)))
        owner = _owner_of(offs, gidx)
        return _fetch_row(self.ctx, self.comm, owner, gidx - int(offs[owner]), self.d)

    def run(self, C: np.ndarray, max_iter: int, tol: float = 1e-4):
        """max_iter Lloyd steps (fewer on convergence): the device loop for
        F32X points, the host-driven sharded F64 steps otherwise."""
        if self.f64:
            return self.run_host(C, max_iter, tol)
        C, self.last_status = device_lloyd(self.ctx, C, max_iter, tol, self.row, self.n_total,
                                           self.comm)
        return C

    def run_host(self, C: np.ndarray, max_iter: int, tol: float = 1e-4):
        """The same iterations with the host forming the means every step."""
        for _ in range(max_iter):
            C, shift = self.step(C, self.row)
            if shift < tol:
                break
        return C


def sharded_medians(ctx, comm: Comm, k: int) -> np.ndarray:
    """Per-cluster, per-feature medians (src/scoring.py:50-54, np.median of
    each cluster's column) of points sharded over the ranks, from the labels
    of the last Lloyd step: one SUM all-reduce of the cluster sizes, then per
    radix pass one SUM all-reduce of the k x d x 2 x 256 digit histograms
    (RCCL on the device buffer under NCCL).  Every rank returns the same
    (k, d) array, equal to the single-process medians."""
    if comm.world == 1:
        return ctx.medians_by_label(k)  # the same passes, histograms never leave the device
    local = ctx.medians_group(k)
    counts = comm.allreduce_i64(local, "sum")
    passes, words = ctx.medians_begin(counts)
    if comm.device is not None and comm.dist:
        import torch

        buf = torch.empty(words, dtype=torch.int32, device=comm.device)
        handle = buf.data_ptr()
    else:
        buf = np.zeros(words, dtype=np.uint32)
        handle = buf
    for p in range(passes):
        ctx.medians_pass_hist(p, handle)
        if comm.dist:
            if comm.device is not None:
                comm.fenced(ctx, comm.dist.all_reduce, buf)
            else:
                import torch

                t = torch.from_numpy(buf.view(np.int32))
                comm.dist.all_reduce(t)
        ctx.medians_pass_select(p, handle)
    return ctx.medians_finish()

