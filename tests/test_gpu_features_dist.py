"""Sharded compute_features on the device (features_dist.py with the real
libcdr context: device ingest of each rank's log slice, the exchange pack /
unpack of csrc/exchange.hip, the hand-written group-by and the split
finalisation): world sizes 1 and 2 (two processes on the one GPU, gloo for
the collectives), bit-identical to the single-process oracle and to the
single-process device job."""
import os

import numpy as np
import pytest

from oracle import features_oracle as fo
from test_features_dist import _case, _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, man, log, out_dir):
    import torch.distributed as dist

    from _cdr import Context
    from cdr_dist import Comm
    from features_dist import sharded_compute_features

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = Context(0)
    paths, table = sharded_compute_features(man, log, ctx, Comm(dist, None))
    if rank == 0:
        np.save(os.path.join(out_dir, "table.npy"), table)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_device_sharded_features(tmp_path, world, ctx):
    import compute_features as cf

    man, log = _case(tmp_path)
    if world == 1:
        from cdr_dist import Comm
        from features_dist import sharded_compute_features

        paths, table = sharded_compute_features(man, log, ctx, Comm(None))
    else:
        mp = pytest.importorskip("torch.multiprocessing")
        mp.spawn(_worker, args=(world, _free_port(), man, log, str(tmp_path)), nprocs=world,
                 join=True)
        table = np.load(tmp_path / "table.npy")
    _, exp_table, _, _ = fo.compute(man, log)
    np.testing.assert_array_equal(table, exp_table)
    _, single = cf.compute_features(man, log, ctx=ctx)
    np.testing.assert_array_equal(table, single)


def test_device_exchange_roundtrip(ctx):
    """pack -> unpack of simulated events over 3 owners: every owner gets
    exactly its files' events (multiset), and the group-by of each owner's
    share equals the matching rows of the whole group-by."""
    nf = 30_000
    ctx.features_simulate(nf, 60.0, 3, seed=2)
    whole, mx = ctx.features_aggregate_resident()
    f, op, cl, ts, pr = ctx.features_events_read()
    bounds = np.array([0, 7_000, 7_000, nf], dtype=np.int64)  # an owner with no rows
    send, counts, pmx = ctx.features_exchange_pack(bounds)
    assert pmx == mx and counts.sum() == f.size
    np.testing.assert_array_equal(
        counts, [((f >= bounds[r]) & (f < bounds[r + 1])).sum() for r in range(3)])
    recs = np.frombuffer(send[: 16 * f.size].tobytes(),
                         dtype=[("ts", "<i8"), ("file", "<i4"), ("cop", "<i4")])
    off = np.concatenate([[0], np.cumsum(counts)])
    for r in (0, 2):
        part = recs[off[r]:off[r + 1]]
        ctx.features_simulate(nf, 60.0, 3, seed=2)  # restore the whole log and primaries
        ctx.features_exchange_unpack(part.view(np.uint8).copy(), part.size, bounds[r],
                                     bounds[r + 1])
        got, _ = ctx.features_aggregate_resident()
        np.testing.assert_array_equal(got, whole[bounds[r]:bounds[r + 1]])
