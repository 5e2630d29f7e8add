#!/usr/bin/env python3
"""Lloyd throughput on MI355X — BASELINE.json metric
"Lloyd point-iters/sec (whole node) + achieved HBM GB/s, 100M files d=16 k=64".

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

A step = one full Lloyd iteration of src/kmeans_plusplus.py:31-48 over the
whole sharded data set: fused assign+update kernels on every rank, one RCCL
SUM all-reduce of the k x (d+1) int64 partials, then the means, the shift
and the convergence test on the device (csrc/loop.hip; the host polls once
per timed region and would take over for an empty cluster) — nothing
skipped; tol is disabled so exactly K steps run.  Inputs are generated on the
device (synthetic, oracle/synth.py formula) and resident in HBM before
timing; the initial centroids come from the sharded k-means++ seeding (timed
separately, `seed_s`).  Default "scaling": "strong": the config's 100M points
in total, sharded in 8192-row blocks over the N ranks (`--scaling weak`: N x
100M).  `--gpus N` without a launcher spawns the N ranks itself.

stdout carries exactly one JSON line (rank 0): native libraries that print
banners (RCCL) are pointed at stderr.

roofline: the dominant kernel is the screen kernel (assign + fused update),
timed by HIP events on the context stream around every 4th launch of the
timed region.  `frac` is an HBM fraction of the bytes that kernel moves: the
PMC-measured HBM bytes per launch (`traffic`, profiles/pmc_traffic.json, when
a rocprof pass of this kernel at this size is committed) or else the bytes it
must move by construction (`kernel_bytes_per_launch`: the bounded screen's
2-byte bound word per point (screen32bs16) + the fp32 row of each point whose
bound failed),
divided by its mean launch time and 8 TB/s.  The SURVEY.md 8(d) contract
figure, n_local * (4*d + 4) bytes (read the fp32 point, write its int32 label),
over the same time is `effective_achieved` / `effective_frac` — above 1,
because the kernel does not need those bytes.

cpu_baseline: the NumPy oracle (restatement of the reference, 1 core — NumPy
ufuncs are single-threaded) timed on this host on a 1M-row sample of the
same data, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "clustering-driven-replication-strategy_amd")
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

CONFIGS = {
    # name: (n_total, d, k, description)
    "2": (10_000_000, 8, 16, "config 2: 10M files x d=8, k=16"),
    "3": (100_000_000, 16, 64, "config 3: 100M files x d=16, k=64"),
    "5": (50_000_000, 64, 1024, "config 5: 50M files x d=64, k=1024"),
}
# config 4 (features): the reference simulator's model (src/access_simulator.py
# with the Makefile's 600 s and 3 datanodes, src/generator.py's category mix:
# ~168 events per file), sized so that 8 GPUs hold ~1B events
FEATURES_CFG = (744_000, 600.0, 3,
                "config 4: 1B access-log events over 8 GPUs -> per-file features "
                "(simulator model: 744K files x 600 s x 3 datanodes = ~125M events per GPU)")
EVENTS_PER_FILE = 168.1  # mean of the simulator model (sum of category rates x 600 s)
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
MFMA_F16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/FP16 MFMA ~2.5 PF dense
METRIC = "Lloyd point-iters/sec (whole node) + achieved HBM GB/s, 100M files d=16 k=64"


def cpu_baseline(d: int, k: int, seed: int, rows: int = 1_000_000, iters: int = 2) -> dict:
    import numpy as np

    from oracle import kmeans_oracle, synth

    # a bounded sample (~10-20 s of NumPy): the oracle's assignment is O(rows k d)
    rows = max(8192, min(rows, int(rows * (16 * 64) / (d * k))))

    X = synth.generate(rows, 0, rows, d, k, seed)
    C = X[:k].copy()
    t0 = time.perf_counter()
    for _ in range(iters):
        labels = kmeans_oracle.assign(X, C)
        C = kmeans_oracle.update(X, labels, C, rows)
    dt = time.perf_counter() - t0
    return {"value": rows * iters / dt, "unit": "point-iters/s", "cores": 1, "kind": "port",
            "sample": f"{rows} rows x {iters} Lloyd iterations (assign + update) of the same "
                      f"synthetic data, d={d}, k={k}; NumPy oracle restatement of "
                      f"src/kmeans_plusplus.py:33-43 (single-threaded ufuncs), "
                      f"host has {os.cpu_count()} logical CPUs",
            "seconds": dt}


def features_bench(args, world: int, rank: int, dist, device, json_fd) -> dict:
    """Config 4: the compute_features group-by (src/compute_features.py:31-54)
    over a device-resident, time-ordered log from the device access simulator
    (csrc/simulate.hip, the model of src/access_simulator.py).  A step = one
    full group-by of this rank's events (csrc/groupby.hip: partition by file
    id, per-bucket LDS hash) plus the MAX all-reduce of the log's last
    timestamp (:48).  Weak scaling: each rank simulates and owns its files."""
    import numpy as np

    import _cdr

    nf, duration, nclients, desc = FEATURES_CFG
    if args.n_total:
        nf = max(1, int(args.n_total / EVENTS_PER_FILE))
    ctx = _cdr.Context(int(os.environ.get("LOCAL_RANK", "0")))
    if dist is not None:
        from cdr_dist import bind_stream

        bind_stream(ctx, device)
    ne = ctx.features_simulate(nf, duration, nclients, seed=args.seed, file_begin=rank * nf)

    def step():
        _, mx = ctx.features_aggregate_resident(to_host=False)
        if dist is not None:
            import torch

            t = torch.tensor([mx], dtype=torch.int64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            mx = int(t.item())
        return mx

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    ctx.synchronize()
    ctx.profile_reset(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile_reset(False)
    info = ctx.features_groupby_info()
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    per_step = elapsed / max(args.steps, 1)
    gb_ms = prof["step_ms"] / max(prof["steps"], 1)  # HIP events around the group-by
    alg_bytes = ne * (4 + 1 + 4 + 8) + nf * (4 + 6 * 8)  # events read once, counters written
    achieved = alg_bytes / (gb_ms / 1e3) / 1e9
    out = {
        "metric": "access-log events aggregated per second (whole node), compute_features group-by",
        "value": world * ne * args.steps / elapsed, "unit": "events/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": per_step * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic time-ordered access log from the device access simulator "
                "(per-file Poisson arrivals at jittered category rates, locality bias)",
        "config": {"workload": desc, "events_per_gpu": ne, "files_per_gpu": nf,
                   "parallelism": f"files and events partitioned over {world} GPU(s), "
                                  "RCCL MAX all-reduce of the last timestamp"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": pmc_traffic("4", ne),
                     "kernel": "features group-by (csrc/groupby.hip: file-id partition + "
                               "per-bucket LDS hash), all kernels of one step",
                     "alg_bytes_per_launch": alg_bytes, "kernel_ms": gb_ms,
                     "partition_ms": prof["screen_ms"] / max(prof["steps"], 1)},
        "groupby": info,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import features_oracle

        s_nf = 60_000
        s_ne = ctx.features_simulate(s_nf, duration, nclients, seed=args.seed)
        f, op, cl, ts, pr = ctx.features_events_read()
        c0 = time.perf_counter()
        features_oracle.counts_from_arrays(f, op, cl, ts, pr, s_nf)
        dt = time.perf_counter() - c0
        out["cpu_baseline"] = {"value": s_ne / dt, "unit": "events/s", "cores": 1, "kind": "port",
                               "sample": f"{s_ne} events x {s_nf} files of the same generator; "
                                         "NumPy restatement of the group-by (oracle/"
                                         "features_oracle.counts_from_arrays), 1 thread",
                               "seconds": dt}
    if rank == 0 and json_fd is not None:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    ctx.close()
    if dist is not None and json_fd is not None:
        dist.destroy_process_group()
    return out


INGEST_CFG = (20_000_000, 2_000_000,
              "config 4 ingest leg: access-log CSV (src/access_simulator.py:61-63 format) -> "
              "device tokenise + path join + group-by (20M events x 2M files per GPU)")


def make_log(ne: int, nf: int, seed: int):
    """Synthetic time-ordered access log in the simulator's line format,
    built with NumPy as fixed-width rows: (bytes, manifest paths, primaries)."""
    import numpy as np

    rng = np.random.default_rng(seed)
    pre = b"2025-11-01T12:00:00.000Z,/user/root/synth/synth_00000000.bin,"
    rd, wr = b"READ,dn0,00000\n", b"WRITE,dn0,0000\n"
    width = len(pre) + len(rd)
    rows = np.empty((ne, width), dtype=np.uint8)
    rows[:, :len(pre)] = np.frombuffer(pre, dtype=np.uint8)
    is_w = rng.random(ne) < 0.1
    rows[:, len(pre):] = np.frombuffer(rd, dtype=np.uint8)
    rows[is_w, len(pre):] = np.frombuffer(wr, dtype=np.uint8)

    def put(mask, col, ndig, vals):
        for j in range(ndig):
            rows[mask, col + ndig - 1 - j] = 48 + (vals // 10 ** j) % 10

    ms_total = (np.arange(ne, dtype=np.int64) * 600_000) // ne
    allr = slice(None)
    put(allr, 14, 2, ms_total // 60_000)
    put(allr, 17, 2, (ms_total // 1000) % 60)
    put(allr, 20, 3, ms_total % 1000)
    put(allr, len(pre) - 13, 8, rng.integers(0, nf, ne))
    cl = rng.integers(1, 4, ne)
    b = len(pre)
    put(~is_w, b + 7, 1, cl[~is_w])
    put(is_w, b + 8, 1, cl[is_w])
    pid = rng.integers(0, 10000, ne)
    put(~is_w, b + 9, 5, pid[~is_w])
    put(is_w, b + 10, 4, pid[is_w])
    paths = [f"/user/root/synth/synth_{i:08d}.bin" for i in range(nf)]
    primary = [f"dn{v}" for v in rng.integers(1, 4, nf)]
    return rows.tobytes(), paths, primary


def ingest_bench(args, world: int, rank: int, dist, device, json_fd: int) -> None:
    """Config 4, ingest leg: the access-log read + path join of
    src/compute_features.py:19-41 on the device (csrc/ingest.hip) followed by
    the group-by, from log bytes resident in HBM.  A step = tokenise + parse
    + hash-join + aggregate.  Weak scaling: each rank owns its log slice."""
    import numpy as np

    import _cdr
    import compute_features as cf

    ne, nf, desc = INGEST_CFG
    if args.n_total:
        ne, nf = args.n_total, max(1, args.n_total // 10)
    data, paths, primary = make_log(ne, nf, args.seed + rank)
    ctx = _cdr.Context(int(os.environ.get("LOCAL_RANK", "0")))
    prim, nodes = cf.encode_primary(primary)
    ctx.ingest_manifest(paths, prim, nodes)
    st = ctx.ingest_log(data)
    if st[0] != ne or st[1] != -1 or st[2] != -1:
        raise RuntimeError(f"ingest status {st.tolist()}")

    def parse_only():
        ctx.ingest_reparse()

    def step():
        ctx.ingest_reparse()
        ctx.features_aggregate_resident(to_host=False)

    def timed(fn, steps):
        for _ in range(args.warmup):
            fn()
        if dist is not None:
            dist.barrier()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        ctx.synchronize()
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            import torch

            t = torch.tensor([el], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    elapsed = timed(step, args.steps)
    parse_s = timed(parse_only, args.steps) / max(args.steps, 1)
    per_step = elapsed / max(args.steps, 1)
    nbytes = len(data)
    alg = nbytes + ne * (8 + 4 + 1 + 4 + 8)  # log read once; ends, events written
    achieved = alg / parse_s / 1e9
    out = {
        "metric": "access-log events ingested + aggregated per second (whole node)",
        "value": world * ne * args.steps / elapsed, "unit": "events/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": per_step * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic time-ordered CSV log in the simulator's format (NumPy fixed-width rows)",
        "config": {"workload": desc, "events_per_gpu": ne, "files_per_gpu": nf,
                   "log_bytes_per_gpu": nbytes,
                   "parallelism": f"log slices partitioned over {world} GPU(s)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                     "kernel": "ingest (nl_count + tile-count scan + nl_write + parse), log bytes "
                               "resident", "alg_bytes_per_launch": alg,
                     "kernel_ms": parse_s * 1e3},
        "log_GBps": nbytes / parse_s / 1e9,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import tempfile

        s_ne = 300_000
        s_data = data[: s_ne * (len(data) // ne)]
        with tempfile.NamedTemporaryFile(suffix=".log", delete=False) as fh:
            fh.write(s_data)
        c0 = time.perf_counter()
        cf.encode(paths, primary, *cf.load_access_log(fh.name))
        dt = time.perf_counter() - c0
        os.unlink(fh.name)
        out["cpu_baseline"] = {"value": s_ne / dt, "unit": "events/s", "cores": 1, "kind": "port",
                               "sample": f"first {s_ne} lines of the same log: python csv + "
                                         "ISO regex + dict join (compute_features."
                                         "load_access_log + encode, the host restatement of "
                                         "src/compute_features.py:19-41), 1 thread",
                               "seconds": dt}
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


F64_CFG = (10_000_000, 5, "F64 leg: 10M files x d=5 min-max-normalised features (not on a "
                          "2^-S grid: src/main.py:81 data), k={k}")


def f64_data(n: int, d: int, k: int, seed: int, device_index: int = 0):
    """Blob data min-max normalised per column as src/main.py:81 does (values
    off any 2^-S grid, so the points load in F64 mode).  The blobs come from
    the library's own device generator (cdr_points_generate: the
    oracle/synth.py formula) and are read back for the host normalisation."""
    import numpy as np

    import _cdr

    g = _cdr.Context(device_index)
    try:
        g.generate_points(n, 0, n, d, k, seed)
        X = g.get_rows(np.arange(n, dtype=np.int64))
    finally:
        g.close()
    mn, mx = X.min(axis=0), X.max(axis=0)
    return (X - mn) / (mx - mn)


def f64_bench(args, world: int, rank: int, dist, device, json_fd) -> dict:
    """F64 mode (`main.py`'s real data path): exact fp64
    NumPy-order assignment of every point + exact sequential-order cluster
    sums (csrc/f64sum.hip), centroids = sums / counts on the host as
    src/kmeans_plusplus.py:41 does.  One GPU: cdr_lloyd_step_f64.  N GPUs:
    the rows sharded in rank order (strong: the config's n in total; weak: n
    per GPU), each step's exact sequential sums composed from the shards'
    programs after two all-gathers (cdr_dist.f64_sharded_sums, DESIGN.md
    4.5b)."""
    import numpy as np

    import _cdr

    n, d, desc = F64_CFG
    if args.n_total:
        n = args.n_total
    k = args.k or 16
    n_total = n * world if args.scaling == "weak" else n
    X = f64_data(n_total, d, k, args.seed, int(os.environ.get("LOCAL_RANK", "0")))
    ctx = _cdr.Context(int(os.environ.get("LOCAL_RANK", "0")))
    comm = None
    if dist is not None and world > 1:
        import torch

        from cdr_dist import Comm, bind_stream, f64_sharded_sums, shard_rows

        comm = Comm(dist, device)
        bind_stream(ctx, device)
        begin, n_local = shard_rows(n_total, world, rank)
        ctx.load_points(X[begin:begin + n_local])
    else:
        ctx.load_points(X)
    if ctx.info()["mode"] != _cdr.MODE_F64:
        raise RuntimeError("F64 leg: the points did not load in F64 mode")
    C = X[np.sort(np.random.default_rng(42).choice(n_total, k, replace=False))].copy()
    # (the CPU baseline's sample: the first rows of the same data)
    cpu_rows = X[:1_000_000].copy() if rank == 0 and world == 1 and not args.no_cpu_baseline else None
    del X

    def step(C):
        if comm is not None:
            sums, counts = f64_sharded_sums(ctx, comm, C)
        else:
            sums, counts = ctx.lloyd_step_f64(C)
        nz = counts > 0
        C = C.copy()
        C[nz] = sums[nz] / counts[nz, None]
        return C

    # one GPU: the steps resident on the device (cdr_lloyd_f64_run: means and
    # shift on the device too, one synchronisation per call; tol -1 = no
    # convergence test, every step applied)
    resident = comm is None and hasattr(ctx, "lloyd_f64_run")

    def run(C, steps):
        if resident:
            C, applied, _, _, _ = ctx.lloyd_f64_run(C, steps, -1.0)
            if applied != steps:
                raise RuntimeError("F64 leg: the device run stopped early (empty cluster)")
            return C
        for _ in range(steps):
            C = step(C)
        return C

    if resident:
        # the whole warmup + timed trajectory once, untimed, from the same
        # start: the host-side data preparation leaves the GPU idle for
        # seconds, and the first milliseconds after it run below full clock
        # (tools/f64_time.py: the first of three identical runs is ~5 % slower)
        run(C, args.warmup + args.steps)
        ctx.synchronize()
    C = run(C, args.warmup)
    ctx.synchronize()
    if dist is not None:
        dist.barrier()
    # HIP events around every 4th step's kernels, as in the Lloyd leg (three
    # events a step cost the GPU a few microseconds each)
    ctx.profile_reset(True, every=4)
    t0 = time.perf_counter()
    C = run(C, args.steps)
    ctx.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    prof = ctx.profile_read()
    ctx.profile_reset(False)
    assign_ms = prof["screen_ms"] / max(prof["steps"], 1)
    kern_ms = prof["step_ms"] / max(prof["steps"], 1)
    n_local = ctx.info()["n"]
    alg = n_local * (8 * d + 4)  # read the fp64 point, write its int32 label
    achieved = alg / (assign_ms / 1e3) / 1e9
    out = {
        "metric": "Lloyd point-iters/sec, F64 mode (exact fp64 assignment + exact sequential sums)",
        "value": n_total * args.steps / elapsed, "unit": "point-iters/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
        "data": "synthetic blobs, min-max normalised on the host (non-grid fp64)",
        "config": {"workload": desc.format(k=k), "n_files": n_total, "d": d, "k": k,
                   "parallelism": "one GPU" if comm is None else
                   f"rows sharded over {world} GPUs; exact sequential sums composed from the "
                   "shards' programs after two all-gathers per step"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": pmc_traffic("f64", n_local, ctx.profile_kernel()),
                     "kernel": ctx.profile_kernel(), "alg_bytes_per_launch": alg,
                     "kernel_ms": assign_ms},
        "step_kernels_ms": kern_ms,
        # every kernel of one step (DRAM counters, profiles/pmc_traffic.json["f64"])
        "step_traffic": pmc_step_bytes("f64", n_local),
        "f64_blocks_walked": ctx.f64_walked(),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import kmeans_oracle

        iters = 2
        Xs = cpu_rows
        rows = Xs.shape[0]
        Cs = Xs[:k].copy()
        c0 = time.perf_counter()
        for _ in range(iters):
            lab = kmeans_oracle.assign(Xs, Cs)
            Cs = kmeans_oracle.update(Xs, lab, Cs, rows)
        dt = time.perf_counter() - c0
        out["cpu_baseline"] = {"value": rows * iters / dt, "unit": "point-iters/s", "cores": 1,
                               "kind": "port",
                               "sample": f"{rows} rows x {iters} Lloyd iterations of the same "
                                         f"F64 data, d={d}, k={k}; NumPy oracle restatement of "
                                         "src/kmeans_plusplus.py:33-43, 1 thread",
                               "seconds": dt}
    if rank == 0 and json_fd is not None:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    ctx.close()
    return out


def pmc_traffic(config: str, n_local: int, kname: str | None = None, steps=None):
    """HBM bytes per launch of the config's dominant kernel from the committed
    PMC passes (profiles/pmc_traffic.json: FETCH_SIZE x2 + WRITE_SIZE, the
    MI355X_MICROARCH.md gfx950 correction), when they were taken on this size
    and, if given, this kernel.  Records with one row per device-loop step
    (per_step_read / per_step_write from first_step on: the bounded screen
    re-reads fewer points as the run converges) are averaged over exactly the
    steps `steps` whose kernel times the run measured; a step outside the
    table gives None (no extrapolation)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        rec = json.load(fh)
    r = rec.get(f"{config}@{n_local}") or rec.get(config)
    if not r or int(r.get("n_local", -1)) != n_local:
        return None
    if kname is not None and not kname.startswith(str(r.get("kernel", "")).split("+")[0].split("<")[0]):
        return None
    if "per_step_read" in r:
        if not steps:
            return None
        first, rd, wr = int(r["first_step"]), r["per_step_read"], r["per_step_write"]
        vals = [rd[s - first] + wr[s - first] for s in steps if 0 <= s - first < min(len(rd), len(wr))]
        if len(vals) != len(steps):
            return None
        return float(sum(vals) / len(vals))
    return float(r["hbm_bytes_per_launch"])


def pmc_step_bytes(config: str, n_local: int):
    """All the step's kernels' HBM bytes from a committed per-step DRAM pass
    (tools/window_stats.py dramstep), when taken on this size."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        r = json.load(fh).get(config)
    if not r or int(r.get("n_local", -1)) != n_local or "step_bytes" not in r:
        return None
    return float(r["step_bytes"])


def kernel_bytes(kname: str, n_local: int, prof: dict, steps: int) -> int:
    """Bytes the step's screen kernel must move by construction (DESIGN.md
    4.3c-4.3e): the fp16 hi copy + one-byte label for screen32h/p; for the
    bounded screen32b the 4-byte bound word of every point, plus, for each
    point whose bound failed (profile counter, per step), its hi row and its
    new bound word."""
    if kname.startswith("screen32bs16<"):  # 2-byte words
        q = int(kname[len("screen32bs16<"):].split(",")[0])
        tight = prof.get("tight_points", 0) / max(steps, 1)
        return int(n_local * 2 + tight * (16 * q + 2))
    if kname.startswith("screen32bs<"):  # the fp32 row (16 Q bytes) of each re-read point
        q = int(kname[len("screen32bs<"):].split(",")[0])
        tight = prof.get("tight_points", 0) / max(steps, 1)
        return int(n_local * 4 + tight * (16 * q + 4))
    if kname.startswith("screen32b"):
        row = 32 if kname.startswith(("screen32b<3", "screen32b<4")) else 16
        tight = prof.get("tight_points", 0) / max(steps, 1)
        return int(n_local * 4 + tight * (row + 4))
    copy_b = {"screen32h1": 2 * 8, "screen32h": 2 * 16, "screen32d<1": 32, "screen32d<2": 64,
              "screen32p<1": 2 * 8, "screen32p<2": 2 * 8, "screen32p<3": 2 * 16,
              "screen32p<4": 2 * 16}
    for pre, b in copy_b.items():
        if kname.startswith(pre):
            return n_local * (b + 1)
    return n_local * (4 * 16 + 4)


def spawn_ranks(n: int) -> None:
    """`bench.py --gpus N` without a launcher: start N rank processes with
    torch.distributed.run (before anything touches the GPU) and exit with its
    status; rank 0's JSON line reaches this process's stdout."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get(
        "HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    sys.exit(subprocess.call(cmd, env=env))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="3", choices=sorted(CONFIGS) + ["4", "4-ingest", "f64"])
    ap.add_argument("--k", type=int, default=0, help="k of the f64 leg (default 16)")
    ap.add_argument("--n-total", type=int, default=0,
                    help="override the per-config point count (testing only)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="strong (default): the config's n points in total over the N GPUs; "
                         "weak: n points per GPU (N x n in total)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="config 3 at N = 1: skip the other configs' legs (secondary)")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED)
    ap.add_argument("--rccl", action="store_true",
                    help="use torch.distributed (RCCL) even at WORLD_SIZE=1 (path testing)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args.gpus)
    json_fd = os.dup(1)
    os.dup2(2, 1)  # RCCL prints its banner on stdout; keep stdout for the JSON line

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = None
    if args.rccl and "RANK" not in os.environ:  # one process without a launcher
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
    if world > 1 or args.rccl:
        import torch  # first: libcdr then binds to torch's HIP runtime
        import torch.distributed as tdist

        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = tdist
        device = torch.device("cuda", local_rank)

    if args.config == "4":
        features_bench(args, world, rank, dist, device, json_fd)
        return
    if args.config == "4-ingest":
        ingest_bench(args, world, rank, dist, device, json_fd)
        return
    if args.config == "f64":
        f64_bench(args, world, rank, dist, device, json_fd)
        if dist is not None:
            dist.destroy_process_group()
        return
    out = lloyd_bench(args, world, rank, local_rank, dist, device)
    if world == 1 and args.config == "3" and not args.no_secondary and not args.n_total:
        out["secondary"] = secondary_configs(args, rank, local_rank)
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()


def secondary_configs(args, rank: int, local_rank: int) -> dict:
    """The other BASELINE configs, measured in the same default run (N = 1
    only) after the headline's context is closed: config 2 (10M x 8, k = 16,
    50 Lloyd iterations), config 4 (its whole 1B-event workload on this one
    GPU), config 5 (50M x 64, k = 1024 + replica scoring) and the F64 leg
    (src/main.py's min-max-normalised data).  Each entry is that leg's own
    bench line (roofline included; no CPU baseline - the committed builder
    lines under profiles/ carry those)."""
    import argparse as _ap

    legs = {}
    plan = [("2", {"steps": 50, "warmup": 3}, None),
            ("4", {"steps": 10, "warmup": 2, "n_total": 1_000_000_000}, features_bench),
            ("5", {"steps": 10, "warmup": 2}, None),
            ("f64", {"steps": 20, "warmup": 2}, f64_bench)]
    for name, over, fn in plan:
        a2 = _ap.Namespace(**vars(args))
        a2.config, a2.n_total, a2.no_cpu_baseline = name, 0, True
        for key, v in over.items():
            setattr(a2, key, v)
        t0 = time.perf_counter()
        try:
            if fn is None:
                o = lloyd_bench(a2, 1, rank, local_rank, None, None)
            else:
                o = fn(a2, 1, rank, None, None, None)
        except Exception as e:  # noqa: BLE001 - recorded, the headline line still prints
            o = {"error": f"{type(e).__name__}: {e}"}
        o["leg_wall_s"] = time.perf_counter() - t0
        legs[name] = o
    return legs


def lloyd_bench(args, world: int, rank: int, local_rank: int, dist, device) -> dict:
    """Lloyd leg (configs 2, 3, 5): generation, sharded seeding, warmup steps,
    then exactly args.steps timed device-loop steps; returns the bench dict."""
    import numpy as np

    import _cdr
    from cdr_dist import Comm, DeviceLloyd, row_fetcher, seed_sharded, shard_rows, unify_points

    n_cfg, d, k, desc = CONFIGS[args.config]
    if args.n_total:
        n_cfg = args.n_total
    n_total = n_cfg * world if args.scaling == "weak" else n_cfg
    if world > 1:
        desc += (f" per GPU ({world} x {n_cfg} points in total)" if args.scaling == "weak"
                 else f", {world} shards of {n_cfg // world}+ points")
    begin, n_local = shard_rows(n_total, world, rank)
    comm = Comm(dist, device)
    ctx = _cdr.Context(local_rank)
    if dist is not None:
        from cdr_dist import bind_stream

        bind_stream(ctx, device)  # one stream: fenced collectives need no host sync
    g0 = time.perf_counter()
    ctx.generate_points(n_total, begin, n_local, d, k, args.seed)
    unify_points(ctx, comm, n_total)  # one scale / screen transform on every rank
    ctx.synchronize()
    gen_ms = (time.perf_counter() - g0) * 1e3
    native = comm.attach_native(ctx)  # each step's all-reduce issued from C (csrc/comm.hip)
    ctx.synchronize()

    t0 = time.perf_counter()
    C = seed_sharded(ctx, comm, begin, n_total, k, random_state=42)
    seed_s = time.perf_counter() - t0
    # the same seeding again with the context's buffers and seeding copies in
    # place (the first run also allocates them and builds the fp16 copy):
    # steady-state seeding, reported beside seed_s, never instead of it
    t0 = time.perf_counter()
    C2 = seed_sharded(ctx, comm, begin, n_total, k, random_state=42)
    seed_warm_s = time.perf_counter() - t0
    if not np.array_equal(C, C2):
        raise RuntimeError("the second seeding run gave other centres")

    # tol disabled: exactly warmup + steps Lloyd iterations, every one of them
    # assign + fused update + all-reduce + means on the device
    np.random.seed(0)
    run = DeviceLloyd(ctx, C, -1.0, row_fetcher(ctx, comm, begin, d), n_total, comm)
    w0 = time.perf_counter()
    if args.warmup:
        run.advance(args.warmup)
    ctx.synchronize()
    warmup_ms = (time.perf_counter() - w0) * 1e3
    # HIP events around every 4th step's kernels (an event record costs the
    # GPU a few microseconds; the kernel times are per launch either way)
    ctx.profile_reset(True, every=4)
    comm.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    done = run.advance(args.steps, chunk=max(args.steps, 1), chunk_max=max(args.steps, 1))
    ctx.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    if done != args.steps:
        raise RuntimeError(f"ran {done} of {args.steps} steps")
    prof = ctx.profile_read()
    st = run.status
    run.finish()
    scoring_ms = None
    if args.config == "5":
        # the config's "+ replica scoring per cluster" (src/main.py:96-107,
        # src/scoring.py:40-130): medians of every cluster's columns over all
        # ranks' points, then the category scores, after the timed Lloyd steps
        from cdr_dist import sharded_medians
        from scoring import ClusterClassifier

        names = [f"f{i}" for i in range(d)]
        cats = ("Hot", "Shared", "Moderate", "Archival")
        clf = ClusterClassifier({nm: 0.5 for nm in names},
                                {c: {nm: 1.0 for nm in names} for c in cats},
                                {c: {nm: (1, 1, 0, -1)[i] for nm in names}
                                 for i, c in enumerate(cats)},
                                {"Hot": 3, "Shared": 2, "Moderate": 1, "Archival": 4},
                                context=ctx)
        comm.barrier()
        ctx.synchronize()
        s0 = time.perf_counter()
        med = sharded_medians(ctx, comm, k)
        clf.classify_medians(med, names)
        comm.barrier()
        scoring_ms = (time.perf_counter() - s0) * 1e3
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    setup_ms = max(warmup_ms - args.warmup * elapsed / max(args.steps, 1) * 1e3, 0.0)
    kname = ctx.profile_kernel()
    screen_ms = prof["screen_ms"] / max(prof["steps"], 1)
    step_kernel_ms = prof["step_ms"] / max(prof["steps"], 1)
    alg_bytes = n_local * (4 * d + 4)
    # the loop steps whose kernels the HIP events timed: every 4th of the
    # timed region, from the first (loop step warmup + 1)
    prof_steps = list(range(args.warmup + 1, args.warmup + args.steps + 1, 4))[:prof["steps"]]
    traffic = pmc_traffic(args.config, n_local, kname, prof_steps)
    value = n_total * args.steps / elapsed
    if kname.startswith("screen_big"):
        # large-k regime: the L1 screen is the dense contraction 2 n k d on
        # the matrix cores (one fp16 product per centroid block)
        achieved = alg_bytes / (screen_ms / 1e3) / 1e9 if screen_ms > 0 else 0.0
        alg_flop = 2.0 * n_local * k * d
        tflops = alg_flop / (screen_ms / 1e3) / 1e12 if screen_ms > 0 else 0.0
        roofline = {"bound": "mfma", "achieved": tflops, "peak": MFMA_F16_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": tflops / MFMA_F16_PEAK_TFLOPS, "traffic": traffic,
                    "kernel": kname, "alg_flop_per_launch": alg_flop, "kernel_ms": screen_ms,
                    "hbm_alg_bytes_per_launch": alg_bytes}
    else:
        # frac is an HBM fraction of the bytes the kernel itself moves: the
        # PMC-measured traffic per launch when a rocprof pass of this kernel
        # and size is committed (profiles/pmc_traffic.json), else the bytes it
        # must move by construction (kernel_bytes_per_launch).  The SURVEY 8(d)
        # contract figure (fp32 point + int32 label per point) is kept as
        # effective_achieved / effective_frac: it exceeds 1 because the
        # kernels read a half-size fp16 copy and, on the bounded screen, only
        # the points whose drift bound failed.
        kb = kernel_bytes(kname, n_local, prof, args.steps)
        moved = traffic if traffic else kb
        achieved = moved / (screen_ms / 1e3) / 1e9 if screen_ms > 0 else 0.0
        eff = alg_bytes / (screen_ms / 1e3) / 1e9 if screen_ms > 0 else 0.0
        roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                    "bytes_basis": "pmc" if traffic else "kernel_bytes_per_launch",
                    "kernel": kname, "kernel_ms": screen_ms, "kernel_bytes_per_launch": kb,
                    "timed_steps": prof_steps,
                    "alg_bytes_per_launch": alg_bytes, "effective_achieved": eff,
                    "effective_frac": eff / HBM_PEAK_GBPS}
    # (the fallback counter accumulates over every profiled-session step)
    fb_frac = prof["fallback_points"] / max(args.steps, 1) / max(n_local, 1)
    # points the pruned screen (screen32p) handed to its k-way MFMA screen
    q_frac = prof["queued_points"] / max(args.steps, 1) / max(n_local, 1)
    # points whose drift bound failed (screen32b), re-decided from their coordinates
    t_frac = prof["tight_points"] / max(args.steps, 1) / max(n_local, 1)

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "point-iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device generator, oracle/synth.py formula; 2^-24-grid blobs)",
        "config": {"workload": desc, "n_files": n_total, "d": d, "k": k,
                   "parallelism": f"rows sharded over {world} GPU(s), RCCL all-reduce of "
                                  f"k x (d+1) int64 per step" + (
                                      " (ncclAllReduce enqueued from libcdr between the "
                                      "step's kernels)" if native else " (none at 1 GPU)"),
                   "screen": "exact drift-bound pruning (Hamerly bounds: a "
                             + ("2-byte" if kname.startswith("screen32bs16") else "4-byte")
                             + " bound word per point, coordinates re-read only where the bound fails), labels "
                             "bit-identical; re-read points decided by a certified fp16 hi/lo "
                             "split MFMA screen + exact fp64 fallback; int64 fixed-point sums "
                             "(results bit-identical to fp64 NumPy)" if kname.startswith("screen32b")
                             else "fp16 hi/lo split MFMA (certified) + exact fp64 fallback; int64 "
                                  "fixed-point sums (results bit-identical to fp64 NumPy)",
                   "loop": "device-resident (means, shift, convergence test on the device; "
                           "host polls once per timed region)"},
        "roofline": roofline,
        "step_kernels_ms": step_kernel_ms,
        "fallback_frac": fb_frac,
        "queued_frac": q_frac,
        "reread_frac": t_frac,
        "seed_s": seed_s,
        "seed_warm_s": seed_warm_s,
        "setup_ms": setup_ms,
        # wall time per Lloyd step from the first step to the last (warmup
        # steps with their one-time copies and the bound rebuild included)
        "run_ms_per_step": (warmup_ms + elapsed * 1e3) / max(args.warmup + args.steps, 1),
        "setup_note": "one-time work outside the timed steps: device point generation + "
                      "statistics (gen_ms), and the warmup steps' one-time copies (pre-centred, "
                      "fp16 hi, row-major, bound words: warmup wall time minus warmup x "
                      "ms_per_step); seeding is seed_s",
        "gen_ms": gen_ms,
        "seed_scans": ctx.seed_stats(),  # cumsum programs / fallbacks to the block walk
        "final_shift": st["shift"],
        "final_inertia": st["inertia"],
    }
    if scoring_ms is not None:
        out["replica_scoring_ms"] = scoring_ms
    ctx.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(d, k, args.seed)
    return out


if __name__ == "__main__":
    main()
