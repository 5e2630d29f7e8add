"""ctypes binding of libcdr.so — the C ABI declared in include/cdr.h.

This module owns no math: every numeric operation of the hot path runs in the
HIP kernels of libcdr.so (gfx950).  If the library is missing or no GPU is
visible, the calls raise — there is deliberately no CPU fallback.

Error mapping (include/cdr.h status codes -> Python exceptions), chosen to
mirror what the reference raises in the same situations:
    CDR_ERR_ARG         -> ValueError
    CDR_ERR_NAN         -> ValueError("Probabilities contain NaN")
                           (numpy Generator.choice, src/kmeans_plusplus.py:19)
    CDR_ERR_HIP         -> RuntimeError
    CDR_ERR_STATE       -> RuntimeError
    CDR_ERR_UNSUPPORTED -> NotImplementedError
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CDR_LIB", os.path.join(_HERE, "libcdr.so"))

CDR_OK = 0
CDR_ERR_ARG = 1
CDR_ERR_HIP = 2
CDR_ERR_NAN = 3
CDR_ERR_STATE = 4
CDR_ERR_UNSUPPORTED = 5
MODE_F32X = 1
MODE_F64 = 2
SEED_BLOCK = 8192

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_F64 = ctypes.c_double
_PI64 = ctypes.POINTER(ctypes.c_int64)
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PF64 = ctypes.POINTER(ctypes.c_double)

# name -> (argtypes, restype); restype None means "int status".
SIGNATURES = {
    "cdr_last_error": ([], ctypes.c_char_p),
    "cdr_version": ([], ctypes.c_int),
    "cdr_device_count": ([ctypes.POINTER(ctypes.c_int)], None),
    "cdr_create": ([ctypes.c_int, ctypes.POINTER(_P)], None),
    "cdr_destroy": ([_P], None),
    "cdr_set_stream": ([_P, _P], None),
    "cdr_synchronize": ([_P], None),
    "cdr_points_load_f64": ([_P, _P, _I64, _I32], None),
    "cdr_points_generate": ([_P, _I64, _I64, _I64, _I32, _I32, _U64], None),
    "cdr_points_info": ([_P, _PI64, _PI32, _PI32, _PI32], None),
    "cdr_points_get_rows": ([_P, _P, _I64, _P], None),
    "cdr_points_stats": ([_P, _P], None),
    "cdr_points_restat": ([_P, _P, _I64], None),
    "cdr_seed_reset": ([_P], None),
    "cdr_seed_update": ([_P, _P], None),
    "cdr_seed_num_blocks": ([_P, _PI64], None),
    "cdr_seed_block_sums": ([_P, _P], None),
    "cdr_seed_scan": ([_P, _F64, _F64, _PF64], None),
    "cdr_seed_search": ([_P, _F64, _F64, _PI64], None),
    "cdr_seed_scan_begin": ([_P, _F64, _F64, _PI64, _PI64], None),
    "cdr_seed_scan_items": ([_P, _P, _I64, _PI64], None),
    "cdr_seed_scan_end": ([_P, _F64, _PF64], None),
    "cdr_seed_program_eval": ([_P, _I64, _F64, _PF64, _PI32], None),
    "cdr_seed_stats": ([_P, _PI64], None),
    "cdr_seed_run": ([_P, _I64, _I32, _P, _P], None),
    "cdr_seed_shard_begin": ([_P, _I64, _I64, _I32, _I32, _I64, _I32, _P, _P, _P], None),
    "cdr_seed_shard_phase": ([_P, _I32, _P, _P], None),
    "cdr_seed_shard_end": ([_P, _P, _P, _P, _P], None),
    "cdr_seed_run_sharded": ([_P, _I64, _I64, _I64, _I32, _P, _P, _P, _P], None),
    "cdr_lloyd_step": ([_P, _P, _I32, _P, _I32], None),
    "cdr_lloyd_step_f64": ([_P, _P, _I32, _P, _P], None),
    "cdr_lloyd_f64_run": ([_P, _P, _I32, _I32, _F64, _P, _P, _P, _P], None),
    "cdr_lloyd_step_f32r": ([_P, _P, _I32, _P, _P], None),
    "cdr_f32r_seed_update": ([_P, _P, _I32, _P], None),
    "cdr_f32r_seed_run": ([_P, _I64, _I32, _P, _P], None),
    "cdr_lloyd_labels": ([_P, _P], None),
    "cdr_lloyd_stats": ([_P, _PI64], None),
    "cdr_debug_screen": ([_P, _P, _I32, _P, _P], None),
    "cdr_profile_reset": ([_P, _I32], None),
    "cdr_profile_read": ([_P, _P], None),
    "cdr_profile_read_sub": ([_P, _P], None),
    "cdr_f64s_begin": ([_P, _P, _I32, _I32, _I32, _P, _P], None),
    "cdr_f64s_build": ([_P, _P, _P], None),
    "cdr_f64s_finish": ([_P, _P, _P, _P, _P, _P], None),
    "cdr_f64s_chain": ([_P, _P], None),
    "cdr_profile_kernel": ([_P, _P, _I32], None),
    "cdr_points_sqdev": ([_P, _P, _PF64], None),
    "cdr_lloyd_begin": ([_P, _P, _I32, _F64, _I32, _P, _F64], None),
    "cdr_lloyd_enqueue_assign": ([_P, _P], None),
    "cdr_lloyd_enqueue_finalize": ([_P, _P], None),
    "cdr_lloyd_status": ([_P, _P, _P], None),
    "cdr_lloyd_read": ([_P, _P, _P, _P], None),
    "cdr_lloyd_resume": ([_P, _P, _I32, _I32], None),
    "cdr_lloyd_end": ([_P], None),
    "cdr_lloyd_enqueue_steps": ([_P, _I32], None),
    "cdr_comm_unique_id": ([_P], None),
    "cdr_comm_init": ([_P, _P, _I32, _I32], None),
    "cdr_comm_destroy": ([_P], None),
    "cdr_comm_available": ([ctypes.POINTER(ctypes.c_int32)], None),
    "cdr_comm_ranks": ([_P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)], None),
    "cdr_build_id": ([], ctypes.c_char_p),
    "cdr_medians_segmented": ([_P, _P, _P, _I64, _P], None),
    "cdr_medians_by_label": ([_P, _I32, _P], None),
    "cdr_features_aggregate": ([_P, _I64, _P, _P, _P, _P, _I64, _P, _P, _PI64], None),
    "cdr_features_finalize": ([_P, _I64, _P, _P, _F64, _P], None),
    "cdr_features_generate": ([_P, _I64, _I64, ctypes.c_uint64, _I64, _I64], None),
    "cdr_features_aggregate_resident": ([_P, _P, _PI64], None),
    "cdr_features_events_read": ([_P, _P, _P, _P, _P, _P], None),
    "cdr_features_groupby_info": ([_P, _P], None),
    "cdr_lloyd_f64_walked": ([_P, _PI64], None),
    "cdr_medians_group": ([_P, _I32, _P], None),
    "cdr_medians_begin": ([_P, _P, ctypes.POINTER(ctypes.c_int32), _PI64], None),
    "cdr_medians_pass_hist": ([_P, _I32, _P], None),
    "cdr_medians_pass_select": ([_P, _I32, _P], None),
    "cdr_medians_finish": ([_P, _P], None),
    "cdr_features_exchange_pack": ([_P, _I32, _P, _P, _P, _PI64], None),
    "cdr_features_exchange_unpack": ([_P, _P, _I64, _I64, _I64], None),
    "cdr_features_load_events": ([_P, _I64, _P, _P, _P, _P, _I64, _P], None),
    "cdr_features_finalize_stats": ([_P, _I64, _P, _P, ctypes.c_double, _P, _P], None),
    "cdr_features_finalize_apply": ([_P, _I64, _P, _P, ctypes.c_double, _P, _P, _I64, _P],
                                    None),
    "cdr_features_simulate": ([_P, _I64, _I64, ctypes.c_double, _I32, ctypes.c_uint64, _I64,
                               _PI64], None),
    "cdr_ingest_manifest": ([_P, _I64, _P, _P, _P, _I32, _P, _P], None),
    "cdr_ingest_log": ([_P, _P, _I64, _P], None),
    "cdr_ingest_reparse": ([_P, _P], None),
    "cdr_host_seq_sum": ([_P, _I64, _F64], ctypes.c_double),
}

_lib = None
_lib_lock = threading.Lock()


def source_build_id() -> str | None:
    """Hash of the sources libcdr.so is built from (csrc/Makefile BUILD_ID):
    the sorted *.hip and *.h of csrc/, then include/cdr.h; None when the
    sources are not next to the module."""
    import hashlib

    csrc = os.path.join(_HERE, "csrc")
    hdr = os.path.join(os.path.dirname(_HERE), "include", "cdr.h")
    if not (os.path.isdir(csrc) and os.path.exists(hdr)):
        return None
    names = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h")))
    h = hashlib.sha256()
    for f in [os.path.join(csrc, f) for f in names] + [hdr]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libcdr.so once.  Raises ImportError when it has not been built or
    was built from other sources than the ones next to it (a stale binary)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise ImportError(
                f"libcdr.so not found at {path}: build it with "
                "`make -C clustering-driven-replication-strategy_amd/csrc` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        want = source_build_id() if path == LIB_PATH else None
        if want is not None:
            fn = getattr(lib, "cdr_build_id", None)
            got = None
            if fn is not None:
                fn.restype = ctypes.c_char_p
                got = fn().decode()
            if got != want:
                raise ImportError(
                    f"stale libcdr.so at {path}: built from sources {got}, the sources "
                    f"here are {want}; rebuild with `make -C "
                    "clustering-driven-replication-strategy_amd/csrc`")
        for name, (argt, rest) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argt
            fn.restype = ctypes.c_int if rest is None else rest
        _lib = lib
        return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class NanProbabilities(ValueError):
    """CDR_ERR_NAN: numpy Generator.choice's "Probabilities contain NaN"
    (src/kmeans_plusplus.py:19); a ValueError like the reference's."""


def _check(rc: int) -> None:
    if rc == CDR_OK:
        return
    msg = load_library().cdr_last_error().decode(errors="replace")
    if rc == CDR_ERR_NAN:
        if "do not sum to 1" in msg:  # Generator.choice on all-zero probabilities
            raise ValueError("Probabilities do not sum to 1. See Notes section of docstring "
                             "for more information.")
        raise NanProbabilities("Probabilities contain NaN")
    if rc == CDR_ERR_ARG:
        raise ValueError(msg)
    if rc == CDR_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(f"libcdr: {msg}")


def device_count() -> int:
    lib = load_library()
    n = ctypes.c_int(0)
    _check(lib.cdr_device_count(ctypes.byref(n)))
    return int(n.value)


def comm_available() -> bool:
    """librccl loads (dlopen / dlsym only; no bootstrap listener is started)."""
    ok = ctypes.c_int32(0)
    _check(load_library().cdr_comm_available(ctypes.byref(ok)))
    return bool(ok.value)


def comm_unique_id() -> bytes:
    """A fresh 128-byte RCCL unique id (one rank creates it and broadcasts)."""
    out = np.zeros(128, dtype=np.uint8)
    _check(load_library().cdr_comm_unique_id(_ptr(out)))
    return out.tobytes()


# cdr_seed_item (include/cdr.h): one item of a shard's cumsum program
SEED_ITEM = np.dtype([("d0", "<i8"), ("d1", "<i8"), ("p", "<f8"), ("e", "<i4"),
                      ("kind", "<i4")])
SEED_RUN, SEED_CROSS, SEED_CONST, SEED_FINE, SEED_MARK, SEED_END, SEED_SKIP, SEED_BAD = range(8)


def seed_program_eval(items: np.ndarray, c_in: float) -> tuple[float, bool]:
    """Runs a cumsum program (cdr_seed_program_eval, host only): the running
    value after the shard from c_in, and whether every item held."""
    items = np.ascontiguousarray(items, dtype=SEED_ITEM)
    c, ok = _F64(), _I32()
    _check(load_library().cdr_seed_program_eval(_ptr(items), items.size, float(c_in),
                                                ctypes.byref(c), ctypes.byref(ok)))
    return float(c.value), bool(ok.value)


def host_seq_sum(v: np.ndarray, init: float = 0.0) -> float:
    """((init + v[0]) + v[1]) + ... in fp64 (plain C on the host)."""
    v = np.ascontiguousarray(v, dtype=np.float64)
    return float(load_library().cdr_host_seq_sum(_ptr(v), v.size, float(init)))


class Context:
    """One libcdr context = one HIP device + one shard of points."""

    def __init__(self, device: int = 0):
        lib = load_library()
        h = _P()
        _check(lib.cdr_create(int(device), ctypes.byref(h)))
        self._lib = lib
        self._h = h
        self.device = int(device)
        self.restat_n = None  # n_sum of the last cdr_points_restat (cdr_dist.unify_points)

    # -- lifecycle -------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.cdr_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle: int | None) -> None:
        _check(self._lib.cdr_set_stream(self._h, _P(stream_handle or 0)))
        self._stream = int(stream_handle) if stream_handle else None

    def stream_handle(self) -> int | None:
        """The caller's HIP stream this context enqueues on (set_stream), or
        None while it uses its own stream."""
        return getattr(self, "_stream", None)

    def synchronize(self) -> None:
        _check(self._lib.cdr_synchronize(self._h))

    # -- points ----------------------------------------------------------
    def load_points(self, X: np.ndarray) -> None:
        X = np.ascontiguousarray(X, dtype=np.float64)
        if X.ndim != 2:
            raise ValueError("X must be 2-dimensional (n_samples, n_features)")
        self.restat_n = None  # (cdr_dist.unify_points: not combined over shards)
        _check(self._lib.cdr_points_load_f64(self._h, _ptr(X), X.shape[0], X.shape[1]))

    def generate_points(self, n_total: int, row_begin: int, n_local: int, d: int,
                        n_blobs: int, seed: int) -> None:
        self.restat_n = None
        _check(self._lib.cdr_points_generate(self._h, n_total, row_begin, n_local, d,
                                             n_blobs, ctypes.c_uint64(seed & (2**64 - 1))))

    def info(self) -> dict:
        n, d, mode, s = _I64(), _I32(), _I32(), _I32()
        _check(self._lib.cdr_points_info(self._h, ctypes.byref(n), ctypes.byref(d),
                                         ctypes.byref(mode), ctypes.byref(s)))
        return {"n": n.value, "d": d.value, "mode": mode.value, "scale_bits": s.value}

    def points_stats(self) -> np.ndarray:
        """This shard's point statistics (include/cdr.h cdr_points_stats)."""
        st = np.zeros(2 * self.info()["d"] + 3, dtype=np.uint64)
        _check(self._lib.cdr_points_stats(self._h, _ptr(st)))
        return st

    def points_restat(self, st: np.ndarray, n_sum: int) -> None:
        """Mode / scale / screen transform from statistics combined over
        every shard (cdr_points_restat)."""
        st = np.ascontiguousarray(st, dtype=np.uint64)
        _check(self._lib.cdr_points_restat(self._h, _ptr(st), int(n_sum)))
        self.restat_n = int(n_sum)

    def get_rows(self, idx) -> np.ndarray:
        idx = np.ascontiguousarray(np.atleast_1d(idx), dtype=np.int64)
        d = self.info()["d"]
        out = np.empty((idx.size, d), dtype=np.float64)
        _check(self._lib.cdr_points_get_rows(self._h, _ptr(idx), idx.size, _ptr(out)))
        return out

    # -- seeding ---------------------------------------------------------
    def seed_reset(self) -> None:
        _check(self._lib.cdr_seed_reset(self._h))

    def seed_update(self, c: np.ndarray) -> None:
        c = np.ascontiguousarray(c, dtype=np.float64).ravel()
        _check(self._lib.cdr_seed_update(self._h, _ptr(c)))

    def seed_num_blocks(self) -> int:
        v = _I64()
        _check(self._lib.cdr_seed_num_blocks(self._h, ctypes.byref(v)))
        return int(v.value)

    def seed_block_sums(self) -> np.ndarray:
        out = np.empty(self.seed_num_blocks(), dtype=np.float64)
        if out.size:
            _check(self._lib.cdr_seed_block_sums(self._h, _ptr(out)))
        return out

    def seed_scan(self, total: float, c_in: float = 0.0) -> float:
        v = _F64()
        _check(self._lib.cdr_seed_scan(self._h, float(total), float(c_in), ctypes.byref(v)))
        return float(v.value)

    def seed_scan_begin(self, total: float, c_guess: float) -> tuple[int, int]:
        """Builds this shard's cumsum program under a guess of its starting
        running value; returns (items, FINE items), items -1 when it did
        not fit (cdr_seed_scan_begin)."""
        ni, nf = _I64(), _I64()
        _check(self._lib.cdr_seed_scan_begin(self._h, float(total), float(c_guess),
                                             ctypes.byref(ni), ctypes.byref(nf)))
        return int(ni.value), int(nf.value)

    def seed_scan_items(self, n_items: int) -> np.ndarray:
        out = np.zeros(max(int(n_items), 0), dtype=SEED_ITEM)
        got = _I64()
        _check(self._lib.cdr_seed_scan_items(self._h, _ptr(out) if out.size else None, out.size,
                                             ctypes.byref(got)))
        return out[: got.value]

    def seed_scan_end(self, c_in: float) -> float:
        """The exact scan from c_in with the program of seed_scan_begin."""
        v = _F64()
        _check(self._lib.cdr_seed_scan_end(self._h, float(c_in), ctypes.byref(v)))
        return float(v.value)

    def seed_run(self, first: int, k: int, u) -> np.ndarray:
        """k-means++ seeding of this context's points with no host round trip
        per step (cdr_seed_run): first row index and the k - 1 uniforms of the
        draws -> the k picked row indices."""
        u = np.ascontiguousarray(u, dtype=np.float64)
        if u.size != max(k - 1, 0):
            raise ValueError("need k - 1 uniforms")
        picks = np.zeros(max(int(k), 1), dtype=np.int64)
        _check(self._lib.cdr_seed_run(self._h, int(first), int(k), _ptr(u) if u.size else None,
                                      _ptr(picks)))
        return picks[:k]

    # -- device-resident seeding over sharded rows (include/cdr.h) -----------
    def seed_shard_begin(self, row_begin: int, n_total: int, nranks: int, rank: int, first: int,
                         k: int, u, red: int) -> np.ndarray:
        """Starts the sharded device seeding; writes this rank's part of the
        first all-reduce into the device buffer `red` (d + 4 doubles) and
        returns the bytes per rank of the three exchanged buffers."""
        u = np.ascontiguousarray(u, dtype=np.float64)
        if u.size != max(k - 1, 0):
            raise ValueError("need k - 1 uniforms")
        sizes = np.zeros(3, dtype=np.int64)
        self._ss_k = int(k)
        _check(self._lib.cdr_seed_shard_begin(self._h, int(row_begin), int(n_total), int(nranks),
                                              int(rank), int(first), int(k),
                                              _ptr(u) if u.size else None, _P(red), _ptr(sizes)))
        return sizes

    def seed_shard_phase(self, phase: int, buf_in: int, buf_out: int) -> None:
        _check(self._lib.cdr_seed_shard_phase(self._h, int(phase), _P(buf_in), _P(buf_out)))

    def seed_shard_end(self, red: int):
        """(picks (k,) global rows, centres (k, d) fp64, status: 0 ok, 1 run
        the host protocol instead, 2 Probabilities contain NaN)."""
        k, d = self._ss_k, self.info()["d"]
        picks = np.zeros(k, dtype=np.int64)
        cents = np.zeros((k, d), dtype=np.float64)
        st = ctypes.c_int32(0)
        _check(self._lib.cdr_seed_shard_end(self._h, _P(red), _ptr(picks), _ptr(cents),
                                            ctypes.byref(st)))
        return picks, cents, int(st.value)

    def seed_run_sharded(self, row_begin: int, n_total: int, first: int, k: int, u):
        """Every step with the context's communicator (cdr_comm_init):
        (picks, centres, status) as seed_shard_end."""
        u = np.ascontiguousarray(u, dtype=np.float64)
        d = self.info()["d"]
        picks = np.zeros(max(k, 1), dtype=np.int64)
        cents = np.zeros((max(k, 1), d), dtype=np.float64)
        st = ctypes.c_int32(0)
        _check(self._lib.cdr_seed_run_sharded(self._h, int(row_begin), int(n_total), int(first),
                                              int(k), _ptr(u) if u.size else None, _ptr(picks),
                                              _ptr(cents), ctypes.byref(st)))
        return picks[:k], cents[:k], int(st.value)

    def seed_stats(self) -> dict:
        """Cumsum scans run through a program, and those that fell back to
        the block walk (cdr_seed_stats)."""
        out = np.zeros(2, dtype=np.int64)
        _check(self._lib.cdr_seed_stats(self._h, out.ctypes.data_as(_PI64)))
        return {"programs": int(out[0]), "fallbacks": int(out[1])}

    def seed_search(self, c_last: float, u: float) -> int:
        v = _I64()
        _check(self._lib.cdr_seed_search(self._h, float(c_last), float(u), ctypes.byref(v)))
        return int(v.value)

    # -- Lloyd -----------------------------------------------------------
    def lloyd_step(self, C: np.ndarray) -> np.ndarray:
        """F32X: (k, d+1) int64 fixed-point sums | counts."""
        C = np.ascontiguousarray(C, dtype=np.float64)
        k, d = C.shape
        out = np.empty((k, d + 1), dtype=np.int64)
        _check(self._lib.cdr_lloyd_step(self._h, _ptr(C), k, _ptr(out), 0))
        return out

    def lloyd_step_device(self, C: np.ndarray, out_device_ptr: int) -> None:
        """F32X: write (k, d+1) int64 into a device buffer (e.g. a torch tensor)."""
        C = np.ascontiguousarray(C, dtype=np.float64)
        _check(self._lib.cdr_lloyd_step(self._h, _ptr(C), C.shape[0], _P(out_device_ptr), 1))

    def lloyd_step_f64(self, C: np.ndarray):
        C = np.ascontiguousarray(C, dtype=np.float64)
        k, d = C.shape
        sums = np.empty((k, d), dtype=np.float64)
        counts = np.empty(k, dtype=np.int64)
        _check(self._lib.cdr_lloyd_step_f64(self._h, _ptr(C), k, _ptr(sums), _ptr(counts)))
        return sums, counts

    F64_RUN_ALL, F64_RUN_CONVERGED, F64_RUN_HOST = 0, 1, 2

    def lloyd_f64_run(self, C: np.ndarray, max_steps: int, tol: float):
        """F64: up to max_steps Lloyd steps resident on the device
        (cdr_lloyd_f64_run).  Returns (C after the applied steps, steps
        applied, reason, means, counts): reason F64_RUN_HOST = the next step
        stopped for the host (empty cluster / shift near tol) with its means
        and counts; F64_RUN_CONVERGED = the last applied step had shift < tol."""
        C = np.ascontiguousarray(C, dtype=np.float64)
        k, d = C.shape
        C_out = np.empty((k, d), dtype=np.float64)
        means = np.empty((k, d), dtype=np.float64)
        counts = np.empty(k, dtype=np.int64)
        info = np.zeros(2, dtype=np.int32)
        _check(self._lib.cdr_lloyd_f64_run(self._h, _ptr(C), k, int(max_steps), float(tol),
                                           _ptr(C_out), _ptr(means), _ptr(counts), _ptr(info)))
        return C_out, int(info[0]), int(info[1]), means, counts

    # -- sharded F64 sums (include/cdr.h cdr_f64s_*; cdr_dist.f64_sharded_sums) --
    def f64s_begin(self, C: np.ndarray, nranks: int, rank: int, tot_buf: int) -> np.ndarray:
        """Assignment of this shard + its approximate totals into its slot of
        the device buffer tot_buf; returns (tot slot bytes, program slot bytes)."""
        C = np.ascontiguousarray(C, dtype=np.float64)
        self._f64s_kd = C.shape
        sizes = np.zeros(2, dtype=np.int64)
        _check(self._lib.cdr_f64s_begin(self._h, _ptr(C), C.shape[0], int(nranks), int(rank),
                                        _P(tot_buf), _ptr(sizes)))
        return sizes

    def f64s_build(self, tot_buf: int, prog_buf: int) -> None:
        _check(self._lib.cdr_f64s_build(self._h, _P(tot_buf), _P(prog_buf)))

    def f64s_finish(self, tot_buf: int, prog_buf: int):
        """(sums (k, d), counts (k,), status: 0 exact, 1 run the rank chain)."""
        k, d = self._f64s_kd
        sums = np.empty((k, d), dtype=np.float64)
        counts = np.empty(k, dtype=np.int64)
        st = ctypes.c_int32(0)
        _check(self._lib.cdr_f64s_finish(self._h, _P(tot_buf), _P(prog_buf), _ptr(sums),
                                         _ptr(counts), ctypes.byref(st)))
        return sums, counts, int(st.value)

    def f64s_chain(self, chain_buf: int) -> None:
        _check(self._lib.cdr_f64s_chain(self._h, _P(chain_buf)))

    def lloyd_step_f32r(self, C: np.ndarray):
        """The reference's float32 step: (sequential fp32 sums as float64
        (k, d), counts (k,)); labels from the fp32 norms."""
        C = np.ascontiguousarray(C, dtype=np.float32)
        k, d = C.shape
        sums = np.empty((k, d), dtype=np.float64)
        counts = np.empty(k, dtype=np.int64)
        _check(self._lib.cdr_lloyd_step_f32r(self._h, _ptr(C), k, _ptr(sums), _ptr(counts)))
        return sums, counts

    def f32r_seed_update(self, c: np.ndarray, reset: bool) -> float:
        """The reference's float32 seeding step; returns dist_sq.sum() (fp32)
        and stages fp32(dist_sq / total) for seed_scan(1.0, ...)."""
        c = np.ascontiguousarray(c, dtype=np.float32).ravel()
        tot = ctypes.c_float()
        code = self._lib.cdr_f32r_seed_update(self._h, _ptr(c), 1 if reset else 0,
                                              ctypes.byref(tot))
        if code == CDR_ERR_NAN:
            raise NanProbabilities("Probabilities contain NaN")
        _check(code)
        return float(np.float32(tot.value))

    def f32r_seed_run(self, first: int, k: int, u) -> np.ndarray:
        """The reference's float32 seeding with every step on the device
        (cdr_f32r_seed_run): u = the k - 1 rng.random() draws; returns the
        k picked rows."""
        u = np.ascontiguousarray(u, dtype=np.float64)
        picks = np.zeros(k, dtype=np.int64)
        _check(self._lib.cdr_f32r_seed_run(self._h, int(first), int(k),
                                           _ptr(u) if u.size else None, _ptr(picks)))
        return picks

    def f64_walked(self) -> int:
        """Blocks the last F64 step re-added element-wise (-1: serial kernel)."""
        v = _I64()
        _check(self._lib.cdr_lloyd_f64_walked(self._h, ctypes.byref(v)))
        return int(v.value)

    def labels(self) -> np.ndarray:
        out = np.empty(self.info()["n"], dtype=np.int64)
        _check(self._lib.cdr_lloyd_labels(self._h, _ptr(out)))
        return out

    def fallback_count(self) -> int:
        v = _I64()
        _check(self._lib.cdr_lloyd_stats(self._h, ctypes.byref(v)))
        return int(v.value)

    def profile_reset(self, enable: bool = True, every: int = 1) -> None:
        """Collect HIP-event timings of every ``every``-th following step."""
        _check(self._lib.cdr_profile_reset(self._h, max(int(every), 1) if enable else 0))

    def profile_read(self) -> dict:
        out = np.zeros(6, dtype=np.float64)
        _check(self._lib.cdr_profile_read(self._h, _ptr(out)))
        return {"screen_ms": out[0], "steps": int(out[1]), "step_ms": out[2],
                "fallback_points": int(out[3]), "queued_points": int(out[4]),
                "tight_points": int(out[5])}

    def profile_read_sub(self) -> dict:
        """Steps whose screen ran as two kernels (the split bounded screen):
        time from the step start to the end of the first kernel (screen32bz)."""
        out = np.zeros(2, dtype=np.float64)
        _check(self._lib.cdr_profile_read_sub(self._h, _ptr(out)))
        return {"first_ms": out[0], "steps": int(out[1])}

    def profile_kernel(self) -> str:
        buf = ctypes.create_string_buffer(96)
        _check(self._lib.cdr_profile_kernel(self._h, buf, 96))
        return buf.value.decode()

    # -- device-resident Lloyd loop (csrc/loop.hip) ---------------------------
    LL_RUNNING, LL_CONVERGED, LL_EMPTY, LL_HOST_PLAN, LL_AMBIGUOUS = 0, 1, 2, 3, 4

    def points_sqdev(self, ref) -> float:
        ref = np.ascontiguousarray(ref, dtype=np.float64)
        v = _F64()
        _check(self._lib.cdr_points_sqdev(self._h, _ptr(ref), ctypes.byref(v)))
        return float(v.value)

    def lloyd_begin(self, C, tol: float, ref, x2_total: float = float("nan"),
                    round32: bool = False) -> None:
        C = np.ascontiguousarray(C, dtype=np.float64)
        ref = np.ascontiguousarray(ref, dtype=np.float64)
        self._ll_shape = C.shape
        _check(self._lib.cdr_lloyd_begin(self._h, _ptr(C), C.shape[0], float(tol),
                                         1 if round32 else 0, _ptr(ref), float(x2_total)))

    def lloyd_enqueue_assign(self, dsums_ptr: int | None = None) -> None:
        _check(self._lib.cdr_lloyd_enqueue_assign(self._h, _P(dsums_ptr or 0)))

    def lloyd_enqueue_finalize(self, dsums_ptr: int | None = None) -> None:
        _check(self._lib.cdr_lloyd_enqueue_finalize(self._h, _P(dsums_ptr or 0)))

    def lloyd_status(self) -> dict:
        st = np.zeros(4, dtype=np.int64)
        v = np.zeros(2, dtype=np.float64)
        _check(self._lib.cdr_lloyd_status(self._h, _ptr(st), _ptr(v)))
        return {"running": bool(st[0]), "steps": int(st[1]), "reason": int(st[2]),
                "enqueued": int(st[3]), "shift": float(v[0]), "inertia": float(v[1])}

    def lloyd_read(self):
        k, d = self._ll_shape
        C = np.empty((k, d), dtype=np.float64)
        means = np.empty((k, d), dtype=np.float64)
        counts = np.empty(k, dtype=np.int64)
        _check(self._lib.cdr_lloyd_read(self._h, _ptr(C), _ptr(means), _ptr(counts)))
        return C, means, counts

    def lloyd_resume(self, C=None, add_steps: int = 0, host_plan_once: bool = False) -> None:
        if C is not None:
            C = np.ascontiguousarray(C, dtype=np.float64)
        _check(self._lib.cdr_lloyd_resume(self._h, _ptr(C) if C is not None else None,
                                          int(add_steps), 1 if host_plan_once else 0))

    def lloyd_end(self) -> None:
        _check(self._lib.cdr_lloyd_end(self._h))

    def lloyd_enqueue_steps(self, m: int) -> None:
        """m loop steps (assign, all-reduce over the context's communicator,
        finalize) enqueued from C (cdr_lloyd_enqueue_steps)."""
        _check(self._lib.cdr_lloyd_enqueue_steps(self._h, int(m)))

    # -- native collective (csrc/comm.hip) ----------------------------------
    def comm_init(self, unique_id: bytes, nranks: int, rank: int) -> None:
        uid = np.frombuffer(bytes(unique_id), dtype=np.uint8).copy()
        if uid.size != 128:
            raise ValueError("unique_id must be 128 bytes")
        _check(self._lib.cdr_comm_init(self._h, _ptr(uid), int(nranks), int(rank)))

    def comm_destroy(self) -> None:
        _check(self._lib.cdr_comm_destroy(self._h))

    def comm_ranks(self) -> tuple[int, int]:
        """(nranks, rank) of the context's communicator; nranks 0: none."""
        nr, r = ctypes.c_int32(0), ctypes.c_int32(0)
        _check(self._lib.cdr_comm_ranks(self._h, ctypes.byref(nr), ctypes.byref(r)))
        return int(nr.value), int(r.value)

    def debug_screen(self, C: np.ndarray):
        C = np.ascontiguousarray(C, dtype=np.float64)
        k = C.shape[0]
        inf = self.info()
        n_pad = -(-max(inf["n"], 1) // SEED_BLOCK) * SEED_BLOCK
        kt = -(-k // 16) * 16
        vals = np.empty((n_pad, kt), dtype=np.float32)
        thr = np.empty(2, dtype=np.float32)
        _check(self._lib.cdr_debug_screen(self._h, _ptr(C), k, _ptr(vals), _ptr(thr)))
        return vals[: inf["n"], :k], thr

    # -- medians ---------------------------------------------------------
    def medians_segmented(self, values: np.ndarray, offsets: np.ndarray) -> np.ndarray:
        values = np.ascontiguousarray(values, dtype=np.float64)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        nseg = offsets.size - 1
        out = np.empty(max(nseg, 0), dtype=np.float64)
        _check(self._lib.cdr_medians_segmented(self._h, _ptr(values) if values.size else None,
                                               _ptr(offsets), nseg,
                                               _ptr(out) if out.size else None))
        return out

    def medians_by_label(self, k: int) -> np.ndarray:
        d = self.info()["d"]
        out = np.empty((k, d), dtype=np.float64)
        _check(self._lib.cdr_medians_by_label(self._h, int(k), _ptr(out)))
        return out

    def medians_group(self, k: int) -> np.ndarray:
        counts = np.zeros(int(k), dtype=np.int64)
        _check(self._lib.cdr_medians_group(self._h, int(k), _ptr(counts)))
        self._med_k = int(k)
        return counts

    def medians_begin(self, global_counts):
        g = np.ascontiguousarray(global_counts, dtype=np.int64)
        passes = ctypes.c_int32()
        words = _I64()
        _check(self._lib.cdr_medians_begin(self._h, _ptr(g), ctypes.byref(passes),
                                           ctypes.byref(words)))
        return int(passes.value), int(words.value)

    def medians_pass_hist(self, p: int, hist) -> None:
        """hist: a uint32 host array or a device pointer (int)."""
        _check(self._lib.cdr_medians_pass_hist(self._h, int(p),
                                               hist if isinstance(hist, int) else _ptr(hist)))

    def medians_pass_select(self, p: int, hist) -> None:
        _check(self._lib.cdr_medians_pass_select(self._h, int(p),
                                                 hist if isinstance(hist, int) else _ptr(hist)))

    def medians_finish(self) -> np.ndarray:
        out = np.empty((self._med_k, self.info()["d"]), dtype=np.float64)
        _check(self._lib.cdr_medians_finish(self._h, _ptr(out)))
        return out

    # -- features --------------------------------------------------------
    def features_aggregate(self, file_idx, op, client, ts_us, primary):
        file_idx = np.ascontiguousarray(file_idx, dtype=np.int32)
        op = np.ascontiguousarray(op, dtype=np.uint8)
        client = np.ascontiguousarray(client, dtype=np.int32)
        ts_us = np.ascontiguousarray(ts_us, dtype=np.int64)
        primary = np.ascontiguousarray(primary, dtype=np.int32)
        ne, nf = file_idx.size, primary.size
        out = np.zeros((nf, 6), dtype=np.int64)
        mx = _I64()
        z = lambda a: _ptr(a) if a.size else None  # noqa: E731
        _check(self._lib.cdr_features_aggregate(self._h, ne, z(file_idx), z(op), z(client),
                                                z(ts_us), nf, z(primary), z(out),
                                                ctypes.byref(mx)))
        return out, int(mx.value)

    def features_generate(self, n_events: int, n_files: int, seed: int = 0x5EED,
                          t0_us: int = 1_700_000_000_000_000, span_us: int = 600_000_000) -> None:
        _check(self._lib.cdr_features_generate(self._h, int(n_events), int(n_files),
                                               int(seed) & 0xFFFFFFFFFFFFFFFF, int(t0_us),
                                               int(span_us)))
        self._ev = (int(n_events), int(n_files))

    def features_simulate(self, n_files: int, duration_s: float = 600.0, n_clients: int = 3,
                          seed: int = 0x5EED, t0_us: int = 1_761_998_400_000_000,
                          file_begin: int = 0) -> int:
        """Device access simulator (include/cdr.h cdr_features_simulate);
        returns the number of events left resident."""
        ne = _I64()
        _check(self._lib.cdr_features_simulate(self._h, int(n_files), int(file_begin),
                                               float(duration_s), int(n_clients),
                                               int(seed) & 0xFFFFFFFFFFFFFFFF, int(t0_us),
                                               ctypes.byref(ne)))
        self._ev = (int(ne.value), int(n_files))
        return int(ne.value)

    def features_aggregate_resident(self, to_host: bool = True):
        ne, nf = self._ev
        out = np.zeros((nf, 6), dtype=np.int64) if to_host else None
        mx = _I64()
        _check(self._lib.cdr_features_aggregate_resident(
            self._h, _ptr(out) if to_host else None, ctypes.byref(mx)))
        return out, int(mx.value)

    def features_groupby_info(self) -> dict:
        """What the last group-by ran (include/cdr.h cdr_features_groupby_info)."""
        info = np.zeros(7, dtype=np.int64)
        _check(self._lib.cdr_features_groupby_info(self._h, _ptr(info)))
        return {"hand": int(info[0]), "L": int(info[1]), "passes": int(info[2]),
                "payload_bytes": int(info[3]), "big_buckets": int(info[4]),
                "dense": int(info[5]), "bucket_grid": int(info[6])}

    def features_events_read(self):
        ne, nf = self._ev
        f = np.empty(ne, dtype=np.int32)
        op = np.empty(ne, dtype=np.uint8)
        cl = np.empty(ne, dtype=np.int32)
        ts = np.empty(ne, dtype=np.int64)
        pr = np.empty(nf, dtype=np.int32)
        _check(self._lib.cdr_features_events_read(self._h, _ptr(f), _ptr(op), _ptr(cl), _ptr(ts),
                                                  _ptr(pr)))
        return f, op, cl, ts, pr

    # -- access-log ingest (csrc/ingest.hip) -------------------------------
    def ingest_manifest(self, paths, primary, nodes) -> None:
        """Device dictionaries of the manifest paths and primary node names
        (None paths never match, like an empty log field)."""
        pb, po = _pack_strings(paths)
        nb, no = _pack_strings(nodes)
        primary = np.ascontiguousarray(primary, dtype=np.int32)
        if primary.size != len(po) - 1:
            raise ValueError("primary must have one entry per manifest path")
        _check(self._lib.cdr_ingest_manifest(self._h, len(po) - 1, _ptr(pb), _ptr(po),
                                             _ptr(primary), len(no) - 1, _ptr(nb), _ptr(no)))
        self._ing_nf = len(po) - 1

    def ingest_log(self, data) -> np.ndarray:
        """Parse the log bytes on the device into the resident events.  Returns
        status (6,) int64: records, first bad-timestamp record, first record
        the device tokeniser does not take, bad-timestamp count, byte span of
        the reported record (include/cdr.h)."""
        buf = np.frombuffer(memoryview(data), dtype=np.uint8)
        st = np.zeros(6, dtype=np.int64)
        _check(self._lib.cdr_ingest_log(self._h, _ptr(buf) if buf.size else None, buf.size,
                                        _ptr(st)))
        self._ev = (int(st[0]), self._ing_nf)
        return st

    def ingest_reparse(self) -> np.ndarray:
        st = np.zeros(6, dtype=np.int64)
        _check(self._lib.cdr_ingest_reparse(self._h, _ptr(st)))
        self._ev = (int(st[0]), self._ing_nf)
        return st

    # -- sharded aggregation (csrc/exchange.hip) ----------------------------
    XREC_BYTES = 16

    def features_exchange_pack(self, bounds, send=None):
        """Resident events grouped by owner rank of bounds (nranks + 1 rows).
        `send`: a host uint8 array or (device pointer) int with room for
        16 bytes per resident event; None -> a host array is allocated.
        Returns (send, counts (nranks,), max_ts_us)."""
        bounds = np.ascontiguousarray(bounds, dtype=np.int64)
        nr = bounds.size - 1
        ne = self._ev[0]
        if send is None:
            send = np.zeros(max(ne, 1) * self.XREC_BYTES, dtype=np.uint8)
        counts = np.zeros(nr, dtype=np.int64)
        mx = _I64()
        ptr = send if isinstance(send, int) else _ptr(send)
        _check(self._lib.cdr_features_exchange_pack(self._h, nr, _ptr(bounds), ptr,
                                                    _ptr(counts), ctypes.byref(mx)))
        return send, counts, int(mx.value)

    def features_exchange_unpack(self, recv, n: int, file_begin: int, file_end: int) -> None:
        ptr = recv if isinstance(recv, int) else (_ptr(recv) if n else None)
        _check(self._lib.cdr_features_exchange_unpack(self._h, ptr, int(n), int(file_begin),
                                                      int(file_end)))
        self._ev = (int(n), int(file_end - file_begin))

    def features_load_events(self, file_idx, op, client, ts_us, primary) -> None:
        f = np.ascontiguousarray(file_idx, dtype=np.int32)
        o = np.ascontiguousarray(op, dtype=np.uint8)
        c = np.ascontiguousarray(client, dtype=np.int32)
        t = np.ascontiguousarray(ts_us, dtype=np.int64)
        p = np.ascontiguousarray(primary, dtype=np.int32)
        _check(self._lib.cdr_features_load_events(self._h, f.size, _ptr(f), _ptr(o), _ptr(c),
                                                  _ptr(t), p.size, _ptr(p)))
        self._ev = (int(f.size), int(p.size))

    def features_finalize_stats(self, counts, creation_s, observation_end: float):
        counts = np.ascontiguousarray(counts, dtype=np.int64)
        creation_s = np.ascontiguousarray(creation_s, dtype=np.float64)
        ist = np.zeros(7, dtype=np.int64)
        dst = np.zeros(4, dtype=np.float64)
        _check(self._lib.cdr_features_finalize_stats(self._h, creation_s.size, _ptr(counts),
                                                     _ptr(creation_s), float(observation_end),
                                                     _ptr(ist), _ptr(dst)))
        return ist, dst

    def features_finalize_apply(self, counts, creation_s, observation_end: float, istats,
                                dstats, n_rows_total: int) -> np.ndarray:
        counts = np.ascontiguousarray(counts, dtype=np.int64)
        creation_s = np.ascontiguousarray(creation_s, dtype=np.float64)
        ist = np.ascontiguousarray(istats, dtype=np.int64)
        dst = np.ascontiguousarray(dstats, dtype=np.float64)
        n = creation_s.size
        out = np.zeros((n, 10), dtype=np.float64)
        _check(self._lib.cdr_features_finalize_apply(self._h, n, _ptr(counts), _ptr(creation_s),
                                                     float(observation_end), _ptr(ist),
                                                     _ptr(dst), int(n_rows_total), _ptr(out)))
        return out

    def features_finalize(self, counts, creation_s, observation_end: float) -> np.ndarray:
        counts = np.ascontiguousarray(counts, dtype=np.int64)
        creation_s = np.ascontiguousarray(creation_s, dtype=np.float64)
        nf = creation_s.size
        out = np.zeros((nf, 10), dtype=np.float64)
        if nf:
            _check(self._lib.cdr_features_finalize(self._h, nf, _ptr(counts), _ptr(creation_s),
                                                   float(observation_end), _ptr(out)))
        return out


def _pack_strings(strs):
    """UTF-8 bytes + int64 offsets (n+1) of a list of str (None -> empty)."""
    enc = [b"" if v is None else v.encode("utf-8") for v in strs]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        np.cumsum([len(b) for b in enc], out=off[1:])
    data = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8)
    return data, off


_default_ctx: Context | None = None


def default_context() -> Context:
    """Process-wide context on LOCAL_RANK's device (0 when not distributed)."""
    global _default_ctx
    if _default_ctx is None:
        dev = int(os.environ.get("CDR_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        _default_ctx = Context(dev)
    return _default_ctx


def loaded_library_path() -> str | None:
    """Path of the loaded libcdr (for 'native code loaded' checks)."""
    return LIB_PATH if _lib is not None else None


__all__ = ["Context", "default_context", "load_library", "device_count", "host_seq_sum",
           "comm_unique_id", "comm_available", "NanProbabilities",
           "MODE_F32X", "MODE_F64", "SEED_BLOCK", "SIGNATURES", "LIB_PATH"]

if __name__ == "__main__":  # pragma: no cover
    load_library()
    print("libcdr loaded from", LIB_PATH, "devices:", device_count(), file=sys.stderr)
