"""NumPy mirror of the device point generator (TEST INFRASTRUCTURE ONLY).

Same integer formula as ``generate_kernel`` in
clustering-driven-replication-strategy_amd/csrc/cdr_runtime.hip, so rows
generated here and on the GPU are bit-identical (checked in
tests/test_gpu_kmeans.py).  Values are u24 / 2^24 in [0, 1): a mixture of
``n_blobs`` blobs with Irwin-Hall(4) noise, clamped.
"""
from __future__ import annotations

import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _s(v: int) -> np.uint64:
    return splitmix64(np.array([v], dtype=np.uint64))[0]


def generate(n_total: int, row_begin: int, n_local: int, d: int, n_blobs: int,
             seed: int) -> np.ndarray:
    """Rows [row_begin, row_begin + n_local) as float64 (n_local, d)."""
    seed = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    s_blob = _s(int(seed ^ np.uint64(0xB10B5EED)))
    s_cent = _s(int(seed ^ np.uint64(0xCE27E25)))
    s_noise = _s(int(seed ^ np.uint64(0x9015E)))
    rows = np.arange(row_begin, row_begin + n_local, dtype=np.uint64)
    with np.errstate(over="ignore"):
        hb = splitmix64(s_blob + rows)
        b = ((hb >> np.uint64(32)) * np.uint64(n_blobs)) >> np.uint64(32)
        out = np.empty((n_local, d), dtype=np.float64)
        for f in range(d):
            hc = splitmix64(s_cent + b * np.uint64(d) + np.uint64(f))
            center = np.int64(1 << 21) + (hc % np.uint64(3 << 22)).astype(np.int64)
            hn = splitmix64(s_noise + rows * np.uint64(d) + np.uint64(f))
            m16 = np.uint64(0xFFFF)
            s = ((hn & m16).astype(np.int64) + ((hn >> np.uint64(16)) & m16).astype(np.int64)
                 + ((hn >> np.uint64(32)) & m16).astype(np.int64)
                 + (hn >> np.uint64(48)).astype(np.int64))
            u = np.clip(center + 13 * (s - 131070), 0, 0xFFFFFF)
            out[:, f] = u.astype(np.float64) / 16777216.0
    return out


def f32_hard_data(n: int, d: int, k: int, transform: str, seed: int) -> np.ndarray:
    """Inputs of the hard float32 k-means fixtures (oracle/gen_golden.py
    float32_hard_cases; the tests re-create them from these parameters):
    "synth" the blobs as they are, "grid8" on a 2^-8 grid (distance ties),
    "near20" offsets of 2^-20 around 0.5 plus a spread fifth."""
    X = generate(n, 0, n, d, max(k, 2), seed)
    if transform == "grid8":
        X = np.floor(X * 256.0) / 256.0
    elif transform == "near20":
        q = np.floor(X * 8.0) - 4.0  # -4 .. 3
        X = 0.5 + np.ldexp(q, -20)
        X[: n // 5] = generate(n, 0, n // 5, d, 3, seed + 1)
    return X.astype(np.float32)
