"""The access-log ingest checker (oracle.features_oracle.encode_log / iso_to_us)
pinned against the reference simulator's golden log (tests/golden/pipeline,
written by oracle/gen_golden.py from src/access_simulator.py) and against the
build's host tokeniser (compute_features.load_access_log + encode)."""
import os

import numpy as np
import pandas as pd

from conftest import GOLDEN
from oracle import features_oracle as fo

PDIR = os.path.join(GOLDEN, "pipeline")


def test_iso_to_us_matches_pandas_on_golden_log():
    with open(os.path.join(PDIR, "access.log"), newline="") as fh:
        ts = [line.split(",")[0] for line in fh if line.strip()]
    exp = pd.to_datetime(pd.Series(ts), format="ISO8601", utc=True).astype("int64") // 1000
    got = np.array([fo.iso_to_us(s) for s in ts], dtype=np.int64)
    np.testing.assert_array_equal(got, exp.to_numpy())


def test_encode_log_matches_host_tokeniser():
    import compute_features as cf

    paths, _, primary = cf.load_manifest(os.path.join(PDIR, "metadata.csv"))
    log = os.path.join(PDIR, "access.log")
    with open(log, "rb") as fh:
        f, o, c, t = fo.encode_log(fh.read(), paths, primary)
    hf, ho, hc, ht, prim = cf.encode(paths, primary, *cf.load_access_log(log))
    np.testing.assert_array_equal(f, hf)
    np.testing.assert_array_equal(o, ho)
    np.testing.assert_array_equal(t, ht)
    n_prim = int(prim.max()) + 1
    np.testing.assert_array_equal(c, np.where(hc >= n_prim, -3, hc))


def test_iso_to_us_agrees_with_host_parser_on_edge_strings():
    import compute_features as cf

    cases = ["2025-11-01T12:00:00.165Z", "0000-02-29", "2023-02-29", "2024-02-29T23:59:59.5+01",
             " 2025-1-2T3:4 ", "2025-11-01T24:00:00", "2025-11-01T12:00:00.1234567890",
             "2025-11-01 12", "2025-11-01T12:00:00+05:3", "2025-11-01T12:00:00 Z", "x", "",
             "2025-11-01\t", "9999-12-31T23:59:59.999999-23:59", "2025-11-01T1:2:3-0800"]
    for s in cases:
        assert fo.iso_to_us(s) == cf.parse_ts_us(s), s
