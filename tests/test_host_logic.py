"""Host-side plumbing of the drop-in modules (no device calls)."""
import json
import math
import os
import random

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN


def test_java_double_layout():
    from compute_features import java_double

    cases = [(0.0, "0.0"), (-0.0, "-0.0"), (1.0, "1.0"), (0.5, "0.5"), (100.0, "100.0"),
             (1e7, "1.0E7"), (12277768.082999945, "1.2277768082999945E7"), (1e-3, "0.001"),
             (9.99e-4, "9.99E-4"), (1e-5, "1.0E-5"), (123.456, "123.456"),
             (9999999.5, "9999999.5"), (0.1 + 0.2, "0.30000000000000004"),
             (-2.5e-7, "-2.5E-7"), (1e300, "1.0E300"), (float("nan"), "NaN"),
             (float("inf"), "Infinity"), (float("-inf"), "-Infinity"),
             (5e-324, "4.9E-324"), (1e-323, "9.9E-324"), (1.7976931348623157e308, "1.7976931348623157E308"),
             (1.0 / 3, "0.3333333333333333"), (2.0 / 3, "0.6666666666666666"),
             (123456789.0, "1.23456789E8"), (1e21, "1.0E21"), (0.001, "0.001"),
             (1234567.0, "1234567.0")]
    for v, s in cases:
        assert java_double(v) == s, (v, java_double(v))
    rng = random.Random(1)
    for _ in range(2000):
        v = rng.uniform(-1, 1) * 10 ** rng.randint(-12, 12)
        assert float(java_double(v).replace("E", "e")) == v


def test_java_double_legacy_pre_jdk19_digits():
    """apache/spark:3.5.2 (docker/docker-compose.yml:67) runs a pre-19 JDK, whose
    Double.toString is not always shortest.  Pinned by the outputs JDK bug 4511638
    lists for JDK <= 18, and by hand derivations of the integer path."""
    from compute_features import java_double, java_double_legacy

    pinned = [(2.82879384806159e17, "2.82879384806159008E17"),
              (1.387364135037754e18, "1.38736413503775411E18"),
              (1.45800632428665e17, "1.45800632428664992E17"),
              (5.684341886080802e-14, "5.6843418860808015E-14"),
              (8.41e21, "8.409999999999999E21"),
              (1.9400994884341945e25, "1.9400994884341944E25"),
              (2e23, "1.9999999999999998E23"),
              # integers below 2^63 keep their digits down to 10^i, i + 1 = the digit
              # count of 2^(binExp - 54), rounded half up: 2^60 = 1152921504606846976,
              # 2^6 = 64 -> drop one digit -> ...697|6 -> ...698
              (2.0 ** 60, "1.15292150460684698E18"),
              (2.0 ** 62, "4.6116860184273879E18"),  # 2^8 = 256 -> drop two digits: ...879|04 -> ...879
              (2.0 ** 63, "9.223372036854776E18"),  # binExp 63 > 62: digit generation
              (2.0 ** 53, "9.007199254740992E15"),
              (5e-324, "4.9E-324"), (1.7976931348623157e308, "1.7976931348623157E308")]
    for v, s in pinned:
        assert java_double_legacy(v) == s, (v, java_double_legacy(v))
        assert java_double_legacy(-v) == "-" + s
    # the layout is the same as JDK 19+ wherever the digits agree
    for v, s in [(0.0, "0.0"), (-0.0, "-0.0"), (1.0, "1.0"), (0.5, "0.5"), (100.0, "100.0"),
                 (1e7, "1.0E7"), (1e-3, "0.001"), (9.99e-4, "9.99E-4"), (1e-5, "1.0E-5"),
                 (9999999.5, "9999999.5"), (0.1 + 0.2, "0.30000000000000004"), (-2.5e-7, "-2.5E-7"),
                 (float("nan"), "NaN"), (float("inf"), "Infinity"), (float("-inf"), "-Infinity"),
                 (1.0 / 3, "0.3333333333333333"), (123456789.0, "1.23456789E8"),
                 (1234567.0, "1234567.0"), (12277768.082999945, "1.2277768082999945E7")]:
        assert java_double_legacy(v) == s, (v, java_double_legacy(v))
    # every output reads back as the same double, and is never shorter than the
    # shortest digits; both formats agree on most values
    rng = random.Random(7)
    same = 0
    for _ in range(4000):
        v = rng.uniform(-1, 1) * 10 ** rng.randint(-30, 30)
        if rng.random() < 0.2:
            v = float(rng.getrandbits(rng.randint(1, 63)))
        a, b = java_double_legacy(v), java_double(v)
        assert float(a.replace("E", "e")) == v, (v, a)
        assert len(a.lstrip("-").split("E")[0]) >= len(b.lstrip("-").split("E")[0]), (v, a, b)
        same += a == b
    assert same > 3000


def test_spark_csv_double_format_switch(tmp_path, monkeypatch):
    from compute_features import write_spark_csv

    table = np.full((1, 10), 2e23)
    monkeypatch.delenv("CDR_JAVA_DOUBLE", raising=False)
    with open(write_spark_csv(str(tmp_path / "a"), ["/p"], table)) as fh:
        assert "1.9999999999999998E23" in fh.read()
    monkeypatch.setenv("CDR_JAVA_DOUBLE", "19")
    with open(write_spark_csv(str(tmp_path / "b"), ["/p"], table)) as fh:
        assert "2.0E23" in fh.read()
    monkeypatch.setenv("CDR_JAVA_DOUBLE", "17")
    with pytest.raises(ValueError):
        write_spark_csv(str(tmp_path / "c"), ["/p"], table)


def test_iso_timestamp_parsing_matches_pandas():
    from compute_features import parse_ts_us

    samples = ["2025-06-12T09:40:32.335400Z", "2025-11-01T12:00:00.165Z", "1969-12-31T23:59:59.5Z",
               "2024-02-29T00:00:00Z", "2025-01-25T17:05:23.323092Z", "2025-03-01T01:02:03+02:00"]
    for s in samples:
        exp = pd.Timestamp(s).tz_convert("UTC") if pd.Timestamp(s).tzinfo else pd.Timestamp(s, tz="UTC")
        assert parse_ts_us(s) == exp.value // 1000, s
    assert parse_ts_us("not a time") is None
    assert parse_ts_us("2025-02-30T00:00:00Z") is None


def test_encode_dictionary():
    from compute_features import encode

    paths = ["/a", "/b", "/c"]
    prim = ["dn1", None, "dn2"]
    f, op, cl, ts, pr = encode(paths, prim, ["2025-01-01T00:00:00.001Z"] * 4,
                               ["/a", "/zzz", "/c", None], ["WRITE", "READ", "read", None],
                               ["dn1", "dn2", None, "dn2"])
    assert list(f) == [0, -1, 2, -1]
    assert list(op) == [1, 2, 0, 0]
    assert cl[2] == -1 and pr[1] == -2
    assert cl[0] == pr[0] and cl[3] == pr[2]


def test_pipeline_features_csv_roundtrip(tmp_path):
    from compute_features import OUT_COLUMNS, write_spark_csv

    pdir = os.path.join(GOLDEN, "pipeline")
    z = np.load(os.path.join(pdir, "features_oracle.npz"))
    df = pd.read_csv(os.path.join(pdir, "features_out", "part-00000-golden-c000.csv"),
                     float_precision="round_trip")
    assert list(df.columns) == OUT_COLUMNS
    np.testing.assert_array_equal(df[OUT_COLUMNS[1:]].to_numpy(dtype=np.float64), z["table"])
    part = write_spark_csv(str(tmp_path / "out"), list(df["path"]), z["table"])
    assert os.path.basename(part).startswith("part-00000")
    assert os.path.exists(str(tmp_path / "out" / "_SUCCESS"))
    with open(part) as a, open(os.path.join(pdir, "features_out", "part-00000-golden-c000.csv")) as b:
        assert a.read() == b.read()  # pre-JDK-19 digits; none of these values differ
    back = pd.read_csv(part, float_precision="round_trip")
    np.testing.assert_array_equal(back[OUT_COLUMNS[1:]].to_numpy(dtype=np.float64), z["table"])


def test_scoring_host_logic_matches_reference_scores():
    from scoring import ClusterClassifier

    with open(os.path.join(GOLDEN, "scoring_cases.json")) as fh:
        cases = json.load(fh)
    for c in cases:
        s = c["spec"]
        clf = ClusterClassifier(s["global_medians"], s["weights"], s["directions"],
                                s["replication_factors"])
        for cname, med in c["medians"].items():
            med = {p: np.float64(v) for p, v in med.items()}
            for cat, val in c["scores"][cname].items():
                got = clf.score_category(med, cat)
                assert (math.isnan(got) and math.isnan(val)) or got == val
            assert clf.classify_cluster(med) == c["result"][cname]


def test_kmeans_keeps_reference_max_iter_formula():
    import inspect
    import kmeans_plusplus

    sig = inspect.signature(kmeans_plusplus.kmeans)
    assert list(sig.parameters)[:5] == ["X", "k", "number_of_files", "tol", "random_state"]
    assert sig.parameters["number_of_files"].default == 100
    assert sig.parameters["tol"].default == 1e-4
    assert sig.parameters["max_iter"].kind is inspect.Parameter.KEYWORD_ONLY
    with pytest.raises(TypeError, match="cannot be interpreted as an integer"):
        range(max(100, 10001 / 100))


def test_classify_medians_vectorised_equals_per_cluster():
    """classify_medians (vectorised over clusters) = classify_cluster on each
    row: random medians, exact score ties (zero deviations, equal factors) and
    NaN rows."""
    import warnings

    from scoring import CATEGORIES, ClusterClassifier

    rng = np.random.default_rng(0)
    names = [f"f{i}" for i in range(7)]
    for trial in range(4):
        gm = {nm: float(rng.random()) for nm in names}
        w = {c: {nm: float(rng.choice([0.0, 0.5, 1.0, rng.random()])) for nm in names}
             for c in CATEGORIES}
        dirs = {c: {nm: int(rng.integers(-1, 2)) for nm in names} for c in CATEGORIES}
        rf = {c: int(rng.integers(1, 3)) for c in CATEGORIES}
        clf = ClusterClassifier(gm, w, dirs, rf)
        med = rng.random((500, 7))
        med[:50] = [gm[nm] for nm in names]            # zero deviation: ties
        med[50:60, 2] = gm["f2"] + 0.05                 # Moderate band
        med[60:63, 4] = np.nan
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            got = clf.classify_medians(med, names)
            exp = {f"C{j}": clf.classify_cluster({nm: np.float64(med[j, i])
                                                  for i, nm in enumerate(names)})
                   for j in range(500)}
        assert got == exp, trial
