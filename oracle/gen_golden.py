"""Write tests/golden/* by running the REFERENCE itself (run in the build
container, where /root/reference exists; the GPU box only reads the fixtures).

    python oracle/gen_golden.py

Nothing from the reference is copied into the repo except data: inputs and
expected outputs (plus src/metadata.csv, the reference's own data fixture).
The reference is imported read-only (sys.dont_write_bytecode, no files
written under /root/reference).
"""
from __future__ import annotations

import contextlib
import datetime as _dt
import importlib.util
import io
import json
import os
import random
import shutil
import subprocess
import sys
import warnings

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from oracle import synth  # noqa: E402
from oracle import features_oracle  # noqa: E402


def load_ref(name):
    spec = importlib.util.spec_from_file_location(f"ref_{name}", os.path.join(REF, f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    with contextlib.redirect_stdout(io.StringIO()):
        spec.loader.exec_module(mod)
    return mod


def kmeans_cases():
    ref = load_ref("kmeans_plusplus")
    rng = np.random.default_rng(20261015)
    cases = []

    def add(name, X, k, rs, np_seed, store_x=True, gen=None, seed_only=False):
        np.random.seed(np_seed)
        init = ref.kmeans_plusplus_init(X, k, random_state=rs)
        entry = {"name": name, "k": k, "rs": rs, "np_seed": np_seed, "init": init,
                 "seed_only": seed_only}
        if not seed_only:
            np.random.seed(np_seed)
            C, labels = ref.kmeans(X, k, number_of_files=X.shape[0], random_state=rs)
            entry.update(centroids=C, labels=labels)
        if store_x:
            entry["X"] = X
        else:
            entry["gen"] = gen
        cases.append(entry)

    g = (3000, 0, 3000, 8, 16, 7)
    add("grid24_d8_k16", synth.generate(*g), 16, 42, 0, store_x=False, gen=g)
    g = (5000, 0, 5000, 16, 64, 11)
    add("grid24_d16_k64", synth.generate(*g), 64, 42, 1, store_x=False, gen=g)
    g = (4000, 1000, 4000, 5, 4, 3)
    add("grid24_d5_k4_offset", synth.generate(*g), 4, 7, 2, store_x=False, gen=g)
    add("float_d5_k4", rng.random((2000, 5)), 4, 42, 3)
    add("float_d1_k3", rng.random((1500, 1)) ** 2, 3, 5, 4)
    add("float_d9_k5", rng.normal(0.0, 100.0, (1200, 9)), 5, 9, 5)
    add("float_d17_k6", rng.random((900, 17)), 6, 11, 6)
    add("ties_grid_d3_k8", rng.integers(0, 4, (2000, 3)) / 4.0, 8, 42, 7)
    add("ties_float_d2_k5", np.repeat(rng.random((40, 2)), 25, axis=0), 5, 3, 8)
    # seeding across several 8192-element blocks (n > 10000: seeding only)
    g = (20000, 0, 20000, 4, 16, 5)
    add("seed_grid_n20000_d4_k16", synth.generate(*g), 16, 42, 9, store_x=False, gen=g,
        seed_only=True)
    add("seed_float_n100003_d2_k6", rng.random((100003, 2)), 6, 1, 10, seed_only=True)
    # error case: fewer distinct points than k -> NaN probabilities
    Xdup = np.repeat(rng.random((3, 2)), 4, axis=0)
    try:
        ref.kmeans_plusplus_init(Xdup, 5, random_state=0)
        err = None
    except ValueError as e:
        err = str(e)
    cases.append({"name": "error_nan_probs", "k": 5, "rs": 0, "np_seed": 0, "X": Xdup,
                  "error": err, "seed_only": True})
    # reference behaviour for n > 10000 in kmeans(): TypeError
    try:
        ref.kmeans(np.zeros((10001, 2)) + np.arange(10001)[:, None], 2, number_of_files=10001)
        terr = None
    except TypeError as e:
        terr = str(e)
    return cases, terr


def save_kmeans(cases, terr):
    arrays = {}
    meta = []
    for i, c in enumerate(cases):
        m = {key: c[key] for key in ("name", "k", "rs", "np_seed", "seed_only") if key in c}
        if "error" in c:
            m["error"] = c["error"]
        if "gen" in c:
            m["gen"] = list(c["gen"])
        for key in ("X", "init", "centroids", "labels"):
            if key in c:
                arrays[f"c{i}_{key}"] = c[key]
        meta.append(m)
    np.savez_compressed(os.path.join(GOLD, "kmeans_cases.npz"), **arrays)
    with open(os.path.join(GOLD, "kmeans_cases.json"), "w") as fh:
        json.dump({"cases": meta, "n_gt_10000_error": terr}, fh, indent=1)


def scoring_cases():
    sc = load_ref("scoring")
    out = []
    demo = dict(clusters=sc.clusters, global_medians=sc.global_medians, weights=sc.weights,
                directions=sc.directions, replication_factors=sc.replication_factors)
    rng = np.random.default_rng(7)

    def run(name, spec):
        clf = sc.ClusterClassifier(spec["global_medians"], spec["weights"], spec["directions"],
                                   spec["replication_factors"])
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            med = clf.compute_cluster_medians(spec["clusters"])
            res = clf.classify(spec["clusters"])
        scores = {c: {cat: float(clf.score_category(m, cat))
                      for cat in ("Hot", "Shared", "Moderate", "Archival")}
                  for c, m in med.items()}
        medf = {c: {p: float(v) for p, v in m.items()} for c, m in med.items()}
        out.append({"name": name, "spec": spec, "medians": medf, "scores": scores,
                    "result": res})

    run("demo", demo)
    feats = ["a", "b", "c", "d", "e"]
    cats = ("Hot", "Shared", "Moderate", "Archival")
    for t in range(6):
        clusters = {}
        for j in range(6):
            clusters[f"C{j}"] = {f: [float(v) for v in rng.random(int(rng.integers(1, 40)))]
                                 for f in feats}
        if t == 1:
            clusters["C5"] = {f: [] for f in feats}  # empty cluster -> NaN medians
        if t == 2:
            clusters["C4"] = {f: [0.5] * 3 for f in feats}  # equal to global medians
        if t == 3:
            clusters["C3"] = {f: [int(x) for x in rng.integers(0, 10, 7)] for f in feats}
        spec = dict(clusters=clusters, global_medians={f: 0.5 for f in feats},
                    weights={c: {f: float(np.round(rng.random(), 2)) for f in feats} for c in cats},
                    directions={c: {f: int(rng.integers(-1, 2)) if c != "Moderate" else 0
                                    for f in feats} for c in cats},
                    replication_factors={"Hot": 3, "Shared": 2, "Moderate": 1, "Archival": 4})
        run(f"random_{t}", spec)
    with open(os.path.join(GOLD, "scoring_cases.json"), "w") as fh:
        json.dump(out, fh, indent=1)


class _FrozenDT(_dt.datetime):
    @classmethod
    def utcnow(cls):
        return cls(2025, 11, 1, 12, 0, 0, 123000)


def pipeline_case():
    pdir = os.path.join(GOLD, "pipeline")
    os.makedirs(pdir, exist_ok=True)
    shutil.copyfile(os.path.join(REF, "metadata.csv"), os.path.join(pdir, "metadata.csv"))
    sim = load_ref("access_simulator")
    sim.datetime = _FrozenDT
    random.seed(0)
    manifest = sim.load_manifest(os.path.join(pdir, "metadata.csv"))
    with contextlib.redirect_stdout(io.StringIO()):
        sim.generate_all(manifest, os.path.join(pdir, "access.log"), 600, ["dn1", "dn2", "dn3"])
    # features: pandas restatement (Spark absent) -> the main.py input fixture
    paths, table, counts, obs_end = features_oracle.compute(
        os.path.join(pdir, "metadata.csv"), os.path.join(pdir, "access.log"))
    sys.path.insert(0, os.path.join(REPO, "clustering-driven-replication-strategy_amd"))
    from compute_features import write_spark_csv  # formatting helper only (no device work)
    fdir = os.path.join(pdir, "features_out")
    part = write_spark_csv(fdir, paths, table)
    os.rename(part, os.path.join(fdir, "part-00000-golden-c000.csv"))
    np.savez_compressed(os.path.join(pdir, "features_oracle.npz"), table=table, counts=counts,
                        obs_end=np.float64(obs_end))
    # reference main.py on that CSV
    out_csv = os.path.join(pdir, "final_categories.csv")
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-B", os.path.join(REF, "main.py"), "--input_path", fdir,
                        "--k", "4", "--output_csv", out_csv], cwd=REF, env=env,
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(r.stderr)
    with open(os.path.join(pdir, "main_stdout.txt"), "w") as fh:
        fh.write(r.stdout)
    main_mod = importlib.util.spec_from_file_location("ref_main", os.path.join(REF, "main.py"))
    mm = importlib.util.module_from_spec(main_mod)
    saved = sys.path[:]
    sys.path.insert(0, REF)
    with contextlib.redirect_stdout(io.StringIO()):
        main_mod.loader.exec_module(mm)
    sys.path[:] = saved
    tables = {"CLUSTERING_FEATURES": mm.CLUSTERING_FEATURES, "GLOBAL_MEDIANS": mm.GLOBAL_MEDIANS,
              "WEIGHTS": mm.WEIGHTS, "DIRECTIONS": mm.DIRECTIONS,
              "REPLICATION_FACTORS": mm.REPLICATION_FACTORS}
    with open(os.path.join(pdir, "main_tables.json"), "w") as fh:
        json.dump(tables, fh, indent=1)
    # the kmeans result main.py computed (same call as src/main.py:91)
    import pandas as pd
    ref = load_ref("kmeans_plusplus")
    df = pd.read_csv(os.path.join(fdir, "part-00000-golden-c000.csv"))
    X = df[mm.CLUSTERING_FEATURES].values
    C, labels = ref.kmeans(X, 4, number_of_files=len(df), random_state=42)
    np.savez_compressed(os.path.join(pdir, "main_kmeans.npz"), centroids=C, labels=labels)


def float32_cases():
    """The reference on float32 X: its centroids have X's
    dtype (kmeans_plusplus.py:6, :37), so seeding distances, probabilities and
    means are computed in float32.  The same data as float64 for contrast.
    tests/test_float32_input.py pins the drop-in's float32 semantics (fp64
    distances, exact means rounded to float32) against these runs: seeds and
    labels equal, centroids within the north_star's 1e-5 relative."""
    ref = load_ref("kmeans_plusplus")
    out = {}
    for i, (n, d, k, seed, rs) in enumerate([(3000, 5, 4, 11, 42), (4000, 8, 16, 12, 7),
                                              (2500, 16, 8, 13, 3)]):
        X = synth.generate(n, 0, n, d, k, seed).astype(np.float32)
        for tag, Xc in (("f32", X), ("f64", X.astype(np.float64))):
            np.random.seed(i)
            init = ref.kmeans_plusplus_init(Xc, k, random_state=rs)
            np.random.seed(i)
            C, labels = ref.kmeans(Xc, k, number_of_files=n, random_state=rs)
            out[f"c{i}_{tag}_init"] = init
            out[f"c{i}_{tag}_centroids"] = C
            out[f"c{i}_{tag}_labels"] = labels
        out[f"c{i}_X"] = X
        out[f"c{i}_meta"] = np.array([n, d, k, seed, rs, i], dtype=np.int64)
    np.savez_compressed(os.path.join(GOLD, "kmeans_f32_cases.npz"), **out)


F32_HARD = [  # name, n, d, k, rs, np_seed, transform
    ("big", 2_400_000, 2, 2, 5, 21, "synth"),       # two ~1.2M-point clusters
    ("coarse", 6000, 3, 12, 9, 22, "grid8"),        # values on a 2^-8 grid: ties
    ("near", 5000, 4, 10, 4, 23, "near20"),         # offsets of 2^-20 around 0.5
]


def float32_hard_cases():
    """The reference on float32 X where its float32 arithmetic matters
    (VERDICT r3 item 6): a ~1.2M-point cluster (sequential fp32 mean drift),
    data on a coarse grid (exact distance ties) and offsets of 2^-20 around
    0.5 (fp32 norms tie where fp64 norms do not).  Stored: parameters, the
    float32 and float64 runs' seeds and centroids, labels bit-packed (k = 2,
    np.packbits) or as uint8, and whether the two runs differ."""
    ref = load_ref("kmeans_plusplus")
    out = {}
    for i, (name, n, d, k, rs, nps, tr) in enumerate(F32_HARD):
        X = synth.f32_hard_data(n, d, k, tr, 1000 + i)
        runs = {}
        for tag, Xc in (("f32", X), ("f64", X.astype(np.float64))):
            np.random.seed(nps)
            init = ref.kmeans_plusplus_init(Xc, k, random_state=rs)
            np.random.seed(nps)
            C, labels = ref.kmeans(Xc, k, number_of_files=100, random_state=rs)
            runs[tag] = (init, C, labels)
            out[f"h{i}_{tag}_init"] = init
            out[f"h{i}_{tag}_centroids"] = C
            if tag == "f32":  # (the float64 run's labels: only whether they differ)
                out[f"h{i}_{tag}_labels"] = (np.packbits(labels.astype(np.uint8)) if k == 2
                                             else labels.astype(np.uint8))
        diff = [int(not np.array_equal(runs["f32"][0].astype(np.float64), runs["f64"][0])),
                int(not np.array_equal(runs["f32"][2], runs["f64"][2])),
                int(np.abs(runs["f32"][1].astype(np.float64) - runs["f64"][1]).max() /
                    np.abs(runs["f64"][1]).max() > 2.0 ** -22)]
        print(name, "f32 vs f64 differ (init, labels, centroids):", diff,
              "max rel", np.abs(runs["f32"][1].astype(np.float64) - runs["f64"][1]).max() /
              np.abs(runs["f64"][1]).max())
        out[f"h{i}_meta"] = np.array([n, d, k, rs, nps, 1000 + i] + diff, dtype=np.int64)
        out[f"h{i}_name"] = np.array(name + ":" + tr)
    np.savez_compressed(os.path.join(GOLD, "kmeans_f32_hard.npz"), **out)


def main():
    os.makedirs(GOLD, exist_ok=True)
    if "--only-f32" in sys.argv:
        float32_cases()
        float32_hard_cases()
        return
    float32_cases()
    float32_hard_cases()
    cases, terr = kmeans_cases()
    save_kmeans(cases, terr)
    scoring_cases()
    pipeline_case()
    print("golden fixtures written to", GOLD)


if __name__ == "__main__":
    main()
