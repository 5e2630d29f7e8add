"""Per-cluster replica scoring (drop-in for the reference's ``src/scoring.py``).

The reference ``ClusterClassifier`` (src/scoring.py:3-130) maps every cluster
to a replication category in two steps:

1. ``compute_cluster_medians`` — ``np.median`` of every feature list of every
   cluster (src/scoring.py:40-55).  This is the only part that scales with the
   number of files, and here it runs on the GPU: all lists are packed into one
   segmented float64 array and libcdr's segmented radix select returns every
   median in one launch (``cdr_medians_segmented``).  NumPy semantics are
   kept: the mean of the middle one/two order statistics summed from +0.0,
   NaN for an empty list (with NumPy's two RuntimeWarnings) or for any NaN.
2. Category scores (src/scoring.py:57-109) — k x 4 x d scalar operations on
   Python floats; they stay on the host and are evaluated in the reference's
   order, term by term, so the float results are identical.

Extension: ``classify_labels`` scores clusters straight from
the labels a ``kmeans_plusplus.kmeans`` call left on the device, without the
O(k*n) list building of src/main.py:96-102.

The reference also runs a demo at import time (src/scoring.py:133-174).  A
module import here does no device work; the same demo is ``demo()`` /
``python scoring.py``.
"""
from __future__ import annotations

import warnings

import numpy as np

from _cdr import Context, default_context

CATEGORIES = ("Hot", "Shared", "Moderate", "Archival")

__all__ = ["ClusterClassifier", "CATEGORIES", "demo"]


def _warn_empty_median() -> None:
    warnings.warn("Mean of empty slice.", RuntimeWarning, stacklevel=4)
    warnings.warn("invalid value encountered in scalar divide", RuntimeWarning, stacklevel=4)


class ClusterClassifier:
    """Weighted-deviation category assignment of clusters.

    global_medians      {feature: median over all files}
    weights             {category: {feature: weight}}
    directions          {category: {feature: +1 | -1 | 0}}
    replication_factors {category: factor}, tie-break: larger factor wins
    """

    def __init__(self, global_medians, weights, directions, replication_factors,
                 *, context: Context | None = None):
        self.global_medians = global_medians
        self.weights = weights
        self.directions = directions
        self.replication_factors = replication_factors
        self._context = context

    def _ctx(self) -> Context:
        return self._context if self._context is not None else default_context()

    def f(self, x):
        """Deviation weighting: x squared (src/scoring.py:28-38)."""
        return x ** 2

    # -- medians (GPU) ---------------------------------------------------
    def compute_cluster_medians(self, clusters):
        """{cluster: {feature: list}} -> {cluster: {feature: np.float64 median}}."""
        order = []
        chunks = []
        sizes = []
        for cname, features in clusters.items():
            for feature, values in features.items():
                # np.median's own conversion: asanyarray, then float64 math
                arr = np.asanyarray(values).ravel().astype(np.float64)
                order.append((cname, feature))
                chunks.append(arr)
                sizes.append(arr.size)
        offsets = np.zeros(len(sizes) + 1, dtype=np.int64)
        np.cumsum(sizes, out=offsets[1:])
        flat = np.concatenate(chunks) if chunks else np.empty(0, dtype=np.float64)
        med = self._ctx().medians_segmented(flat, offsets) if order else np.empty(0)
        result = {cname: {} for cname in clusters}
        for (cname, feature), size, value in zip(order, sizes, med):
            if size == 0:
                _warn_empty_median()
            result[cname][feature] = np.float64(value)
        return result

    # -- scoring (host, reference float order) ---------------------------
    def score_category(self, cluster_medians, category):
        """Score of one cluster for one category (src/scoring.py:57-84)."""
        total = 0
        w = self.weights[category]
        dirs = self.directions[category]
        for feature, median_value in cluster_medians.items():
            dev = median_value - self.global_medians[feature]
            want = dirs[feature]
            if category == "Moderate":
                if abs(dev) < 0.1:  # small deviations are rewarded
                    total += w[feature] * self.f(1 - abs(dev))
                continue
            if want == 0 or np.sign(dev) == want:
                total += w[feature] * self.f(abs(dev))
        return total

    def classify_cluster(self, cluster_medians):
        """Best category; exact-equality ties go to the largest factor."""
        scores = {cat: self.score_category(cluster_medians, cat) for cat in CATEGORIES}
        best = max(scores.values())
        leaders = [cat for cat, s in scores.items() if s == best]
        if len(leaders) > 1:
            # stable: among equal factors the earlier category stays first
            leaders.sort(key=lambda cat: self.replication_factors[cat], reverse=True)
            return leaders[0]
        return max(scores, key=scores.get)

    def classify(self, clusters):
        """{cluster: {feature: list}} -> {cluster: category}."""
        medians = self.compute_cluster_medians(clusters)
        return {cname: self.classify_cluster(m) for cname, m in medians.items()}

    # -- array-native extension ------------------------------------------
    def classify_labels(self, k, feature_names, *, prefix="C", context: Context | None = None,
                        comm=None):
        """Classify clusters 0..k-1 from the labels of the last Lloyd step on
        ``context`` (default: the process context ``kmeans`` used).  Same
        result as building ``{f"C{i}": {feature: list}}`` as src/main.py:96-102
        does and calling ``classify``; medians are computed on the device.
        With ``comm`` (cdr_dist.Comm over several ranks, each holding a shard
        of the points) the medians are those of the whole point set
        (cdr_dist.sharded_medians)."""
        ctx = context if context is not None else self._ctx()
        if comm is not None and comm.world > 1:
            from cdr_dist import sharded_medians

            med = sharded_medians(ctx, comm, int(k))
        else:
            med = ctx.medians_by_label(int(k))
        return self.classify_medians(med, feature_names, prefix=prefix)

    def classify_medians(self, med, feature_names, *, prefix="C"):
        """{prefix + j: category} from a (k, d) array of cluster medians.

        Vectorised over the clusters with the reference's float order kept:
        each category's total is accumulated feature by feature exactly as
        score_category does (a skipped term leaves the total unchanged), and
        ties go to the larger factor, then the earlier category.  Clusters
        with a NaN median take the per-cluster path (Python's max over NaN
        scores depends on order)."""
        med = np.asarray(med, dtype=np.float64)
        if med.shape[1] != len(feature_names):
            raise ValueError("feature_names must name every column of X")
        k = med.shape[0]
        bad = np.isnan(med).any(axis=1)
        scores = np.zeros((k, len(CATEGORIES)))
        for ci, cat in enumerate(CATEGORIES):
            w, dirs = self.weights[cat], self.directions[cat]
            total = np.zeros(k)
            for i, name in enumerate(feature_names):
                dev = med[:, i] - self.global_medians[name]
                if cat == "Moderate":
                    add = np.abs(dev) < 0.1
                    term = w[name] * self.f(1 - np.abs(dev))
                else:
                    want = dirs[name]
                    add = (want == 0) | (np.sign(dev) == want)
                    term = w[name] * self.f(np.abs(dev))
                total = np.where(add, total + term, total)
            scores[:, ci] = total
        best = scores.max(axis=1)
        factors = np.array([self.replication_factors[c] for c in CATEGORIES])
        order = sorted(range(len(CATEGORIES)), key=lambda c: -factors[c])  # stable
        out = {}
        for j in range(k):
            if bad[j]:
                cm = {name: np.float64(med[j, i]) for i, name in enumerate(feature_names)}
                _warn_empty_median()
                out[f"{prefix}{j}"] = self.classify_cluster(cm)
                continue
            leaders = scores[j] == best[j]
            if leaders.sum() > 1:
                out[f"{prefix}{j}"] = CATEGORIES[next(c for c in order if leaders[c])]
            else:
                out[f"{prefix}{j}"] = CATEGORIES[int(np.argmax(scores[j]))]
        return out


def demo(context: Context | None = None):
    """The reference's import-time example (src/scoring.py:137-174)."""
    clusters = {
        "C1": {"IOPS": [100, 110, 105], "Latency": [2, 3, 2.5]},
        "C2": {"IOPS": [50, 55, 60], "Latency": [5, 6, 5.5]},
        "C3": {"IOPS": [10, 12, 11], "Latency": [8, 9, 7]},
        "C4": {"IOPS": [200, 210, 220], "Latency": [1, 1.5, 1.2]},
    }
    medians = {"IOPS": 60, "Latency": 4}
    weights = {"Hot": {"IOPS": 1.0, "Latency": 0.8}, "Shared": {"IOPS": 0.7, "Latency": 0.7},
               "Moderate": {"IOPS": 0.5, "Latency": 0.5},
               "Archival": {"IOPS": 0.9, "Latency": 1.0}}
    directions = {"Hot": {"IOPS": +1, "Latency": -1}, "Shared": {"IOPS": +1, "Latency": +1},
                  "Moderate": {"IOPS": 0, "Latency": 0},
                  "Archival": {"IOPS": -1, "Latency": +1}}
    factors = {"Hot": 3, "Shared": 2, "Moderate": 1, "Archival": 4}
    clf = ClusterClassifier(medians, weights, directions, factors, context=context)
    results = clf.classify(clusters)
    print("Final Category Assignments:")
    for name, cat in results.items():
        print(name, "→", cat)
    return results


if __name__ == "__main__":
    demo()
