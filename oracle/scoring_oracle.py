"""Scoring oracle (TEST INFRASTRUCTURE ONLY).

np.median per (cluster, feature) list — the reference's own call at
/root/reference/src/scoring.py:53 — and the category scorer of
src/scoring.py:57-109 restated as plain functions.
"""
from __future__ import annotations

import warnings

import numpy as np

CATEGORIES = ("Hot", "Shared", "Moderate", "Archival")


def cluster_medians(clusters):
    out = {}
    for cname, feats in clusters.items():
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            out[cname] = {p: np.median(v) for p, v in feats.items()}
    return out


def score(medians, gm, weights, directions, category):
    s = 0
    for p, m in medians.items():
        delta = m - gm[p]
        want = directions[category][p]
        if category == "Moderate":
            if abs(delta) < 0.1:
                s += weights[category][p] * (1 - abs(delta)) ** 2
        elif want == 0 or np.sign(delta) == want:
            s += weights[category][p] * abs(delta) ** 2
    return s


def classify(clusters, gm, weights, directions, factors):
    res = {}
    for cname, med in cluster_medians(clusters).items():
        scores = {c: score(med, gm, weights, directions, c) for c in CATEGORIES}
        best = max(scores.values())
        tied = [c for c, v in scores.items() if v == best]
        if len(tied) > 1:
            tied.sort(key=lambda c: factors[c], reverse=True)
            res[cname] = tied[0]
        else:
            res[cname] = max(scores, key=scores.get)
    return res
