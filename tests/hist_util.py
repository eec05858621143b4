"""Helpers for the dataset-histogram tests: golden fixtures (made by the
reference, oracle/gen_golden_hist.py) and bin comparison."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "histograms")


def fixtures():
    out = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, "*.json"))):
        with open(path) as f:
            d = json.load(f)
        d["name"] = os.path.basename(path)[len("dataset_histograms_"):-len(".json")]
        out.append(d)
    return out


def codes(rows):
    """dense codes of the pid / pk columns (first-appearance order is
    irrelevant to the histograms)."""
    pid = np.unique([str(r[0]) for r in rows], return_inverse=True)[1].astype(np.int64)
    pk = np.unique([str(r[1]) for r in rows], return_inverse=True)[1].astype(np.int64)
    return pid, pk, np.asarray([r[2] for r in rows], dtype=np.float64)


def as_tuples(bins):
    return [(b.lower, b.upper, b.count, b.sum, b.max) if hasattr(b, "lower") else tuple(b) for b in bins]


FLOAT_FIELDS = ("linf_sum_contributions_histogram", "sum_per_partition_histogram")


def _close(a, b, rtol):
    return abs(a - b) <= rtol * max(1.0, abs(b))


def assert_bins_equal(got, want, what, rtol=1e-9, exact=False):
    """Integer histograms: every field exact.  Float histograms (`what` names
    a FLOAT_FIELDS field): counts exact; lower / upper / sum / max — all
    derived from fp64 value sums, which the reference adds in insertion order
    and the GPU in atomic order — within rtol, or exact when `exact` (dyadic
    values: every order gives the same sums)."""
    got, want = as_tuples(got), as_tuples(want)
    is_float = any(f in what for f in FLOAT_FIELDS)
    tol = 0.0 if exact else rtol
    assert len(got) == len(want), f"{what}: {len(got)} bins vs {len(want)}"
    for g, w in zip(got, want):
        assert g[2] == w[2], f"{what}: count {g} vs {w}"
        if is_float:
            for j in (0, 1, 3, 4):
                assert _close(g[j], w[j], tol), f"{what}: {g} vs {w}"
        else:
            assert g[0] == w[0] and g[1] == w[1] and g[4] == w[4], f"{what}: {g} vs {w}"
            assert _close(g[3], w[3], tol), f"{what}: sum {g} vs {w}"
