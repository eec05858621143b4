"""Helpers for the dataset-histogram tests: golden fixtures (made by the
reference, oracle/gen_golden_hist.py) and bin comparison."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "histograms")


def _load(pattern, prefix):
    out = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, pattern))):
        with open(path) as f:
            d = json.load(f)
        d["name"] = os.path.basename(path)[len(prefix):-len(".json")]
        out.append(d)
    return out


def fixtures():
    """raw-row cases: rows (pid, pk, value)"""
    return [d for d in _load("dataset_histograms_*.json", "dataset_histograms_") if not d["name"].startswith("pre_")]


def pre_fixtures():
    """pre-aggregated cases: rows (pk, count, sum, n_partitions, n_contributions)"""
    return _load("dataset_histograms_pre_*.json", "dataset_histograms_pre_")


def pre_columns(rows):
    """dense pk codes + the four pre-aggregated columns"""
    pk = np.unique([str(r[0]) for r in rows], return_inverse=True)[1].astype(np.int64)
    a = np.asarray([r[1:] for r in rows], dtype=np.float64).reshape(-1, 4)
    return (pk, a[:, 0].astype(np.int64), a[:, 1], a[:, 2].astype(np.int64), a[:, 3].astype(np.int64))


def preaggregate(pid, pk, val):
    """(pk, count, sum, n_partitions, n_contributions) per (pid, pk) pair of
    raw dense-code columns (what analysis/pre_aggregation.py:19-58 emits)"""
    pid = np.asarray(pid, dtype=np.int64)
    pk = np.asarray(pk, dtype=np.int64)
    val = np.asarray(val, dtype=np.float64)
    pairs, inv = np.unique(np.stack([pid, pk], 1), axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    cnt = np.bincount(inv)
    tot = np.bincount(inv, weights=val)
    upid, pid_inv = np.unique(pairs[:, 0], return_inverse=True)
    n_part = np.bincount(pid_inv.reshape(-1))
    rows_of_pid = np.bincount(np.searchsorted(upid, pid))
    pi = pid_inv.reshape(-1)
    return pairs[:, 1].copy(), cnt.astype(np.int64), tot, n_part[pi].astype(np.int64), rows_of_pid[pi].astype(np.int64)


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


# Known answers from the reference's tests
# (tests/dataset_histograms/computing_histograms_test.py): (privacy_id,
# partition) rows -> the expected bins of one histogram.
KAT_L0 = [  # test_compute_l0_contributions_histogram
    ([(1, 1), (1, 2), (2, 1)], [(1, 2, 1, 1, 1), (2, 3, 1, 2, 2)]),
    ([(i, i) for i in range(100)], [(1, 2, 100, 100, 1)]),
    ([(0, 0)], [(1, 2, 1, 1, 1)]),
    ([(0, i) for i in range(1234)], [(1230, 1240, 1, 1234, 1234)]),
    ([(0, i) for i in range(15)] + [(1, i) for i in range(10, 25)], [(15, 16, 2, 30, 15)]),
]
KAT_L1 = [  # test_compute_l1_contributions_histogram
    ([(1, 1), (1, 2), (2, 1)], [(1, 2, 1, 1, 1), (2, 3, 1, 2, 2)]),
    ([(i, i) for i in range(100)], [(1, 2, 100, 100, 1)]),
    ([(0, 0)] * 100, [(100, 101, 1, 100, 100)]),
    ([(0, i // 2) for i in range(1235)], [(1230, 1240, 1, 1235, 1235)]),
    ([(0, i) for i in range(15)] + [(1, i) for i in range(10, 25)], [(15, 16, 2, 30, 15)]),
]


def kat_cases():
    return ([("l0_contributions_histogram", rows, exp) for rows, exp in KAT_L0] +
            [("l1_contributions_histogram", rows, exp) for rows, exp in KAT_L1])
