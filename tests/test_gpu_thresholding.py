"""PostAggregationThresholding end to end on the GPU.

The reference replaces the PRIVACY_ID_COUNT combiner by
PostAggregationThresholdingCombiner when post_aggregation_thresholding=True
(combiners.py:328-382, 892-895), skips private partition selection
(dp_engine.py:162) and drops the partitions whose thresholded value is None
(dp_engine.py:184-185, 544-549).  Pinned by fixtures the reference itself
produced (oracle/gen_golden.py post_threshold_fixture: huge epsilon, so the
kept set is deterministic) and by keep-rate tests of the Laplace / Gaussian
thresholding strategies at a moderate epsilon.
"""
import json
import math
import os

import numpy as np
import pytest

import pipelinedp_amd as pdp
from pipelinedp_amd import columnar_backend as CB
from pipelinedp_amd import dp_computations as dpc

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _engine(eps, delta, seed):
    backend = CB.ColumnarBackend(seed=seed)
    acc = pdp.NaiveBudgetAccountant(total_epsilon=eps, total_delta=delta)
    return pdp.DPEngine(acc, backend), acc


@pytest.mark.parametrize("kind", ["laplace", "gaussian"])
@pytest.mark.parametrize("columnar", [False, True])
def test_post_aggregation_thresholding_matches_reference_golden(device, kind, columnar):
    with open(os.path.join(GOLDEN, f"post_aggregation_thresholding_{kind}.json")) as f:
        fx = json.load(f)
    rows = [tuple(r) for r in fx["rows"]]
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.PRIVACY_ID_COUNT],
                                 noise_kind=getattr(pdp.NoiseKind, fx["noise_kind"]),
                                 max_partitions_contributed=fx["l0"], max_contributions_per_partition=fx["linf"],
                                 post_aggregation_thresholding=True)
    engine, acc = _engine(fx["eps"], fx["delta"], seed=31)
    if columnar:
        arr = np.asarray(rows, dtype=np.int64)
        src = pdp.ColumnTable({"pid": arr[:, 0], "pk": arr[:, 1], "v": arr[:, 2]})
        ext = pdp.DataExtractors(privacy_id_extractor=pdp.ColumnExtractor("pid"),
                                 partition_extractor=pdp.ColumnExtractor("pk"),
                                 value_extractor=pdp.ColumnExtractor("v"))
    else:
        src = rows
        ext = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                                 value_extractor=lambda r: r[2])
    sink = engine.aggregate(src, params, ext)
    acc.compute_budgets()
    # the budget requests equal the reference's (COUNT mechanism + thresholding)
    got_budgets = [[m.mechanism_spec.mechanism_type.value, m.mechanism_spec.eps, m.mechanism_spec.delta]
                   for m in acc._mechanisms]
    assert got_budgets == fx["budgets"]
    out = sorted((int(k), m) for k, m in sink)
    want = fx["expected"]
    assert [k for k, _ in out] == [k for k, _ in want]  # the same partitions kept / dropped
    for (k, m), (_, w) in zip(out, want):
        assert list(m._fields) == fx["field_order"]
        for name in fx["field_order"]:  # both noisy: within 1 of each other (12 sigma at these budgets)
            assert abs(getattr(m, name) - w[name]) < 1.0, (k, name)


def _uniform_groups(ns, per_n):
    """per_n partitions with exactly n distinct privacy ids, for each n."""
    pid, pk = [], []
    nxt = part = 0
    for n in ns:
        for _ in range(per_n):
            pid.extend(range(nxt, nxt + n))
            pk.extend([part] * n)
            nxt += n
            part += 1
    return (pdp.ColumnTable({"pid": np.asarray(pid, np.int64), "pk": np.asarray(pk, np.int64),
                             "v": np.zeros(len(pid))}), part)


@pytest.mark.parametrize("kind", ["laplace", "gaussian"])
def test_post_aggregation_thresholding_keep_rates(device, kind):
    """Partitions with n privacy ids survive with P(n + noise > T): Laplace
    thresholding b = l0/eps', T = 1 - b ln(2 delta'); Gaussian sigma with
    l2 = sqrt(l0), T = 1 + sigma Phi^-1(1 - delta') (PyDP partition selection
    restated, dp_computations.py thresholding params).  Binomial 5-sigma bands."""
    from scipy.stats import laplace, norm
    ns, per_n = [1, 2, 3, 4, 5, 6, 8], 3000
    table, n_parts = _uniform_groups(ns, per_n)
    nk = pdp.NoiseKind.LAPLACE if kind == "laplace" else pdp.NoiseKind.GAUSSIAN
    params = pdp.AggregateParams(metrics=[pdp.Metrics.PRIVACY_ID_COUNT], noise_kind=nk,
                                 max_partitions_contributed=1, max_contributions_per_partition=1,
                                 post_aggregation_thresholding=True)
    eps, delta = 1.0, 1e-3
    engine, acc = _engine(eps, delta, seed=32 if kind == "laplace" else 33)
    sink = engine.aggregate(table, params, pdp.DataExtractors(privacy_id_extractor=pdp.ColumnExtractor("pid"),
                                                             partition_extractor=pdp.ColumnExtractor("pk"),
                                                             value_extractor=pdp.ColumnExtractor("v")))
    acc.compute_budgets()
    out = dict((int(k), m.privacy_id_count) for k, m in sink)
    (spec,) = [m.mechanism_spec for m in acc._mechanisms]  # the thresholding mechanism only
    if kind == "laplace":
        b, T = dpc.laplace_thresholding_params(spec.eps, spec.delta, 1)
        dist = laplace(scale=b)
    else:
        s, T = dpc.gaussian_thresholding_params(spec.eps, spec.delta, 1)
        dist = norm(scale=s)
    kept = np.zeros(n_parts, dtype=bool)
    kept[list(out)] = True
    for i, n in enumerate(ns):
        p = float(dist.sf(T - n))
        k = int(kept[i * per_n:(i + 1) * per_n].sum())
        sd = math.sqrt(per_n * p * (1 - p))
        assert abs(k - per_n * p) <= 5 * sd + 1, (kind, n, k, per_n * p)
    vals = np.array(list(out.values()))
    assert np.all(vals > T)  # released values are the noised counts above the threshold
