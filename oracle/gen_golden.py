"""TEST INFRASTRUCTURE — regenerate tests/golden/*.json by running the reference.

Runs only in the build container (it reads /root/reference, which never travels
to the GPU box).  The reference imports with the python-dp stand-in in
oracle/pydp_standin (PyDP is not installed; no permission denial was involved).

For every case the reference's DPEngine.aggregate runs on LocalBackend with
* CompoundCombiner.compute_metrics patched to return the raw accumulator
  (pre-noise, exact), and
* private partition selection patched to keep every partition,
on inputs where no contribution sampling fires (every pid has <= L0 distinct
partitions and every (pid, pk) <= Linf rows), so the expected per-partition
accumulators are deterministic.  Sampling itself is pinned with inclusion
counts of LocalBackend.sample_fixed_per_key under np.random.seed.

Usage: python -m oracle.gen_golden   (from the repo root)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden")


def _import_reference():
    for p in (os.path.join(ROOT, "oracle", "pydp_standin"), ROOT, REFERENCE):
        if p not in sys.path:
            sys.path.insert(0, p)
    import pipeline_dp
    return pipeline_dp


def _py(x):
    if isinstance(x, (tuple, list)):
        return [_py(v) for v in x]
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    return x


def _no_sampling_rows(rng, n_pids, l0, linf, n_partitions, value_fn, pid_fmt=None, pk_fmt=None,
                      rows_per_pid=None):
    rows = []
    for u in range(n_pids):
        d = int(rng.integers(1, l0 + 1))
        pks = rng.choice(n_partitions, size=d, replace=False)
        budget = rows_per_pid  # SamplingPerPrivacyId: <= max_contributions rows per pid
        for k in pks:
            r = int(rng.integers(1, linf + 1))
            if budget is not None:
                r = min(r, budget)
                budget -= r
            for _ in range(r):
                pid = pid_fmt(u) if pid_fmt else u
                pk = pk_fmt(int(k)) if pk_fmt else int(k)
                rows.append([pid, pk, value_fn(rng)])
    order = rng.permutation(len(rows))
    return [rows[i] for i in order]


CASES = [
    dict(name="count_sum_int_movie", metrics=["COUNT", "SUM"], noise="LAPLACE", l0=2, linf=1,
         min_value=1, max_value=5, n_pids=400, n_partitions=60, value="int1_5"),
    dict(name="count_sum_mean_f64", metrics=["COUNT", "SUM", "MEAN"], noise="LAPLACE", l0=3, linf=2,
         min_value=0.0, max_value=10.0, n_pids=500, n_partitions=80, value="normal5_3"),
    dict(name="variance_pid_count", metrics=["VARIANCE", "PRIVACY_ID_COUNT"], noise="GAUSSIAN", l0=4,
         linf=2, min_value=0.0, max_value=10.0, n_pids=300, n_partitions=50, value="normal5_4"),
    dict(name="mean_variance_all", metrics=["VARIANCE", "MEAN", "COUNT", "SUM"], noise="LAPLACE", l0=2,
         linf=3, min_value=-2.0, max_value=6.0, n_pids=300, n_partitions=40, value="normal2_3"),
    dict(name="sum_per_partition_int", metrics=["SUM", "COUNT"], noise="LAPLACE", l0=3, linf=2,
         min_sum=-3, max_sum=7, n_pids=300, n_partitions=30, value="int_m4_9"),
    dict(name="privacy_id_count_only", metrics=["PRIVACY_ID_COUNT"], noise="LAPLACE", l0=2, linf=1,
         n_pids=300, n_partitions=40, value="int1_5", rows_per_pair=4),
    dict(name="public_partitions", metrics=["COUNT", "SUM", "PRIVACY_ID_COUNT"], noise="LAPLACE", l0=2,
         linf=2, min_value=0, max_value=4, n_pids=200, n_partitions=30, value="int1_5",
         public=[0, 1, 2, 3, 5, 8, 13, 21, 34, 55, 89]),
    dict(name="string_keys", metrics=["COUNT", "SUM"], noise="LAPLACE", l0=2, linf=2, min_value=0.0,
         max_value=3.0, n_pids=150, n_partitions=20, value="normal1_1", string_keys=True),
    # bounders other than Cross+Per (dp_engine.py:380-400); "gen_*" shape the
    # data so that no sampling fires under the case's bounds
    dict(name="linf_sampler", bounder="linf", metrics=["COUNT", "SUM", "MEAN"], noise="LAPLACE", l0=2,
         linf=2, min_value=0.0, max_value=8.0, n_pids=300, n_partitions=40, value="normal5_3",
         gen_pairs_per_pid=7, gen_rows_per_pair=2),
    dict(name="noop_sampler", bounder="noop", metrics=["SUM", "PRIVACY_ID_COUNT"],
         noise="LAPLACE", l0=1, linf=1, min_sum=-5.0, max_sum=12.0, n_pids=300, n_partitions=40,
         value="normal2_3", gen_pairs_per_pid=5, gen_rows_per_pair=4),
    dict(name="max_contributions", bounder="per_pid", metrics=["COUNT", "SUM", "PRIVACY_ID_COUNT"],
         noise="LAPLACE", max_contributions=6, min_value=1, max_value=4, n_pids=300, n_partitions=30,
         value="int1_5", gen_pairs_per_pid=4, gen_rows_per_pair=3, public=list(range(0, 30, 2))),
    dict(name="bounds_already_enforced", bounder="enforced", metrics=["COUNT", "SUM", "MEAN"],
         noise="LAPLACE", l0=3, linf=2, min_value=0.0, max_value=6.0, n_pids=200, n_partitions=25,
         value="normal2_3", gen_pairs_per_pid=3, gen_rows_per_pair=3),
]


def case_params(pdp, case):
    """AggregateParams of a fixture case (shared with tests/golden_util.py)."""
    kw = {}
    for k in ("min_value", "max_value", "min_sum", "max_sum"):
        if k in case:
            kw[{"min_sum": "min_sum_per_partition", "max_sum": "max_sum_per_partition"}.get(k, k)] = case[k]
    bounder = case.get("bounder", "default")
    if bounder == "per_pid":
        kw["max_contributions"] = case["max_contributions"]
    else:
        kw["max_partitions_contributed"] = case["l0"]
        kw["max_contributions_per_partition"] = case["linf"]
    if bounder in ("linf", "noop"):
        kw["perform_cross_partition_contribution_bounding"] = False
    if bounder == "enforced":
        kw["contribution_bounds_already_enforced"] = True
    return pdp.AggregateParams(metrics=[getattr(pdp.Metrics, m) for m in case["metrics"]],
                               noise_kind=getattr(pdp.NoiseKind, case["noise"]), **kw)

VALUE_FNS = {
    "int1_5": lambda r: int(r.integers(1, 6)),
    "int_m4_9": lambda r: int(r.integers(-4, 10)),
    "normal5_3": lambda r: float(r.normal(5, 3)),
    "normal5_4": lambda r: float(r.normal(5, 4)),
    "normal2_3": lambda r: float(r.normal(2, 3)),
    "normal1_1": lambda r: float(r.normal(1, 1)),
}


def run_case(pdp, case, seed):
    from pipeline_dp import combiners, partition_selection

    rng = np.random.default_rng(seed)
    fmt_pid = (lambda u: f"user-{u}") if case.get("string_keys") else None
    fmt_pk = (lambda k: f"item/{k}") if case.get("string_keys") else None
    pairs = case.get("gen_pairs_per_pid", case.get("l0"))
    per_pair = case.get("gen_rows_per_pair", case.get("rows_per_pair", case.get("linf")))
    rows = _no_sampling_rows(rng, case["n_pids"], pairs, per_pair, case["n_partitions"],
                             VALUE_FNS[case["value"]], fmt_pid, fmt_pk,
                             rows_per_pid=case.get("max_contributions"))
    params = case_params(pdp, case)
    accountant = pdp.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
    engine = pdp.DPEngine(accountant, pdp.LocalBackend())
    enforced = case.get("bounder") == "enforced"
    extractors = pdp.DataExtractors(privacy_id_extractor=None if enforced else (lambda r: r[0]),
                                    partition_extractor=lambda r: r[1],
                                    value_extractor=lambda r: r[2])

    class KeepAll:

        def should_keep(self, n):
            return True

    saved_cm = combiners.CompoundCombiner.compute_metrics
    saved_ps = partition_selection.create_partition_selection_strategy
    combiners.CompoundCombiner.compute_metrics = lambda self, acc: acc
    partition_selection.create_partition_selection_strategy = lambda *a, **k: KeepAll()
    try:
        public = case.get("public")
        out = engine.aggregate(rows, params, extractors, public_partitions=public)
        accountant.compute_budgets()
        result = sorted(([_py(pk), _py(acc)] for pk, acc in out), key=lambda t: str(t[0]))
    finally:
        combiners.CompoundCombiner.compute_metrics = saved_cm
        partition_selection.create_partition_selection_strategy = saved_ps
    budgets = [[m.mechanism_spec.mechanism_type.value, m.mechanism_spec.eps, m.mechanism_spec.delta]
               for m in accountant._mechanisms]
    # the bounder class the reference's DPEngine picks for these params (dp_engine.py:380-400)
    probe = pdp.DPEngine(pdp.NaiveBudgetAccountant(1.0, 1e-6), pdp.LocalBackend())
    comb = combiners.create_compound_combiner(params, pdp.NaiveBudgetAccountant(1.0, 1e-6))
    bounder = None if params.contribution_bounds_already_enforced else type(
        probe._create_contribution_bounder(params, comb.expects_per_partition_sampling())).__name__
    return {"name": case["name"], "case": case, "rows": rows, "expected": result, "budgets": budgets,
            "reference_bounder": bounder}


def sampling_fixture(pdp, trials=4000):
    """Inclusion counts of the reference's sampling under np.random.seed."""
    backend = pdp.LocalBackend()
    np.random.seed(2024)
    linf_counts = [0] * 5
    for _ in range(trials):
        for _, vals in backend.sample_fixed_per_key([("k", i) for i in range(5)], 2):
            for v in vals:
                linf_counts[v] += 1
    from pipeline_dp import contribution_bounders
    from pipeline_dp.report_generator import ReportGenerator

    class P:
        max_partitions_contributed = 2
        max_contributions_per_partition = 1

    l0_counts = [0] * 6
    rows = [("u", k, 1.0) for k in range(6)]
    for _ in range(trials):
        out = contribution_bounders.SamplingCrossAndPerPartitionContributionBounder().bound_contributions(
            rows, P, backend, ReportGenerator(None, "t"), lambda v: len(v))
        for (pid, pk), _ in out:
            l0_counts[pk] += 1
    return {"trials": trials, "linf": {"rows": 5, "n": 2, "counts": linf_counts},
            "l0": {"partitions": 6, "n": 2, "counts": l0_counts}}


def select_partitions_fixture(pdp, seed=300):
    """DPEngine.select_partitions on LocalBackend: every pid has <= L0 distinct
    partitions (no sampling fires); eps = 1e4, delta = 1e-12 makes truncated-
    geometric selection keep every partition with >= 2 privacy ids and drop
    those with 1 (keep probabilities 1 - O(e^-1e4) and delta' = O(1e-12))."""
    rng = np.random.default_rng(seed)
    rows = []
    for u in range(400):
        for k in rng.choice(120, size=int(rng.integers(1, 4)), replace=False):
            rows.extend([[u, f"p{int(k)}"]] * int(rng.integers(1, 3)))
    params = pdp.SelectPartitionsParams(max_partitions_contributed=3)
    accountant = pdp.NaiveBudgetAccountant(total_epsilon=1e4, total_delta=1e-12)
    engine = pdp.DPEngine(accountant, pdp.LocalBackend())
    ext = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1])
    out = engine.select_partitions(rows, params, ext)
    accountant.compute_budgets()
    keys = sorted(out)
    pids = {}
    for u, k in rows:
        pids.setdefault(k, set()).add(u)
    assert keys == sorted(k for k, s in pids.items() if len(s) >= 2)
    return {"name": "select_partitions", "rows": rows, "max_partitions_contributed": 3,
            "eps": 1e4, "delta": 1e-12, "expected_keys": keys}


def post_threshold_fixture(pdp, noise_kind, eps, seed=400):
    """DPEngine.aggregate(COUNT, PRIVACY_ID_COUNT, post_aggregation_thresholding
    = True) on LocalBackend, real noise path (no patching): the
    PostAggregationThresholdingCombiner (combiners.py:328-382) replaces the
    PRIVACY_ID_COUNT combiner and DPEngine drops partitions whose thresholded
    value is None (dp_engine.py:184-185, 544-549).  A huge eps (1e4 Laplace,
    1300 Gaussian: the stand-in's calibration needs eps < 700 per mechanism)
    and delta = 1e-10 make the outcome deterministic up to O(e^-20):
    partitions with >= 2 privacy ids are kept, those with 1 dropped, and every
    released value is within 1 of its exact count (12 sigma)."""
    rng = np.random.default_rng(seed)
    rows = []
    for u in range(300):
        for k in rng.choice(80, size=int(rng.integers(1, 3)), replace=False):
            rows.extend([[u, int(k), 1]] * int(rng.integers(1, 3)))
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.PRIVACY_ID_COUNT],
                                 noise_kind=getattr(pdp.NoiseKind, noise_kind), max_partitions_contributed=2,
                                 max_contributions_per_partition=2, post_aggregation_thresholding=True)
    accountant = pdp.NaiveBudgetAccountant(total_epsilon=eps, total_delta=1e-10)
    engine = pdp.DPEngine(accountant, pdp.LocalBackend())
    ext = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                             value_extractor=lambda r: r[2])
    out = engine.aggregate(rows, params, ext)
    accountant.compute_budgets()
    got = sorted([int(pk), m._asdict()] for pk, m in out)
    pids, cnt = {}, {}
    for u, k, _ in rows:
        pids.setdefault(k, set()).add(u)
        cnt[k] = cnt.get(k, 0) + 1
    assert [k for k, _ in got] == sorted(k for k, s in pids.items() if len(s) >= 2)
    for k, m in got:
        assert abs(m["privacy_id_count"] - len(pids[k])) < 1.0 and abs(m["count"] - cnt[k]) < 1.0
    budgets = [[m.mechanism_spec.mechanism_type.value, m.mechanism_spec.eps, m.mechanism_spec.delta]
               for m in accountant._mechanisms]
    return {"name": f"post_aggregation_thresholding_{noise_kind.lower()}", "rows": rows, "eps": eps,
            "delta": 1e-10, "noise_kind": noise_kind, "l0": 2, "linf": 2,
            "field_order": list(got[0][1]) if got else [], "expected": got, "budgets": budgets}


def main_post_threshold():
    pdp = _import_reference()
    for kind, eps in (("LAPLACE", 1e4), ("GAUSSIAN", 1300.0)):
        fx = post_threshold_fixture(pdp, kind, eps)
        with open(os.path.join(OUT, f"{fx['name']}.json"), "w") as f:
            json.dump(fx, f)
        print(fx["name"], len(fx["rows"]), "rows", len(fx["expected"]), "partitions", fx["field_order"])


def main():
    pdp = _import_reference()
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "select_partitions.json"), "w") as f:
        json.dump(select_partitions_fixture(pdp), f)
    print("select_partitions written")
    for i, case in enumerate(CASES):
        fx = run_case(pdp, case, seed=100 + i)
        with open(os.path.join(OUT, f"{case['name']}.json"), "w") as f:
            json.dump(fx, f)
        print(case["name"], len(fx["rows"]), "rows", len(fx["expected"]), "partitions")
    with open(os.path.join(OUT, "sampling_inclusion.json"), "w") as f:
        json.dump(sampling_fixture(pdp), f)
    print("sampling_inclusion written")
    main_post_threshold()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "post_threshold":
        main_post_threshold()  # only the post-aggregation-thresholding fixtures
    else:
        main()
