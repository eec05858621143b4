"""Helpers for the golden fixtures in tests/golden (made by oracle/gen_golden.py
from the reference's own DPEngine.aggregate on LocalBackend)."""
import glob
import json
import math
import os

import numpy as np

import pipelinedp_amd as pdp
from pipelinedp_amd import combiners as C

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REL_TOL = 1e-9  # fp64 sums: north-star tolerance (order of summation differs)


# fixtures with their own layout (their own tests read them)
_NOT_AGGREGATE_CASES = ("sampling_inclusion.json", "select_partitions.json")


def fixtures():
    out = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, "*.json"))):
        if path.endswith(_NOT_AGGREGATE_CASES) or "post_aggregation_thresholding" in path:
            continue
        with open(path) as f:
            out.append(json.load(f))
    return out


def fixture_ids():
    return [os.path.basename(p)[:-5] for p in sorted(glob.glob(os.path.join(GOLDEN, "*.json")))
            if not p.endswith(_NOT_AGGREGATE_CASES) and "post_aggregation_thresholding" not in p]


def aggregate_params(case, module=pdp):
    """AggregateParams of a fixture case (as oracle/gen_golden.py:case_params
    built them for the reference); `module` is pipelinedp_amd or pipeline_dp."""
    kw = {}
    for k, name in (("min_value", "min_value"), ("max_value", "max_value"),
                    ("min_sum", "min_sum_per_partition"), ("max_sum", "max_sum_per_partition")):
        if k in case:
            kw[name] = case[k]
    bounder = bounder_of(case)
    if bounder == "per_pid":
        kw["max_contributions"] = case["max_contributions"]
    else:
        kw["max_partitions_contributed"] = case["l0"]
        kw["max_contributions_per_partition"] = case["linf"]
    if bounder in ("linf", "noop"):
        kw["perform_cross_partition_contribution_bounding"] = False
    if bounder == "enforced":
        kw["contribution_bounds_already_enforced"] = True
    return module.AggregateParams(metrics=[getattr(module.Metrics, m) for m in case["metrics"]],
                                  noise_kind=getattr(module.NoiseKind, case["noise"]), **kw)


def bounder_of(case):
    """'default' (Cross+Per or Cross), 'linf', 'noop', 'per_pid' or 'enforced'."""
    return case.get("bounder", "default")


def extractors(case, module=pdp):
    pid = None if bounder_of(case) == "enforced" else (lambda r: r[0])
    return module.DataExtractors(privacy_id_extractor=pid, partition_extractor=lambda r: r[1],
                                 value_extractor=lambda r: r[2])


def combiner_kinds(case):
    comp = C.create_compound_combiner(aggregate_params(case), pdp.NaiveBudgetAccountant(1.0, 1e-6))
    return [type(c).__name__ for c in comp.combiners], comp.expects_per_partition_sampling()


def _key(k):
    return tuple(k) if isinstance(k, list) else k


def expected_map(fx):
    return {_key(pk): acc for pk, acc in fx["expected"]}


def assert_acc_equal(want, got, where=""):
    """Nested accumulator equality: ints exact, floats within REL_TOL of the
    magnitude (or 1e-9 absolute near zero)."""
    if isinstance(want, (list, tuple)):
        assert isinstance(got, (list, tuple)) and len(want) == len(got), f"{where}: {want} vs {got}"
        for i, (w, g) in enumerate(zip(want, got)):
            assert_acc_equal(w, g, f"{where}[{i}]")
        return
    if isinstance(want, int) and not isinstance(want, bool) and isinstance(got, (int, np.integer)):
        assert int(got) == want, f"{where}: {want} vs {got}"
        return
    w, g = float(want), float(got)
    assert math.isclose(w, g, rel_tol=REL_TOL, abs_tol=1e-9), f"{where}: {want} vs {got}"
