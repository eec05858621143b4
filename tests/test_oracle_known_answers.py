"""Known answers the reference's own tests hold for the aggregate path
(SURVEY §4 table), restated against (a) the oracle's PyDP restatement and
(b) the product's host-side calibration (pipelinedp_amd.dp_computations,
partition_selection, combiners, budget_accounting).  CPU only."""
import math

import numpy as np
import pytest

import pipelinedp_amd as pdp
from oracle import pydp_restatement as pydp
from pipelinedp_amd import combiners as C
from pipelinedp_amd import dp_computations as dpc
from pipelinedp_amd import partition_selection as ps

# (eps, delta, l2, sigma) stated exactly in tests/dp_computations_test.py:62-67,
# 371-405, 485-545 of the reference
SIGMA_EXACT = [
    (0.5, 1e-10, 10, 114.375),
    (1.0, 1e-10, 15, 88.06640625),
    (2, 1e-15, 4.5, 17.1826171875),
    (0.1, 1e-5, 0.55, 16.9125),
    (0.2, 1e-10, 10, 277.34375),
    (1, 1e-5, 5.0, 18.662109375),               # compute_dp_sum_noise_std, l0=1, max|sum|=5
    (2.0, 1e-8, math.sqrt(2) * 10, 37.53742639189524),  # l0=2, max|sum|=10
]


@pytest.mark.parametrize("eps,delta,l2,sigma", SIGMA_EXACT)
def test_gaussian_sigma_exact(eps, delta, l2, sigma):
    assert dpc.compute_sigma(eps, delta, l2) == sigma
    assert pydp.GaussianMechanism(eps, delta, l2).std == sigma


def test_sensitivity_norms():
    """dp_computations_test.py: l1 = l0 * linf, l2 = sqrt(l0) * linf."""
    assert dpc.compute_l1_sensitivity(4.5, 12.123) == pytest.approx(54.5535, abs=0.1)
    assert dpc.compute_l2_sensitivity(4.5, 12.123) == pytest.approx(25.716766525, abs=0.1)


# The 3-decimal sigmas (15.835, 5.278, 11.197, 110.847; combiners_test.py:272-288,
# 344-360, 564-593) are checked through the combiners below.
def _agg_params(**kw):
    base = dict(metrics=[pdp.Metrics.COUNT], noise_kind=pdp.NoiseKind.GAUSSIAN,
                max_partitions_contributed=2, max_contributions_per_partition=3,
                min_value=0, max_value=1.0)
    base.update(kw)
    return pdp.AggregateParams(**base)


def _spec(mech_type, eps=1.0, delta=1e-5):
    s = pdp.MechanismSpec(mech_type)
    s.set_eps_delta(eps, delta)
    return s


@pytest.mark.parametrize("mtype,expected", [(pdp.MechanismType.GAUSSIAN, 15.835),
                                            (pdp.MechanismType.LAPLACE, 6.0)])
def test_count_mechanism_parameter(mtype, expected):
    """combiners_test.py:272-288 (l0=2, linf=3, eps=1, delta=1e-5)."""
    c = C.CountCombiner(_spec(mtype), _agg_params())
    assert c.get_mechanism().noise_parameter == pytest.approx(expected, abs=1e-3)


@pytest.mark.parametrize("mtype,expected", [(pdp.MechanismType.GAUSSIAN, 5.278),
                                            (pdp.MechanismType.LAPLACE, 2.0)])
def test_privacy_id_count_mechanism_parameter(mtype, expected):
    """combiners_test.py:344-360."""
    c = C.PrivacyIdCountCombiner(_spec(mtype), _agg_params())
    assert c.get_mechanism().noise_parameter == pytest.approx(expected, abs=1e-3)


@pytest.mark.parametrize("mtype,per_partition,expected", [
    (pdp.MechanismType.GAUSSIAN, True, 11.197), (pdp.MechanismType.GAUSSIAN, False, 110.847),
    (pdp.MechanismType.LAPLACE, True, 3.0), (pdp.MechanismType.LAPLACE, False, 42.0)])
def test_sum_mechanism_parameter(mtype, per_partition, expected):
    """combiners_test.py:564-593 (max_value=7, per-partition bounds [0, 3], l0=linf=1)."""
    if per_partition:
        params = pdp.AggregateParams(min_sum_per_partition=0, max_sum_per_partition=3,
                                     max_contributions_per_partition=1, max_partitions_contributed=1,
                                     noise_kind=pdp.NoiseKind.GAUSSIAN, metrics=[pdp.Metrics.SUM])
    else:
        params = _agg_params(max_value=7.0, metrics=[pdp.Metrics.SUM])
    c = C.SumCombiner(_spec(mtype), params)
    assert c.get_mechanism().noise_parameter == pytest.approx(expected, abs=1e-3)


@pytest.mark.parametrize("eps,l1,b", [(2, 4.5, 2.25), (0.1, 0.55, 5.5), (2.0, 25, 12.5)])
def test_laplace_diversity(eps, l1, b):
    """dp_computations_test.py:429-445."""
    m = dpc.LaplaceMechanism.create_from_epsilon(eps, l1)
    assert m.noise_parameter == pytest.approx(b, abs=1e-12)
    assert m.std == pytest.approx(b * math.sqrt(2), abs=1e-12)
    assert pydp.LaplaceMechanism(eps, l1).diversity == pytest.approx(b, abs=1e-12)


def test_mechanism_describe_strings():
    """dp_computations_test.py (describe tests)."""
    g = dpc.GaussianMechanism.create_from_epsilon_delta(1.0, 1e-10, 15)
    assert g.describe() == ("Gaussian mechanism:  parameter=88.06640625  eps=1.0  delta=1e-10  "
                            "l2_sensitivity=15")
    lap = dpc.LaplaceMechanism.create_from_epsilon(2.0, 25)
    assert lap.describe() == "Laplace mechanism:  parameter=12.5  eps=2.0  l1_sensitivity=25"


def test_laplace_and_gaussian_from_stddev():
    lap = dpc.LaplaceMechanism.create_from_std_deviation(10, 3.5)
    assert lap.noise_parameter == pytest.approx(10 / np.sqrt(2) * 3.5, abs=1e-12)
    assert lap.std == pytest.approx(35)
    g = dpc.GaussianMechanism.create_from_std_deviation(5, 15)
    assert g.noise_parameter == 75 and g.std == 75 and g.sensitivity == 15


@pytest.mark.parametrize("n,pre,expected", [(10, None, 0.12818308050524607),
                                            (12, 3, 0.12818308050524607)])
def test_truncated_geometric_keep_probability(n, pre, expected):
    """analysis/tests/per_partition_combiners_test.py:199-238 (eps=1, delta=1e-5, l0=1)."""
    assert dpc.truncated_geometric_keep_probability(n, 1, 1e-5, 1, pre) == pytest.approx(expected, abs=1e-10)
    s = ps.create_partition_selection_strategy(pdp.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC,
                                               1, 1e-5, 1, pre)
    assert s.probability_of_keep(n) == pytest.approx(expected, abs=1e-10)
    o = pydp.create_partition_strategy("truncated_geometric", 1, 1e-5, 1, pre)
    assert o.probability_of_keep(n) == pytest.approx(expected, abs=1e-10)


def test_truncated_geometric_mixture():
    """Binomial(100, 0.1) mixture of keep probabilities = 0.3321336253750503
    (per_partition_combiners_test.py 'Small eps delta')."""
    from scipy.stats import binom
    table = dpc.truncated_geometric_keep_table(1, 1e-5, 1)
    n = np.arange(101)
    p = np.array([table[min(k, len(table) - 1)] for k in n])
    assert float((binom.pmf(n, 100, 0.1) * p).sum()) == pytest.approx(0.3321336253750503, abs=1e-10)
    # 'Large eps delta' keeps everything with probability 1
    assert dpc.truncated_geometric_keep_probability(100, 100, 0.5, 1) == 1.0


def test_thresholds():
    """Gaussian thresholding 'threshold=56.5' (combiners_test.py:476-480, eps=1,
    delta=1e-10, l0=2); Laplace thresholding '~= 3.2' (dp_engine_test.py:1233-1250,
    eps=10, delta=1e-10, l0=1)."""
    g = ps.create_partition_selection_strategy(pdp.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING,
                                               1.0, 1e-10, 2)
    assert f"{g.threshold:.1f}" == "56.5"
    lap = ps.create_partition_selection_strategy(pdp.PartitionSelectionStrategy.LAPLACE_THRESHOLDING,
                                                 10.0, 1e-10, 1)
    assert lap.threshold == pytest.approx(3.2, abs=0.05)
    mech = C.ThresholdingMechanism(1.0, 1e-10, pdp.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING, 2, None)
    assert mech.describe() == "Gaussian Thresholding with threshold=56.5 eps=1.0 delta=1e-10"
    assert pydp.create_partition_strategy("gaussian", 1.0, 1e-10, 2).threshold == pytest.approx(g.threshold)


def test_budget_split():
    """budget_accounting_test.py:57-71."""
    acc = pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=1e-6)
    b1 = acc.request_budget(mechanism_type=pdp.MechanismType.LAPLACE)
    b2 = acc.request_budget(mechanism_type=pdp.MechanismType.GAUSSIAN, weight=3)
    with pytest.raises(AssertionError):
        _ = b1.eps
    acc.compute_budgets()
    assert (b1.eps, b1.delta) == (0.25, 0)
    assert (b2.eps, b2.delta) == (0.75, 1e-6)


def test_budget_scopes_normalise():
    acc = pdp.NaiveBudgetAccountant(total_epsilon=1, total_delta=1e-6)
    with acc.scope(weight=0.4):
        b1 = acc.request_budget(mechanism_type=pdp.MechanismType.LAPLACE)
        b2 = acc.request_budget(mechanism_type=pdp.MechanismType.LAPLACE)
    with acc.scope(weight=0.6):
        b3 = acc.request_budget(mechanism_type=pdp.MechanismType.LAPLACE)
    acc.compute_budgets()
    assert b1.eps == pytest.approx(0.2) and b2.eps == pytest.approx(0.2) and b3.eps == pytest.approx(0.6)
    with pytest.raises(Exception):
        acc.compute_budgets()


def test_equally_split_budget():
    """dp_computations_test.py:229-243: the last share takes the remainder."""
    budgets = dpc.equally_split_budget(0.5, 1e-6, 3)
    assert budgets[0] == (0.5 / 3, 1e-6 / 3)
    assert sum(b[0] for b in budgets) == 0.5
    assert budgets[2] == (0.5 - 2 * (0.5 / 3), 1e-6 - 2 * (1e-6 / 3))
    with pytest.raises(ValueError):
        dpc.equally_split_budget(1, 1, 0)


def test_combiner_accumulators():
    """combiners_test.py:242-254, 314-326, 514-531, 612-624, 659-671, 792-806."""
    spec = _spec(pdp.MechanismType.GAUSSIAN)
    cnt = C.CountCombiner(spec, _agg_params())
    assert cnt.create_accumulator([]) == 0 and cnt.create_accumulator([1, 2]) == 2
    pid = C.PrivacyIdCountCombiner(spec, _agg_params())
    assert pid.create_accumulator([]) == 0 and pid.create_accumulator([1, 2]) == 1
    s = C.SumCombiner(spec, _agg_params(max_value=1.0, metrics=[pdp.Metrics.SUM]))
    assert [s.create_accumulator(v) for v in ([], [1, 1], [1, 3], [0, 3])] == [0, 2, 2, 1]
    sp = C.SumCombiner(spec, pdp.AggregateParams(min_sum_per_partition=0, max_sum_per_partition=3,
                                                 max_contributions_per_partition=1,
                                                 max_partitions_contributed=1, metrics=[pdp.Metrics.SUM]))
    assert [sp.create_accumulator(v) for v in ([], [2, 0.5], [4, 1], [-10, 5, 3])] == [0, 2.5, 3, 0]
    assert not sp.expects_per_partition_sampling()
    m = C.MeanCombiner(spec, spec, _agg_params(max_value=4), ["count", "sum", "mean"])
    assert m.create_accumulator([1, 3]) == (2, 0)
    v = C.VarianceCombiner(C.CombinerParams(spec, _agg_params(max_value=4)), ["count", "sum", "mean", "variance"])
    assert v.create_accumulator([1, 2]) == (2, -1, 1)
    comp = C.CompoundCombiner([C.CountCombiner(spec, _agg_params()), C.SumCombiner(spec, _agg_params())],
                              return_named_tuple=True)
    assert comp.create_accumulator((1, 1)) == (1, (2, 2))
    assert comp.create_accumulator((0, 3, 4)) == (1, (3, 2))
    assert comp.merge_accumulators((1, (2, 2)), (1, (2, 2))) == (2, (4, 4))
    assert comp.merge_accumulators((2, (2, 3)), (1, (2, 2))) == (3, (4, 5))


def test_mean_with_deterministic_noise():
    """combiners_test.py:633-647: add_noise = x + 1 -> count 101, sum 353, mean 353/101."""
    spec = _spec(pdp.MechanismType.GAUSSIAN)
    m = C.MeanCombiner(spec, spec, _agg_params(max_value=4), ["count", "sum", "mean"])
    mech = m.get_mechanism()
    mech._count_mechanism.add_noise = lambda x: x + 1
    mech._sum_mechanism.add_noise = lambda x: x + 1
    out = m.compute_metrics((100, 150))
    assert out["count"] == 101 and out["sum"] == 353
    assert out["mean"] == pytest.approx(353 / 101, abs=1e-12)
    assert list(out) == ["mean", "count", "sum"]


def test_variance_no_noise():
    """combiners_test.py:673-680 with a huge budget (eps=1e5, delta=1-1e-5)."""
    spec = _spec(pdp.MechanismType.GAUSSIAN, eps=1e5, delta=1 - 1e-5)
    v = C.VarianceCombiner(C.CombinerParams(spec, _agg_params(max_value=4)), ["count", "sum", "mean", "variance"])
    res = v.compute_metrics((4, 0, 2))
    assert res["count"] == pytest.approx(4, abs=1e-5) and res["sum"] == pytest.approx(8, abs=1e-5)
    assert res["mean"] == pytest.approx(2, abs=1e-5) and res["variance"] == pytest.approx(0.5, abs=1e-5)
    assert list(res) == ["variance", "count", "sum", "mean"]


def test_compound_metrics_field_order():
    """MetricsTuple fields follow the combiners' compute_metrics dicts."""
    acc = pdp.NaiveBudgetAccountant(1, 1e-6)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT, pdp.Metrics.COUNT,
                                          pdp.Metrics.MEAN, pdp.Metrics.VARIANCE],
                                 max_partitions_contributed=1, max_contributions_per_partition=1,
                                 min_value=0, max_value=1)
    comp = C.create_compound_combiner(params, acc)
    assert [type(c).__name__ for c in comp.combiners] == ["VarianceCombiner", "PrivacyIdCountCombiner"]
    assert comp.metrics_names() == ("variance", "mean", "count", "sum", "privacy_id_count")
