"""Host side of the drop-in boundary on the CPU: DPEngine.aggregate graphs
built on ColumnarBackend are recognised into the kernels' configuration
(bounding, selection, metric program, budgets), unsupported modes raise the
reference's error types at the same points, and execution without a GPU fails
loudly instead of falling back to a CPU path.

The reference-engine test builds the graph with the reference's own
pipeline_dp.DPEngine (imported from /root/reference with the PyDP stand-in in
oracle/pydp_standin; skipped when the reference is absent, e.g. on the GPU box)."""
import math
import os
import sys

import numpy as np
import pytest

import pipelinedp_amd as pdp
from pipelinedp_amd import _native as N
from pipelinedp_amd import columnar_backend as CB
from pipelinedp_amd import dp_computations as dpc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = "/root/reference"

ROWS = [(u, u % 7, float(u % 11)) for u in range(200)]


def _extractors():
    return pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                              value_extractor=lambda r: r[2])


def _graph(params, engine_mod=pdp, backend=None, public=None, rows=ROWS, eps=1.0, delta=1e-6):
    backend = backend or CB.ColumnarBackend()
    acc = engine_mod.NaiveBudgetAccountant(total_epsilon=eps, total_delta=delta)
    engine = engine_mod.DPEngine(acc, backend)
    sink = engine.aggregate(rows, params, _extractors(), public_partitions=public)
    acc.compute_budgets()
    return sink, engine, acc


def _params(**kw):
    base = dict(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM], noise_kind=pdp.NoiseKind.LAPLACE,
                max_partitions_contributed=2, max_contributions_per_partition=3, min_value=0.0,
                max_value=10.0)
    base.update(kw)
    return pdp.AggregateParams(**base)


def _run_of(sink):
    plan = CB.recognise(sink)
    return plan, CB.AggregateRun(CB.ColumnarBackend(), plan)


def test_count_sum_laplace_private_partitions():
    sink, _, _ = _graph(_params())
    plan, run = _run_of(sink)
    assert plan.bounder == "cross_and_per" and plan.public_keys is None
    spec = run._bounding_spec(N.VALUE_F64)
    assert (spec.l0, spec.linf, spec.flags) == (2, 3, N.ACC_SUM)
    assert (spec.min_value, spec.max_value) == (0.0, 10.0)
    assert run.prog.fields == ["count", "sum"]
    # 3 mechanisms share eps = 1: COUNT, SUM, GENERIC selection (budget_accounting.py:301-408)
    b_count = dpc.laplace_diversity(1 / 3, 2 * 3)
    b_sum = dpc.laplace_diversity(1 / 3, 2 * 3 * 10.0)
    assert [op.kind for op in run.prog.ops] == [N.OP_COUNT, N.OP_SUM]
    assert math.isclose(run.prog.ops[0].scale[0], b_count, rel_tol=1e-12)
    assert math.isclose(run.prog.ops[1].scale[0], b_sum, rel_tol=1e-12)
    sel = run._selection()
    assert sel.strategy == N.SELECT_TRUNCATED_GEOMETRIC
    want = dpc.truncated_geometric_keep_table(1 / 3, 1e-6, 2)
    np.testing.assert_array_equal(np.asarray(sel.keep_prob), want)


def test_mean_gaussian_uses_normalised_sum():
    sink, _, _ = _graph(_params(metrics=[pdp.Metrics.MEAN, pdp.Metrics.COUNT, pdp.Metrics.SUM],
                                noise_kind=pdp.NoiseKind.GAUSSIAN))
    _, run = _run_of(sink)
    assert run.prog.flags == N.ACC_NSUM
    assert run.prog.middle == 5.0
    assert [op.kind for op in run.prog.ops] == [N.OP_MEAN]
    assert sorted(run.prog.fields) == ["count", "mean", "sum"]
    assert run.prog.ops[0].noise_kind == N.NOISE_GAUSSIAN


def test_variance_requests_three_sums():
    sink, _, _ = _graph(_params(metrics=[pdp.Metrics.VARIANCE, pdp.Metrics.PRIVACY_ID_COUNT],
                                min_value=-1.0, max_value=3.0))
    _, run = _run_of(sink)
    assert run.prog.flags == N.ACC_NSUM | N.ACC_NSUM2
    kinds = [op.kind for op in run.prog.ops]
    assert kinds == [N.OP_VARIANCE, N.OP_PRIVACY_ID_COUNT]
    assert run.prog.ops[0].sq_min_value == 0.0  # lo < 0 < hi: squares interval starts at 0


def test_privacy_id_count_alone_uses_cross_partition_bounder():
    sink, _, _ = _graph(_params(metrics=[pdp.Metrics.PRIVACY_ID_COUNT], min_value=None, max_value=None))
    plan, run = _run_of(sink)
    assert plan.bounder == "cross"
    spec = run._bounding_spec(N.VALUE_NONE)
    assert spec.linf == 0 and spec.flags == 0 and not run.prog.needs_values


def test_sum_per_partition_bounds():
    sink, _, _ = _graph(_params(metrics=[pdp.Metrics.SUM], min_value=None, max_value=None,
                                min_sum_per_partition=-3, max_sum_per_partition=9))
    plan, run = _run_of(sink)
    assert plan.bounder == "cross"
    spec = run._bounding_spec(N.VALUE_I64)
    assert spec.flags == N.SUM_PER_PARTITION | N.SUM_INT
    assert (spec.min_sum, spec.max_sum) == (-3.0, 9.0)


def test_public_partitions_select_public():
    sink, _, _ = _graph(_params(), public=[0, 1, 2, 99])
    plan, run = _run_of(sink)
    assert plan.public_keys is not None or plan.public_padding is not None
    assert run._selection().strategy == N.SELECT_PUBLIC


@pytest.mark.parametrize("strategy,code", [
    (pdp.PartitionSelectionStrategy.LAPLACE_THRESHOLDING, N.SELECT_LAPLACE_THRESHOLDING),
    (pdp.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING, N.SELECT_GAUSSIAN_THRESHOLDING),
])
def test_thresholding_strategies(strategy, code):
    sink, _, _ = _graph(_params(partition_selection_strategy=strategy, pre_threshold=3))
    _, run = _run_of(sink)
    sel = run._selection()
    assert sel.strategy == code and sel.pre_threshold == 3
    assert sel.threshold > 1.0 and sel.noise_scale > 0.0


def test_post_aggregation_thresholding():
    sink, _, _ = _graph(_params(metrics=[pdp.Metrics.COUNT, pdp.Metrics.PRIVACY_ID_COUNT],
                                post_aggregation_thresholding=True,
                                partition_selection_strategy=pdp.PartitionSelectionStrategy.LAPLACE_THRESHOLDING))
    plan, run = _run_of(sink)
    assert plan.threshold_drop
    assert run.prog.threshold_combiner is not None
    assert run.prog.ops[-1].kind == N.OP_THRESHOLDED_PID
    assert run._selection().strategy == N.SELECT_LAPLACE_THRESHOLDING


_MODES = {  # AggregateParams kwargs -> (plan.bounder, l0, linf, max_contributions, rows_are_units)
    "linf": (dict(perform_cross_partition_contribution_bounding=False), ("linf", 0, 3, 0, False)),
    "noop": (dict(metrics=[pdp.Metrics.SUM], min_value=None, max_value=None, min_sum_per_partition=-3.0,
                  max_sum_per_partition=9.0, perform_cross_partition_contribution_bounding=False),
             ("noop", 0, 0, 0, False)),
    "per_privacy_id": (dict(max_contributions=3, max_partitions_contributed=None,
                            max_contributions_per_partition=None), ("per_privacy_id", 0, 0, 3, False)),
    "already_enforced": (dict(contribution_bounds_already_enforced=True),
                         ("already_enforced", 0, 0, 0, True)),
}


@pytest.mark.parametrize("mode", sorted(_MODES))
def test_bounding_modes_recognised(mode):
    """Every bounder DPEngine can pick (dp_engine.py:380-400, and the
    contribution_bounds_already_enforced branch :143-150) maps to one kernel
    configuration (pdp_pairs.hip for all but Cross+Per / Cross)."""
    kw, (bounder, l0, linf, maxc, units) = _MODES[mode]
    public = [0, 1, 2, 3] if mode == "per_privacy_id" else None  # PyDP needs l0 for private selection
    sink, _, _ = _graph(_params(**kw), public=public)
    plan, run = _run_of(sink)
    assert plan.bounder == bounder
    spec = run._bounding_spec(N.VALUE_F64)
    assert (spec.l0, spec.linf, spec.max_contributions, spec.rows_are_units) == (l0, linf, maxc, units)


@pytest.mark.parametrize("mode", sorted(_MODES))
def test_reference_dpengine_bounding_modes_recognised(mode):
    """The reference's own DPEngine builds the same bounder stages."""
    pipeline_dp = _import_reference()
    kw, (bounder, l0, linf, maxc, units) = _MODES[mode]
    base = dict(metrics=[pipeline_dp.Metrics.COUNT, pipeline_dp.Metrics.SUM],
                noise_kind=pipeline_dp.NoiseKind.LAPLACE, max_partitions_contributed=2,
                max_contributions_per_partition=3, min_value=0.0, max_value=10.0)
    for k, v in kw.items():
        base[k] = [getattr(pipeline_dp.Metrics, m.name) for m in v] if k == "metrics" else v
    params = pipeline_dp.AggregateParams(**base)
    acc = pipeline_dp.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
    engine = pipeline_dp.DPEngine(acc, CB.ColumnarBackend())
    pid = None if units else (lambda r: r[0])
    ext = pipeline_dp.DataExtractors(privacy_id_extractor=pid, partition_extractor=lambda r: r[1],
                                     value_extractor=lambda r: r[2])
    public = [0, 1, 2, 3] if mode == "per_privacy_id" else None
    sink = engine.aggregate(ROWS, params, ext, public_partitions=public)
    acc.compute_budgets()
    plan, run = _run_of(sink)
    assert plan.bounder == bounder
    spec = run._bounding_spec(N.VALUE_F64)
    assert (spec.l0, spec.linf, spec.max_contributions, spec.rows_are_units) == (l0, linf, maxc, units)


def test_unrecognised_graph_raises():
    backend = CB.ColumnarBackend()
    col = backend.map([1, 2, 3], lambda x: x, "some other pipeline")
    with pytest.raises(NotImplementedError):
        CB.recognise(col)


@pytest.mark.parametrize("kw", [
    dict(metrics=[pdp.Metrics.SUM], min_value=None, max_value=None),     # bounds required
    dict(max_partitions_contributed=0),
    dict(max_contributions_per_partition=-1),
    dict(min_value=5.0, max_value=1.0),
])
def test_invalid_params_raise_like_reference(kw):
    with pytest.raises((ValueError, TypeError)):
        _graph(_params(**kw))


def test_execution_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    sink, _, _ = _graph(_params())
    with pytest.raises((RuntimeError, N.NativeLibraryError)):
        list(sink)


def test_explain_report_lists_columnar_stages():
    sink, engine, _ = _graph(_params())
    report = engine.explain_computations_report()[0]
    assert "DPEngine method: aggregate" in report
    assert "Cross-partition contribution bounding" in report
    assert "Private Partition selection" in report


def _import_reference():
    if not os.path.isdir(os.path.join(REFERENCE, "pipeline_dp")):
        pytest.skip("reference checkout not present")
    for p in (os.path.join(ROOT, "oracle", "pydp_standin"), REFERENCE):
        if p not in sys.path:
            sys.path.append(p)
    import pipeline_dp
    return pipeline_dp


def test_reference_dpengine_drives_columnar_backend():
    """The reference's own DPEngine, unchanged, builds a graph ColumnarBackend
    recognises: same bounding, selection and noise configuration as the mirror."""
    pipeline_dp = _import_reference()
    rp = pipeline_dp.AggregateParams(metrics=[pipeline_dp.Metrics.COUNT, pipeline_dp.Metrics.SUM,
                                              pipeline_dp.Metrics.MEAN],
                                     noise_kind=pipeline_dp.NoiseKind.LAPLACE, max_partitions_contributed=8,
                                     max_contributions_per_partition=2, min_value=0.0, max_value=10.0)
    acc = pipeline_dp.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
    engine = pipeline_dp.DPEngine(acc, CB.ColumnarBackend())
    ext = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                                     value_extractor=lambda r: r[2])
    sink = engine.aggregate(ROWS, rp, ext)
    acc.compute_budgets()
    plan, run = _run_of(sink)
    assert plan.bounder == "cross_and_per"
    spec = run._bounding_spec(N.VALUE_F64)
    assert (spec.l0, spec.linf, spec.flags) == (8, 2, N.ACC_NSUM)
    assert [op.kind for op in run.prog.ops] == [N.OP_MEAN]
    b_count = dpc.laplace_diversity(1 / 3, 8 * 2)
    b_nsum = dpc.laplace_diversity(1 / 3, 8 * 5.0 * 2)
    assert math.isclose(run.prog.ops[0].scale[0], b_count, rel_tol=1e-12)
    assert math.isclose(run.prog.ops[0].scale[1], b_nsum, rel_tol=1e-12)
    assert run._selection().strategy == N.SELECT_TRUNCATED_GEOMETRIC


@pytest.mark.parametrize("case", ["variance_gaussian", "public", "pid_count_threshold", "sum_per_partition"])
def test_reference_dpengine_variants_recognised(case):
    """C4-style VARIANCE + PRIVACY_ID_COUNT (Gaussian), public partitions,
    post-aggregation thresholding and per-partition SUM bounds, all built by
    the reference's DPEngine, map to the same kernel configuration as the
    mirror's DPEngine."""
    pipeline_dp = _import_reference()
    M = pipeline_dp.Metrics
    public = None
    if case == "variance_gaussian":
        kw = dict(metrics=[M.VARIANCE, M.PRIVACY_ID_COUNT], noise_kind=pipeline_dp.NoiseKind.GAUSSIAN,
                  max_partitions_contributed=4, max_contributions_per_partition=2, min_value=0.0, max_value=10.0)
    elif case == "public":
        kw = dict(metrics=[M.COUNT, M.SUM], noise_kind=pipeline_dp.NoiseKind.LAPLACE,
                  max_partitions_contributed=2, max_contributions_per_partition=1, min_value=1, max_value=5)
        public = [0, 3, 5, 42]
    elif case == "pid_count_threshold":
        kw = dict(metrics=[M.COUNT, M.PRIVACY_ID_COUNT], noise_kind=pipeline_dp.NoiseKind.LAPLACE,
                  max_partitions_contributed=2, max_contributions_per_partition=1,
                  post_aggregation_thresholding=True,
                  partition_selection_strategy=pipeline_dp.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING)
    else:
        kw = dict(metrics=[M.SUM], noise_kind=pipeline_dp.NoiseKind.LAPLACE, max_partitions_contributed=2,
                  max_contributions_per_partition=1, min_sum_per_partition=-3, max_sum_per_partition=9)

    def plan_for(mod, params):
        acc = mod.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
        engine = mod.DPEngine(acc, CB.ColumnarBackend())
        ext = mod.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                                 value_extractor=lambda r: r[2])
        sink = engine.aggregate(ROWS, params, ext, public_partitions=public)
        acc.compute_budgets()
        return _run_of(sink)

    def ours_kw():
        conv = {}
        for k, v in kw.items():
            if k == "metrics":
                conv[k] = [getattr(pdp.Metrics, m.name) for m in v]
            elif k == "noise_kind":
                conv[k] = pdp.NoiseKind(v.value)
            elif k == "partition_selection_strategy":
                conv[k] = pdp.PartitionSelectionStrategy(v.value)
            else:
                conv[k] = v
        return conv

    ref_plan, ref_run = plan_for(pipeline_dp, pipeline_dp.AggregateParams(**kw))
    our_plan, our_run = plan_for(pdp, pdp.AggregateParams(**ours_kw()))
    vk = N.VALUE_I64 if case in ("public", "sum_per_partition") else N.VALUE_F64
    assert ref_plan.bounder == our_plan.bounder
    assert vars(ref_run._bounding_spec(vk)) == vars(our_run._bounding_spec(vk))
    assert [o.as_dict() for o in ref_run.prog.ops] == [o.as_dict() for o in our_run.prog.ops]
    assert ref_run.prog.fields == our_run.prog.fields
    rs, os_ = ref_run._selection(), our_run._selection()
    assert (rs.strategy, rs.pre_threshold, rs.threshold, rs.noise_scale) == \
        (os_.strategy, os_.pre_threshold, os_.threshold, os_.noise_scale)


@pytest.mark.parametrize("engine_name", ["mirror", "reference"])
def test_select_partitions_recognised(engine_name):
    """DPEngine.select_partitions (dp_engine.py:212-288) maps to the Cross
    bounder (L0 sampling, no values) + private selection, keys out."""
    mod = pdp if engine_name == "mirror" else _import_reference()
    acc = mod.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
    engine = mod.DPEngine(acc, CB.ColumnarBackend())
    ext = mod.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1])
    params = mod.SelectPartitionsParams(
        max_partitions_contributed=4,
        partition_selection_strategy=mod.PartitionSelectionStrategy.LAPLACE_THRESHOLDING, pre_threshold=2)
    sink = engine.select_partitions(ROWS, params, ext)
    acc.compute_budgets()
    plan, run = _run_of(sink)
    assert plan.keys_only and plan.bounder == "cross"
    spec = run._bounding_spec(N.VALUE_NONE)
    assert (spec.l0, spec.linf, spec.flags) == (4, 0, 0)
    assert run.prog.ops == [] and not run.prog.needs_values
    sel = run._selection()
    assert sel.strategy == N.SELECT_LAPLACE_THRESHOLDING and sel.pre_threshold == 2
    # the whole budget goes to selection: b = l0 / eps
    assert math.isclose(sel.noise_scale, 4.0, rel_tol=1e-12)


def test_select_partitions_validation_like_reference():
    engine = pdp.DPEngine(pdp.NaiveBudgetAccountant(1.0, 1e-6), CB.ColumnarBackend())
    ext = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1])
    with pytest.raises(ValueError):
        engine.select_partitions(ROWS, pdp.SelectPartitionsParams(max_partitions_contributed=0), ext)
    with pytest.raises(TypeError):
        engine.select_partitions(ROWS, _params(), ext)
    with pytest.raises(ValueError):
        engine.select_partitions([], pdp.SelectPartitionsParams(max_partitions_contributed=1), ext)


@pytest.mark.parametrize("engine_name", ["mirror", "reference"])
@pytest.mark.parametrize("kind", ["laplace", "gaussian"])
def test_add_dp_noise_recognised(engine_name, kind):
    """DPEngine.add_dp_noise (dp_engine.py:551-607) maps to one noise kernel
    over the value column with the mechanism its lambda closes over:
    Laplace b = l0*linf/eps, Gaussian sigma = calibrate(eps, delta, sqrt(l0)*linf)."""
    mod = pdp if engine_name == "mirror" else _import_reference()
    acc = mod.NaiveBudgetAccountant(total_epsilon=2.0, total_delta=1e-6)
    engine = mod.DPEngine(acc, CB.ColumnarBackend())
    nk = mod.NoiseKind.LAPLACE if kind == "laplace" else mod.NoiseKind.GAUSSIAN
    params = mod.AddDPNoiseParams(noise_kind=nk, l0_sensitivity=3, linf_sensitivity=1.5)
    sink = engine.add_dp_noise([(k, float(k)) for k in range(10)], params)
    acc.compute_budgets()
    plan = CB.recognise(sink)
    assert isinstance(plan, CB.NoisePlan)
    noise = CB.noise_mechanism_of(plan.noise_fn)
    code, scale = noise.kind, noise.scale
    if kind == "laplace":
        assert code == N.NOISE_LAPLACE and math.isclose(scale, 3 * 1.5 / 2.0, rel_tol=1e-12)
        assert noise == dpc.laplace_noise_params(2.0, 3 * 1.5)
    else:
        assert code == N.NOISE_GAUSSIAN
        assert math.isclose(scale, dpc.compute_sigma(2.0, 1e-6, math.sqrt(3) * 1.5), rel_tol=1e-12)
        assert noise == dpc.gaussian_noise_params(scale)


def test_add_dp_noise_validation_like_reference():
    with pytest.raises(ValueError):
        pdp.AddDPNoiseParams(noise_kind=pdp.NoiseKind.LAPLACE, l0_sensitivity=0, linf_sensitivity=1.0)
    with pytest.raises(ValueError):
        pdp.AddDPNoiseParams(noise_kind=pdp.NoiseKind.LAPLACE, l0_sensitivity=1, linf_sensitivity=-1.0)


def test_add_dp_noise_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    acc = pdp.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
    engine = pdp.DPEngine(acc, CB.ColumnarBackend())
    sink = engine.add_dp_noise([(0, 1.0)], pdp.AddDPNoiseParams(noise_kind=pdp.NoiseKind.LAPLACE,
                                                                 l0_sensitivity=1, linf_sensitivity=1.0))
    acc.compute_budgets()
    with pytest.raises(RuntimeError):
        list(sink)
