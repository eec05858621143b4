"""DPEngine (mirror of pipeline_dp/dp_engine.py) for the aggregate path.

The engine only *describes* the computation: it validates parameters,
requests budgets and chains PipelineBackend calls with the reference's stage
names (dp_engine.py:109-187, contribution_bounders.py:72-111).  With
ColumnarBackend those calls are recorded and executed on the GPU; the same
engine drives any other PipelineBackend row-wise.
"""
import functools
from typing import Any, Callable, Optional, Tuple

from pipelinedp_amd import aggregate_params as agg
from pipelinedp_amd import budget_accounting
from pipelinedp_amd import combiners
from pipelinedp_amd import contribution_bounders
from pipelinedp_amd import data_extractors as de
from pipelinedp_amd import partition_selection
from pipelinedp_amd import report_generator


def _key_by(backend, col, key_fn: Callable, stage_name: str):
    """pipeline_functions.key_by (reference pipeline_functions.py:23-27)."""
    return backend.map(col, lambda el: (key_fn(el), el),
                       f"{stage_name}: key collection by keys from key extractor.")


def _require_col(col):
    if col is None or not col:
        raise ValueError("col must be non-empty")


def _require_extractors(data_extractors):
    if data_extractors is None:
        raise ValueError("data_extractors must be set to a DataExtractors")
    if not isinstance(data_extractors, de.DataExtractors):
        raise TypeError("data_extractors must be set to a DataExtractors")


class DPEngine:
    """Builds DP aggregations on a PipelineBackend."""

    def __init__(self, budget_accountant, backend):
        self._budget_accountant = budget_accountant
        self._backend = backend
        self._report_generators = []

    # -------------------------------------------------------- reports --
    @property
    def _current_report_generator(self):
        return self._report_generators[-1]

    def _add_report_generator(self, params, method_name: str, is_public_partition=None):
        self._report_generators.append(
            report_generator.ReportGenerator(params, method_name, is_public_partition))

    def _add_report_stage(self, stage_description):
        self._current_report_generator.add_stage(stage_description)

    def explain_computations_report(self):
        return [g.report() for g in self._report_generators]

    # ------------------------------------------------------ aggregate --
    def aggregate(self, col, params: agg.AggregateParams, data_extractors: de.DataExtractors,
                  public_partitions=None,
                  out_explain_computation_report: Optional[report_generator.ExplainComputationReport] = None):
        """DP metrics per partition: a lazy collection of (partition_key, MetricsTuple)."""
        self._check_aggregate_params(col, params, data_extractors)
        self._check_budget_accountant_compatibility(public_partitions is not None, params.metrics,
                                                    params.custom_combiners is not None)
        with self._budget_accountant.scope(weight=params.budget_weight):
            self._add_report_generator(params, "aggregate", public_partitions is not None)
            if out_explain_computation_report is not None:
                out_explain_computation_report._set_report_generator(self._current_report_generator)
            col = self._aggregate(col, params, data_extractors, public_partitions)
            budget = self._budget_accountant._compute_budget_for_aggregation(params.budget_weight)
            return self._annotate(col, params=params, budget=budget)

    def _aggregate(self, col, params, data_extractors, public_partitions):
        if params.custom_combiners:
            combiner = combiners.create_compound_combiner_with_custom_combiners(
                params, self._budget_accountant, params.custom_combiners)
        else:
            combiner = self._create_compound_combiner(params)
        backend = self._backend
        col = self._extract_columns(col, data_extractors)
        # (privacy_id, partition_key, value)
        if public_partitions is not None and not params.public_partitions_already_filtered:
            col = self._drop_partitions(col, public_partitions, lambda row: row[1])
            self._add_report_stage("Public partition selection: dropped non public partitions")
        if params.contribution_bounds_already_enforced:
            col = backend.map(col, lambda row: row[1:], "Remove privacy_id")
            col = backend.map_values(col, lambda value: combiner.create_accumulator([value]),
                                     "Wrap values into accumulators")
        else:
            bounder = self._create_contribution_bounder(params, combiner.expects_per_partition_sampling())
            col = bounder.bound_contributions(col, params, backend, self._current_report_generator,
                                              combiner.create_accumulator)
            # ((privacy_id, partition_key), accumulator)
            col = backend.map_tuple(col, lambda pid_pk, acc: (pid_pk[1], acc), "Drop privacy id")
        if public_partitions:
            col = self._add_empty_public_partitions(col, public_partitions, combiner.create_accumulator)
        col = backend.combine_accumulators_per_key(col, combiner, "Reduce accumulators per partition key")
        # (partition_key, accumulator)
        if public_partitions is None and not params.post_aggregation_thresholding:
            max_rows = 1
            if params.contribution_bounds_already_enforced:
                # one row is not necessarily one privacy unit (dp_engine.py:166-172)
                max_rows = params.max_contributions or params.max_contributions_per_partition
            col = self._select_private_partitions_internal(col, params.max_partitions_contributed, max_rows,
                                                           params.partition_selection_strategy,
                                                           params.pre_threshold)
        for stage in combiner.explain_computation():
            self._add_report_stage(stage)
        col = backend.map_values(col, combiner.compute_metrics, "Compute DP metrics")
        if params.post_aggregation_thresholding:
            col = self._drop_partitions_under_threshold(col)
        return col

    # ---------------------------------------------- select_partitions --
    def select_partitions(self, col, params: agg.SelectPartitionsParams, data_extractors: de.DataExtractors):
        """DP set of partition keys (reference dp_engine.py:212-233): per
        privacy id a uniform sample of <= max_partitions_contributed distinct
        partitions, privacy-id count per partition, private selection."""
        self._check_select_private_partitions(col, params, data_extractors)
        self._check_budget_accountant_compatibility(False, [], False)
        with self._budget_accountant.scope(weight=params.budget_weight):
            self._add_report_generator(params, "select_partitions")
            col = self._select_partitions(col, params, data_extractors)
            budget = self._budget_accountant._compute_budget_for_aggregation(params.budget_weight)
            return self._annotate(col, params=params, budget=budget)

    def _select_partitions(self, col, params: agg.SelectPartitionsParams, data_extractors: de.DataExtractors):
        """Stage chain of dp_engine.py:235-288 (ColumnarBackend runs it on the GPU)."""
        l0 = params.max_partitions_contributed
        backend = self._backend
        col = backend.map(col, lambda row: (data_extractors.privacy_id_extractor(row),
                                            data_extractors.partition_extractor(row)),
                          "Extract (privacy_id, partition_key))")
        col = backend.group_by_key(col, "Group by privacy_id")

        def sample_unique(pid_and_pks):
            pid, pks = pid_and_pks
            sampled = contribution_bounders.choose_from_list_without_replacement(list(set(pks)), l0)
            return ((pid, pk) for pk in sampled)

        col = backend.flat_map(col, sample_unique, "Sample cross-partition contributions")
        compound = combiners.CompoundCombiner([], return_named_tuple=False)
        col = backend.map_tuple(col, lambda pid, pk: (pk, compound.create_accumulator([])),
                                "Drop privacy id and add accumulator")
        col = backend.combine_accumulators_per_key(col, compound, "Combine accumulators per partition key")
        col = self._select_private_partitions_internal(col, l0, 1, params.partition_selection_strategy,
                                                       params.pre_threshold)
        return backend.keys(col, "Drop accumulators, keep only partition keys")

    def add_dp_noise(self, col, params: agg.AddDPNoiseParams, out_explain_computation_report=None):
        """Noise on pre-aggregated (partition_key, value) pairs (reference
        dp_engine.py:551-607): one budget request of params.noise_kind, then
        the "Add noise" map_values stage.  The sensitivities are the caller's
        (no contribution bounding).  With ColumnarBackend the stage runs as
        one GPU kernel over the value column (`pdp_add_noise`)."""
        from pipelinedp_amd import dp_computations
        mechanism_spec = self._budget_accountant.request_budget(params.noise_kind.convert_to_mechanism_type())
        sensitivities = dp_computations.Sensitivities(l0=params.l0_sensitivity, linf=params.linf_sensitivity)
        self._add_report_generator(params, "add_dp_noise", is_public_partition=True)
        if out_explain_computation_report is not None:
            out_explain_computation_report._set_report_generator(self._current_report_generator)

        def create_mechanism():
            return dp_computations.create_additive_mechanism(mechanism_spec, sensitivities)

        self._add_report_stage(lambda: f"Adding {create_mechanism().noise_kind} noise with "
                               f"parameter {create_mechanism().noise_parameter}")
        anonymized = self._backend.map_values(col, lambda value: create_mechanism().add_noise(float(value)),
                                              "Add noise")
        budget = self._budget_accountant._compute_budget_for_aggregation(params.budget_weight)
        return self._annotate(anonymized, params=params, budget=budget)

    def _check_select_private_partitions(self, col, params, data_extractors):
        """dp_engine.py:189-210."""
        _require_col(col)
        if params is None:
            raise ValueError("params must be set to a valid SelectPrivatePartitionsParams")
        if not isinstance(params, agg.SelectPartitionsParams):
            raise TypeError("params must be set to a valid SelectPrivatePartitionsParams")
        if not isinstance(params.max_partitions_contributed, int) or params.max_partitions_contributed <= 0:
            raise ValueError("params.max_partitions_contributed must be set (to a positive integer)")
        _require_extractors(data_extractors)

    def _extract_columns(self, col, data_extractors: de.DataExtractors):
        pid_fn = data_extractors.privacy_id_extractor or (lambda row: None)
        pk_fn = data_extractors.partition_extractor
        value_fn = data_extractors.value_extractor
        return self._backend.map(col, lambda row: (pid_fn(row), pk_fn(row), value_fn(row)),
                                 "Extract (privacy_id, partition_key, value))")

    def _drop_partitions(self, col, partitions, partition_extractor: Callable):
        col = _key_by(self._backend, col, partition_extractor, "Key by partition")
        col = self._backend.filter_by_key(col, partitions, "Filtering out partitions")
        return self._backend.values(col, "Drop key")

    def _add_empty_public_partitions(self, col, public_partitions, aggregator_fn):
        self._add_report_stage("Adding empty partitions for public partitions that are missing in data")
        public = self._backend.to_collection(public_partitions, col, "Public partitions to collection")
        empty = self._backend.map(public, lambda pk: (pk, aggregator_fn([])), "Build empty accumulators")
        return self._backend.flatten((col, empty), "Join public partitions with partitions from data")

    def _select_private_partitions_internal(self, col, max_partitions_contributed: int,
                                            max_rows_per_privacy_id: int,
                                            strategy: agg.PartitionSelectionStrategy,
                                            pre_threshold: Optional[int]):
        budget = self._budget_accountant.request_budget(mechanism_type=agg.MechanismType.GENERIC)
        # a partial (not a closure) so the function stays serialisable and
        # introspectable (dp_engine.py:360-364)
        keep_fn = functools.partial(_keep_partition, budget, max_partitions_contributed,
                                    max_rows_per_privacy_id, strategy, pre_threshold)
        pre_str = f", pre_threshold={pre_threshold}" if pre_threshold else ""
        self._add_report_stage(lambda: f"Private Partition selection: using {strategy.value} method with "
                                       f"(eps={budget.eps}, delta={budget.delta}{pre_str})")
        return self._backend.filter(col, keep_fn, "Filter private partitions")

    def _drop_partitions_under_threshold(self, col):
        self._add_report_stage("Drop partitions which have noised privacy_id_count less than threshold.")
        return self._backend.filter(col, lambda row: row[1].privacy_id_count is not None,
                                    "Drop partitions under threshold")

    def _create_compound_combiner(self, params):
        return combiners.create_compound_combiner(params, self._budget_accountant)

    def _create_contribution_bounder(self, params, expects_per_partition_sampling: bool):
        """dp_engine.py:380-400."""
        if params.max_contributions:
            return contribution_bounders.SamplingPerPrivacyIdContributionBounder()
        if params.perform_cross_partition_contribution_bounding:
            if expects_per_partition_sampling:
                return contribution_bounders.SamplingCrossAndPerPartitionContributionBounder()
            return contribution_bounders.SamplingCrossPartitionContributionBounder()
        if expects_per_partition_sampling:
            return contribution_bounders.LinfSampler()
        return contribution_bounders.NoOpSampler()

    # ----------------------------------------------------- validation --
    def _check_aggregate_params(self, col, params, data_extractors, check_data_extractors: bool = True):
        if params is not None and getattr(params, "max_contributions", None) is not None:
            allowed = {agg.Metrics.PRIVACY_ID_COUNT, agg.Metrics.COUNT, agg.Metrics.SUM, agg.Metrics.MEAN}
            bad = set(params.metrics) - allowed
            if bad:
                raise NotImplementedError(f"max_contributions is not supported for {bad}")
        _require_col(col)
        if params is None:
            raise ValueError("params must be set to a valid AggregateParams")
        if not isinstance(params, agg.AggregateParams):
            raise TypeError("params must be set to a valid AggregateParams")
        if check_data_extractors:
            _require_extractors(data_extractors)
        if params.contribution_bounds_already_enforced and agg.Metrics.PRIVACY_ID_COUNT in params.metrics:
            raise ValueError("PRIVACY_ID_COUNT cannot be computed when "
                             "contribution_bounds_already_enforced is True.")
        if params.post_aggregation_thresholding and agg.Metrics.PRIVACY_ID_COUNT not in params.metrics:
            raise ValueError("When post_aggregation_thresholding = True, PRIVACY_ID_COUNT must be in metrics")

    def _check_budget_accountant_compatibility(self, is_public_partition: bool, metrics,
                                               custom_combiner: bool) -> None:
        if isinstance(self._budget_accountant, budget_accounting.NaiveBudgetAccountant):
            return
        if not is_public_partition:
            raise NotImplementedError("PLD budget accounting does not support private partition selection")
        bad = set(metrics) - {agg.Metrics.COUNT, agg.Metrics.PRIVACY_ID_COUNT, agg.Metrics.SUM,
                              agg.Metrics.MEAN}
        if bad:
            raise NotImplementedError(f"Metrics {bad} do not support PLD budget accounting")
        if custom_combiner:
            raise ValueError("PLD budget accounting does not support custom combiners")

    def _annotate(self, col, params, budget):
        return self._backend.annotate(col, "annotation", params=params, budget=budget)


def _keep_partition(budget, max_partitions: int, max_rows_per_privacy_id: int, strategy,
                    pre_threshold: Optional[int], row: Tuple[Any, Any]) -> bool:
    """Row-wise private selection of one (partition_key, accumulator)
    (dp_engine.py:335-358): privacy units = ceil(row_count / max_rows)."""
    row_count, _ = row[1]
    n = (row_count + max_rows_per_privacy_id - 1) // max_rows_per_privacy_id
    selector = partition_selection.create_partition_selection_strategy(
        strategy, budget.eps, budget.delta, max_partitions, pre_threshold)
    return selector.should_keep(n)
