"""Parameter objects of the aggregate path (mirror of the reference API).

Same names, fields, defaults and validation rules as
pipeline_dp/aggregate_params.py (reference): Metric/Metrics (:28-72),
NoiseKind (:75-83), PartitionSelectionStrategy (:86-89), MechanismType
(:92-117), AggregateParams (:189-395), SelectPartitionsParams (:398-425),
AddDPNoiseParams (:645-675), parameters_to_readable_string (:707-738).
"""
import dataclasses
import enum
import logging
import math
from typing import Any, Callable, List, Optional, Sequence

import numpy as np


def validate_epsilon_delta(epsilon: float, delta: float, obj_name: str):
    """input_validators.py:17-34."""
    if epsilon <= 0:
        raise ValueError(f"{obj_name}: epsilon must be positive, not {epsilon}.")
    if delta < 0:
        raise ValueError(f"{obj_name}: delta must be non-negative, not {delta}.")
    if delta >= 1:
        raise ValueError(f"{obj_name}: delta must be less than 1, not {delta}.")


@dataclasses.dataclass
class Metric:
    """A DP metric: a name plus an optional parameter (percentile rank)."""
    name: str
    parameter: Optional[float] = None

    def __eq__(self, other) -> bool:
        return isinstance(other, Metric) and (self.name, self.parameter) == (other.name, other.parameter)

    def __str__(self):
        return self.name if self.parameter is None else f"{self.name}({self.parameter})"

    __repr__ = __str__

    def __hash__(self):
        return hash(str(self))

    @property
    def is_percentile(self) -> bool:
        return self.name == "PERCENTILE"


class Metrics:
    COUNT = Metric("COUNT")
    PRIVACY_ID_COUNT = Metric("PRIVACY_ID_COUNT")
    SUM = Metric("SUM")
    MEAN = Metric("MEAN")
    VARIANCE = Metric("VARIANCE")
    VECTOR_SUM = Metric("VECTOR_SUM")

    @classmethod
    def PERCENTILE(cls, percentile_to_compute: float) -> Metric:
        return Metric("PERCENTILE", percentile_to_compute)


class NoiseKind(enum.Enum):
    LAPLACE = "laplace"
    GAUSSIAN = "gaussian"

    def convert_to_mechanism_type(self) -> "MechanismType":
        return {"laplace": MechanismType.LAPLACE, "gaussian": MechanismType.GAUSSIAN}[self.value]


class PartitionSelectionStrategy(enum.Enum):
    TRUNCATED_GEOMETRIC = "Truncated Geometric"
    LAPLACE_THRESHOLDING = "Laplace Thresholding"
    GAUSSIAN_THRESHOLDING = "Gaussian Thresholding"


class MechanismType(enum.Enum):
    LAPLACE = "Laplace"
    GAUSSIAN = "Gaussian"
    LAPLACE_THRESHOLDING = "Laplace Thresholding"
    GAUSSIAN_THRESHOLDING = "Gaussian Thresholding"
    GENERIC = "Generic"

    def to_noise_kind(self) -> NoiseKind:
        kinds = {
            "Laplace": NoiseKind.LAPLACE,
            "Gaussian": NoiseKind.GAUSSIAN,
            "Laplace Thresholding": NoiseKind.LAPLACE,
            "Gaussian Thresholding": NoiseKind.GAUSSIAN,
        }
        if self.value not in kinds:
            raise ValueError(f"MechanismType {self.value} can not be converted to NoiseKind")
        return kinds[self.value]

    def to_partition_selection_strategy(self) -> PartitionSelectionStrategy:
        strategies = {
            "Laplace Thresholding": PartitionSelectionStrategy.LAPLACE_THRESHOLDING,
            "Gaussian Thresholding": PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING,
        }
        if self.value not in strategies:
            raise ValueError(f"MechanismType {self.value} can not be converted to "
                             f"PartitionSelectionStrategy")
        return strategies[self.value]


def noise_to_thresholding(noise_kind: NoiseKind) -> MechanismType:
    if noise_kind == NoiseKind.LAPLACE:
        return MechanismType.LAPLACE_THRESHOLDING
    if noise_kind == NoiseKind.GAUSSIAN:
        return MechanismType.GAUSSIAN_THRESHOLDING
    raise ValueError(f"NoiseKind {noise_kind} can not be converted to Thresholding mechanism")


class NormKind(enum.Enum):
    Linf = "linf"
    L0 = "l0"
    L1 = "l1"
    L2 = "l2"


def _is_int(value: Any) -> bool:
    return isinstance(value, (int, np.integer)) and not isinstance(value, bool)


def _require_positive_int(value: Any, field_name: str):
    if not (_is_int(value) and value > 0):
        raise ValueError(f"{field_name} has to be positive integer, but {value} given.")


def _not_finite(num: Any) -> bool:
    return math.isnan(num) or math.isinf(num)


@dataclasses.dataclass
class AggregateParams:
    """Parameters of DPEngine.aggregate (reference aggregate_params.py:189-395)."""
    metrics: List[Metric]
    noise_kind: NoiseKind = NoiseKind.LAPLACE
    max_partitions_contributed: Optional[int] = None
    max_contributions_per_partition: Optional[int] = None
    max_contributions: Optional[int] = None
    budget_weight: float = 1
    min_value: Optional[float] = None
    max_value: Optional[float] = None
    min_sum_per_partition: Optional[float] = None
    max_sum_per_partition: Optional[float] = None
    custom_combiners: Sequence[Any] = None
    vector_norm_kind: Optional[NormKind] = None
    vector_max_norm: Optional[float] = None
    vector_size: Optional[int] = None
    contribution_bounds_already_enforced: bool = False
    public_partitions_already_filtered: bool = False
    partition_selection_strategy: PartitionSelectionStrategy = PartitionSelectionStrategy.TRUNCATED_GEOMETRIC
    pre_threshold: Optional[int] = None
    post_aggregation_thresholding: bool = False
    perform_cross_partition_contribution_bounding: bool = True

    @property
    def metrics_str(self) -> str:
        if self.custom_combiners:
            return f"custom combiners={[c.metrics_names() for c in self.custom_combiners]}"
        if self.metrics:
            return f"metrics={[str(m) for m in self.metrics]}"
        return "metrics=[]"

    @property
    def bounds_per_contribution_are_set(self) -> bool:
        return self.min_value is not None and self.max_value is not None

    @property
    def bounds_per_partition_are_set(self) -> bool:
        return self.min_sum_per_partition is not None and self.max_sum_per_partition is not None

    def __post_init__(self):
        for lo_name, hi_name in (("min_value", "max_value"),
                                 ("min_sum_per_partition", "max_sum_per_partition")):
            if (getattr(self, lo_name) is None) != (getattr(self, hi_name) is None):
                raise ValueError(f"AggregateParams: {lo_name} and {hi_name} should"
                                 f" be both set or both None.")
        value_bound = self.min_value is not None
        partition_bound = self.min_sum_per_partition is not None
        if value_bound and partition_bound:
            raise ValueError("min_value and min_sum_per_partition can not be both set.")
        if value_bound:
            self._check_range("min_value", "max_value")
        if partition_bound:
            self._check_range("min_sum_per_partition", "max_sum_per_partition")
        if self.metrics:
            self._check_metrics(value_bound, partition_bound)
        if self.custom_combiners:
            logging.warning("Warning: custom combiners are used. This is an experimental feature. "
                            "It might not work properly and it might be changed or removed "
                            "without any notifications.")
        if self.metrics and self.custom_combiners:
            raise ValueError("Custom combiners can not be used with standard metrics")
        self._check_contribution_bounds()
        if self.pre_threshold is not None:
            _require_positive_int(self.pre_threshold, "pre_threshold")

    def _check_metrics(self, value_bound: bool, partition_bound: bool):
        metrics = set(self.metrics)
        if Metrics.VECTOR_SUM in metrics:
            if metrics & {Metrics.SUM, Metrics.MEAN, Metrics.VARIANCE}:
                raise ValueError("AggregateParams: vector sum can not be computed together "
                                 "with scalar metrics such as sum, mean etc")
        elif partition_bound:
            bad = metrics - {Metrics.SUM, Metrics.PRIVACY_ID_COUNT, Metrics.COUNT}
            if bad:
                raise ValueError(f"AggregateParams: min_sum_per_partition is not compatible "
                                 f"with metrics {bad}. Please use min_value/max_value.")
        elif not value_bound:
            bad = metrics - {Metrics.PRIVACY_ID_COUNT, Metrics.COUNT}
            if bad:
                raise ValueError(f"AggregateParams: for metrics {bad} bounds per partition are "
                                 f"required (e.g. min_value,max_value).")
        if self.contribution_bounds_already_enforced and Metrics.PRIVACY_ID_COUNT in metrics:
            raise ValueError("AggregateParams: Cannot calculate PRIVACY_ID_COUNT when "
                             "contribution_bounds_already_enforced is set to True.")

    def _check_contribution_bounds(self):
        l0, linf = self.max_partitions_contributed, self.max_contributions_per_partition
        if self.max_contributions is not None:
            _require_positive_int(self.max_contributions, "max_contributions")
            if l0 is not None or linf is not None:
                raise ValueError("AggregateParams: only one in max_contributions or both "
                                 "max_partitions_contributed and max_contributions_per_partition "
                                 "must be set")
            return
        n_set = (l0 is not None) + (linf is not None)
        if n_set == 0:
            raise ValueError("AggregateParams: either max_contributions must be set or both "
                             "max_partitions_contributed and max_contributions_per_partition "
                             "must be set.")
        if n_set == 1:
            raise ValueError("AggregateParams: either none or both max_partitions_contributed "
                             "and max_contributions_per_partition must be set.")
        _require_positive_int(l0, "max_partitions_contributed")
        _require_positive_int(linf, "max_contributions_per_partition")

    def _check_range(self, lo_name: str, hi_name: str):
        for name in (lo_name, hi_name):
            if _not_finite(getattr(self, name)):
                raise ValueError(f"AggregateParams: {name} must be a finite number")
        if getattr(self, lo_name) > getattr(self, hi_name):
            raise ValueError(f"AggregateParams: {hi_name} must be equal to or greater than {lo_name}")

    def __str__(self):
        return parameters_to_readable_string(self)


@dataclasses.dataclass
class SelectPartitionsParams:
    """Parameters of DPEngine.select_partitions (reference :398-425)."""
    max_partitions_contributed: int
    budget_weight: float = 1
    partition_selection_strategy: PartitionSelectionStrategy = PartitionSelectionStrategy.TRUNCATED_GEOMETRIC
    pre_threshold: Optional[int] = None

    def __post_init__(self):
        if self.pre_threshold is not None:
            _require_positive_int(self.pre_threshold, "pre_threshold")

    def __str__(self):
        return "Private Partitions"


@dataclasses.dataclass
class AddDPNoiseParams:
    """Parameters of DPEngine.add_dp_noise (reference :645-675)."""
    noise_kind: NoiseKind
    l0_sensitivity: int
    linf_sensitivity: float
    budget_weight: float = 1

    def __post_init__(self):
        for name in ("l0_sensitivity", "linf_sensitivity", "budget_weight"):
            v = getattr(self, name)
            if v is not None and v <= 0:
                raise ValueError(f"{name} must be positive, but {v} given.")


def parameters_to_readable_string(params, is_public_partition: Optional[bool] = None) -> str:
    """Human-readable parameter block of the explain-computation report."""
    lines = [f"{type(params).__name__}:"]
    if hasattr(params, "metrics_str"):
        lines.append(f" {params.metrics_str}")
    if hasattr(params, "noise_kind"):
        lines.append(f" noise_kind={params.noise_kind.value}")
    if hasattr(params, "budget_weight"):
        lines.append(f" budget_weight={params.budget_weight}")
    lines.append(" Contribution bounding:")
    for name in ("max_partitions_contributed", "max_contributions_per_partition",
                 "max_contributions", "min_value", "max_value", "min_sum_per_partition",
                 "max_sum_per_partition"):
        if getattr(params, name, None) is not None:
            lines.append(f"  {name}={getattr(params, name)}")
    if getattr(params, "contribution_bounds_already_enforced", False):
        lines.append("  contribution_bounds_already_enforced=True")
    for name in ("vector_max_norm", "vector_size", "vector_norm_kind"):
        if getattr(params, name, None) is not None:
            lines.append(f"  {name}={getattr(params, name)}")
    if is_public_partition is not None:
        lines.append(f" Partition selection: {'public' if is_public_partition else 'private'} partitions")
    return "\n".join(lines)
