"""Partition selection strategies (mirror of pipeline_dp/partition_selection.py).

The reference maps PartitionSelectionStrategy to a PyDP strategy object
(partition_selection.py:19-44).  Here each strategy object holds the host-side
calibration (keep-probability table, noise scale, threshold) and exports the
parameters of the GPU selection kernel (``device_spec``); the per-partition
keep decisions and noise draws run in ``k_select`` (csrc/pdp_kernels.hip).
The host methods (should_keep etc.) exist for API parity and single values.
"""
from typing import Optional

import numpy as np

from pipelinedp_amd import _native as N
from pipelinedp_amd import aggregate_params as agg
from pipelinedp_amd import dp_computations as dpc

PARTITION_STRATEGY_ENUM_TO_STR = {
    agg.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC: "truncated_geometric",
    agg.PartitionSelectionStrategy.LAPLACE_THRESHOLDING: "laplace",
    agg.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING: "gaussian",
}


class PartitionSelectionStrategy:

    def __init__(self, epsilon: float, delta: float, max_partitions_contributed: int,
                 pre_threshold: Optional[int] = None):
        self.epsilon = epsilon
        self.delta = delta
        self.max_partitions_contributed = max_partitions_contributed
        self.pre_threshold = pre_threshold

    def _shifted(self, n: int) -> Optional[int]:
        if self.pre_threshold:
            return None if n < self.pre_threshold else n - (self.pre_threshold - 1)
        return n

    def device_spec(self, max_rows_per_privacy_id: int = 1):
        raise NotImplementedError


class TruncatedGeometricPartitionSelection(PartitionSelectionStrategy):

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._table = dpc.truncated_geometric_keep_table(self.epsilon, self.delta,
                                                         self.max_partitions_contributed)

    @property
    def keep_probability_table(self) -> np.ndarray:
        return self._table

    def probability_of_keep(self, n: int) -> float:
        m = self._shifted(n)
        if m is None or m <= 0:
            return 0.0
        return float(self._table[min(m, len(self._table) - 1)])

    def should_keep(self, n: int) -> bool:
        return bool(np.random.default_rng().random() < self.probability_of_keep(n))

    def device_spec(self, max_rows_per_privacy_id: int = 1):
        from pipelinedp_amd.executor import SelectionSpec
        return SelectionSpec(strategy=N.SELECT_TRUNCATED_GEOMETRIC,
                             max_rows_per_privacy_id=max_rows_per_privacy_id,
                             pre_threshold=self.pre_threshold or 0, keep_prob=self._table)


class _ThresholdingPartitionSelection(PartitionSelectionStrategy):
    """PyDP Laplace / GaussianPartitionSelection: keep iff the secure
    mechanism's AddNoise(n) exceeds the threshold (noise = `noise`, the
    mechanism with sensitivity l0 / sqrt(l0) and linf 1)."""
    _kernel_strategy = None
    noise_scale = 0.0
    threshold = 0.0
    noise: dpc.NoiseParams = dpc.NO_NOISE

    def noised_value_if_should_keep(self, n: int) -> Optional[float]:
        m = self._shifted(n)
        if m is None:
            return None
        v = dpc.secure_sampler().add_noise(self.noise, float(m))
        return v + (n - m) if v > self.threshold else None

    def should_keep(self, n: int) -> bool:
        return self.noised_value_if_should_keep(n) is not None

    def device_spec(self, max_rows_per_privacy_id: int = 1):
        from pipelinedp_amd.executor import SelectionSpec
        return SelectionSpec(strategy=self._kernel_strategy,
                             max_rows_per_privacy_id=max_rows_per_privacy_id,
                             pre_threshold=self.pre_threshold or 0, noise=self.noise,
                             threshold=self.threshold, want_noised_count=True)


class LaplacePartitionSelection(_ThresholdingPartitionSelection):
    _kernel_strategy = N.SELECT_LAPLACE_THRESHOLDING

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.noise_scale, self.threshold = dpc.laplace_thresholding_params(
            self.epsilon, self.delta, self.max_partitions_contributed)
        self.noise = dpc.laplace_noise_params(self.epsilon, self.max_partitions_contributed)


class GaussianPartitionSelection(_ThresholdingPartitionSelection):
    _kernel_strategy = N.SELECT_GAUSSIAN_THRESHOLDING

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.noise_scale, self.threshold = dpc.gaussian_thresholding_params(
            self.epsilon, self.delta, self.max_partitions_contributed)
        self.noise = dpc.gaussian_noise_params(self.noise_scale)


_CLASSES = {
    "truncated_geometric": TruncatedGeometricPartitionSelection,
    "laplace": LaplacePartitionSelection,
    "gaussian": GaussianPartitionSelection,
}


def create_partition_selection_strategy(strategy: agg.PartitionSelectionStrategy, epsilon: float,
                                        delta: float, max_partitions_contributed: int,
                                        pre_threshold: Optional[int] = None):
    """Same signature and meaning as the reference (partition_selection.py:29-44)."""
    return _CLASSES[PARTITION_STRATEGY_ENUM_TO_STR[strategy]](epsilon, delta,
                                                              max_partitions_contributed,
                                                              pre_threshold)
