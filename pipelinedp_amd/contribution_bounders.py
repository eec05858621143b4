"""Contribution bounders (mirror of pipeline_dp/contribution_bounders.py).

Each bounder expresses its sampling as PipelineBackend calls with the
reference's stage names; ColumnarBackend recognises those names and runs the
sampling in the HIP bounding kernels (csrc/pdp_bound.hip) instead of calling
the lambdas below row by row.
"""
import abc
import collections
from typing import Callable

import numpy as np


def choose_from_list_without_replacement(a: list, size: int) -> list:
    """sampling_utils.py:19-29: a uniform sample of `size` elements."""
    if len(a) <= size:
        return a
    picked = np.random.choice(np.arange(len(a)), size, replace=False)
    return [a[i] for i in picked]


class ContributionBounder(abc.ABC):

    @abc.abstractmethod
    def bound_contributions(self, col, params, backend, report_generator, aggregate_fn: Callable):
        """(privacy_id, partition_key, value) -> ((privacy_id, partition_key), accumulator)."""


class SamplingCrossAndPerPartitionContributionBounder(ContributionBounder):
    """<= max_contributions_per_partition rows per (pid, pk) and
    <= max_partitions_contributed partitions per pid (reference :62-111)."""

    def bound_contributions(self, col, params, backend, report_generator, aggregate_fn):
        l0, linf = params.max_partitions_contributed, params.max_contributions_per_partition
        col = backend.map_tuple(col, lambda pid, pk, v: ((pid, pk), v),
                                "Rekey to ( (privacy_id, partition_key), value))")
        col = backend.sample_fixed_per_key(col, linf, "Sample per (privacy_id, partition_key)")
        report_generator.add_stage(
            f"Per-partition contribution bounding: for each privacy_id and each partition, randomly "
            f"select max(actual_contributions_per_partition, {linf}) contributions.")
        col = backend.map_values(col, aggregate_fn, "Apply aggregate_fn after per partition bounding")
        col = backend.map_tuple(col, lambda pid_pk, acc: (pid_pk[0], (pid_pk[1], acc)),
                                "Rekey to (privacy_id, (partition_key, accumulator))")
        col = backend.sample_fixed_per_key(col, l0, "Sample per privacy_id")
        report_generator.add_stage(
            f"Cross-partition contribution bounding: for each privacy_id randomly select "
            f"max(actual_partition_contributed, {l0}) partitions")
        return backend.flat_map(col, lambda kv: (((kv[0], pk), acc) for pk, acc in kv[1]),
                                "Rekey by privacy_id and unnest")


def collect_values_per_partition_key_per_privacy_id(col, backend):
    """(pid, [(pk, v)]) -> (pid, [(pk, [v])]) (reference :249-276)."""

    def collect(items):
        groups = collections.defaultdict(list)
        for pk, v in items:
            groups[pk].append(v)
        return list(groups.items())

    return backend.map_values(col, collect, "Collect values per privacy_id and partition_key")


def _unnest(kv):
    pid, partitions = kv
    for pk, values in partitions:
        yield (pid, pk), values


class SamplingPerPrivacyIdContributionBounder(ContributionBounder):
    """<= max_contributions rows per pid overall (reference :114-156)."""

    def bound_contributions(self, col, params, backend, report_generator, aggregate_fn):
        n = params.max_contributions
        col = backend.map_tuple(col, lambda pid, pk, v: (pid, (pk, v)),
                                "Rekey to ((privacy_id), (partition_key, value))")
        col = backend.sample_fixed_per_key(col, n, "Sample per privacy_id")
        report_generator.add_stage(
            f"User contribution bounding: randomly selected not more than {n} contributions")
        col = collect_values_per_partition_key_per_privacy_id(col, backend)
        col = backend.flat_map(col, _unnest, "Unnest")
        return backend.map_values(col, aggregate_fn,
                                  "Apply aggregate_fn after per privacy_id contribution bounding")


class SamplingCrossPartitionContributionBounder(ContributionBounder):
    """<= max_partitions_contributed partitions per pid, every row of a kept
    partition (reference :159-201)."""

    def bound_contributions(self, col, params, backend, report_generator, aggregate_fn):
        col = backend.map_tuple(col, lambda pid, pk, v: (pid, (pk, v)),
                                "Rekey to ((privacy_id), (partition_key, value))")
        col = backend.group_by_key(col, "Group by privacy_id")
        col = collect_values_per_partition_key_per_privacy_id(col, backend)
        l0 = params.max_partitions_contributed
        col = backend.map_values(col, lambda a: choose_from_list_without_replacement(a, l0), "Sample")
        col = backend.flat_map(col, _unnest, "Unnest per privacy_id")
        return backend.map_values(col, aggregate_fn,
                                  "Apply aggregate_fn after cross-partition contribution bounding")


class LinfSampler(ContributionBounder):
    """Per-partition sampling only (reference :204-230)."""

    def bound_contributions(self, col, params, backend, report_generator, aggregate_fn):
        linf = params.max_contributions_per_partition
        col = backend.map_tuple(col, lambda pid, pk, v: ((pid, pk), v),
                                "Rekey to ((privacy_id, partition_key), value)")
        col = backend.sample_fixed_per_key(col, linf, "Sample per (privacy_id, partition_key)")
        report_generator.add_stage(
            f"Per-partition contribution bounding: for each privacy_id and each partition, randomly "
            f"select max(actual_contributions_per_partition, {linf}) contributions.")
        return backend.map_values(col, aggregate_fn,
                                  "Apply aggregate_fn after cross-partition contribution bounding")


class NoOpSampler(ContributionBounder):
    """Grouping only (reference :233-246)."""

    def bound_contributions(self, col, params, backend, report_generator, aggregate_fn):
        col = backend.map_tuple(col, lambda pid, pk, v: ((pid, pk), v),
                                "Rekey to ((privacy_id, partition_key), value)")
        col = backend.group_by_key(col, "Group by (privacy_id, partition_key)")
        return backend.map_values(col, aggregate_fn, "Apply aggregate_fn")
