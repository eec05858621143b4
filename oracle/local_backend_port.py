"""TEST INFRASTRUCTURE — row-wise restatement of the reference's CPU path.

This is the reference's LocalBackend execution of DPEngine.aggregate
restated for the benchmark's metric set (COUNT + SUM + MEAN -> one MeanCombiner),
keeping the reference's execution model: single-threaded Python generators,
dict group-bys in insertion order (pipeline_backend.py:503-512), per-key
np.random.choice sampling (pipeline_backend.py:531-547), np.clip on each
(pid, pk)'s small list (combiners.py:474-480), functools.reduce merges
(pipeline_backend.py:555-565), a partition-selection strategy object per
partition (dp_engine.py:335-358) and per-partition noise
(dp_computations.py:562-568).  bench.py times it as the CPU baseline
("port", 1 core) because the reference itself never travels to the GPU box.
"""
import collections
import functools

import numpy as np

from oracle import pydp_restatement as pydp


def _group_by_key(col):
    groups = collections.defaultdict(list)
    for key, value in col:
        groups[key].append(value)
    yield from groups.items()


def _sample_fixed_per_key(col, n):
    for key, values in _group_by_key(col):
        if len(values) > n:
            picked = np.random.choice(range(len(values)), n, replace=False)
            values = [values[i] for i in picked]
        yield key, values


def aggregate_count_sum_mean(rows, *, l0, linf, min_value, max_value, eps, delta):
    """rows: iterable of (privacy_id, partition_key, value). Returns a list of
    (partition_key, (mean, count, sum)) for the kept partitions."""
    middle = min_value + (max_value - min_value) / 2
    eps_each = eps / 3  # MEAN count, MEAN normalized sum, GENERIC selection
    count_mech = pydp.LaplaceMechanism(eps_each, l0 * linf)
    nsum_mech = pydp.LaplaceMechanism(eps_each, l0 * linf * (max_value - min_value) / 2)

    def create_accumulator(values):
        normalized = np.clip(values, min_value, max_value) - middle
        return 1, ((len(values), normalized.sum()),)

    def merge(a, b):
        (ca, ((na, sa),)), (cb, ((nb, sb),)) = a, b
        return ca + cb, ((na + nb, sa + sb),)

    col = (((pid, pk), v) for pid, pk, v in rows)
    col = _sample_fixed_per_key(col, linf)
    col = ((key, create_accumulator(values)) for key, values in col)
    col = ((key[0], (key[1], acc)) for key, acc in col)
    col = _sample_fixed_per_key(col, l0)
    col = (((pid, pk), acc) for pid, pk_accs in col for pk, acc in pk_accs)
    col = ((pid_pk[1], acc) for pid_pk, acc in col)
    col = ((pk, functools.reduce(merge, accs)) for pk, accs in _group_by_key(col))

    def keep(item):
        row_count = item[1][0]
        strategy = pydp.create_partition_strategy("truncated_geometric", eps_each, delta, l0)
        return strategy.should_keep(row_count)

    out = []
    for pk, (_, ((count, nsum),)) in filter(keep, col):
        dp_count = count_mech.add_noise(count)
        dp_nsum = nsum_mech.add_noise(nsum)
        mean = middle + dp_nsum / max(1.0, dp_count)
        out.append((pk, (mean, dp_count, mean * dp_count)))
    return out
