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


def aggregate_count_sum(rows, *, l0, linf, min_value, max_value, eps, delta):
    """BASELINE config 1 (C1): COUNT + SUM on LocalBackend -- CountCombiner and
    SumCombiner under one CompoundCombiner (combiners.py:400-475), per-value
    clipping of SUM to [min_value, max_value], Laplace noise, private
    partitions (truncated geometric).  rows: iterable of (privacy_id,
    partition_key, value).  Returns [(partition_key, (count, sum))] kept."""
    eps_each = eps / 3  # COUNT, SUM, GENERIC selection
    count_mech = pydp.LaplaceMechanism(eps_each, l0 * linf)
    sum_mech = pydp.LaplaceMechanism(eps_each, l0 * linf * max(abs(min_value), abs(max_value)))

    def create_accumulator(values):
        return 1, (len(values), np.clip(values, min_value, max_value).sum())

    def merge(a, b):
        (ca, (na, sa)), (cb, (nb, sb)) = a, b
        return ca + cb, (na + nb, sa + sb)

    col = (((pid, pk), v) for pid, pk, v in rows)
    col = _sample_fixed_per_key(col, linf)
    col = ((key, create_accumulator(values)) for key, values in col)
    col = ((key[0], (key[1], acc)) for key, acc in col)
    col = _sample_fixed_per_key(col, l0)
    col = (((pid, pk), acc) for pid, pk_accs in col for pk, acc in pk_accs)
    col = ((pid_pk[1], acc) for pid_pk, acc in col)
    col = ((pk, functools.reduce(merge, accs)) for pk, accs in _group_by_key(col))

    def keep(item):
        strategy = pydp.create_partition_strategy("truncated_geometric", eps_each, delta, l0)
        return strategy.should_keep(item[1][0])

    return [(pk, (count_mech.add_noise(c), sum_mech.add_noise(sm))) for pk, (_, (c, sm)) in filter(keep, col)]


def movie_view_rows(n_rows=1_000_000, seed=0):
    """BASELINE config 1's synthetic movie_view rows:
    user_id uniform over [0, 1e5), movie_id = min(Zipf(1.3), 17,770), rating
    uniform over {1..5}; numpy.random.default_rng(seed)."""
    rng = np.random.default_rng(seed)
    user = rng.integers(0, 100_000, n_rows)
    movie = np.minimum(rng.zipf(1.3, n_rows), 17_770)
    rating = rng.integers(1, 6, n_rows)
    return list(zip(user.tolist(), movie.tolist(), rating.tolist()))

