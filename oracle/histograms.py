"""TEST INFRASTRUCTURE — NumPy restatement of the reference's dataset
histograms (pipeline_dp/dataset_histograms/computing_histograms.py).

Only tests/ may import this module, as the checker of the HIP path
(pipelinedp_amd/csrc/pdp_hist.hip); the product never does.  Pinned against
tests/golden/histograms/*.json, which the reference itself produced
(oracle/gen_golden_hist.py).

A bin is the tuple (lower, upper, count, sum, max) of hist.FrequencyBin
(histograms.py:21-57); a histogram is its list of bins sorted by lower
(computing_histograms.py:191-193).
"""
import numpy as np

NUMBER_OF_BUCKETS_SUM_HISTOGRAM = 10000  # computing_histograms.py:25

HIST_FIELDS = ("l0_contributions_histogram", "l1_contributions_histogram",
               "linf_contributions_histogram", "linf_sum_contributions_histogram",
               "count_per_partition_histogram", "count_privacy_id_per_partition",
               "sum_per_partition_histogram")


def log_bin(value: int):
    """_to_bin_lower_upper_logarithmic (computing_histograms.py:28-47): keep
    the 3 leading digits of value; the bin of 10^k is 10x wider."""
    bound = 1000
    while value > bound:
        bound *= 10
    round_base = bound // 1000
    lower = value // round_base * round_base
    return lower, lower + (round_base if value != bound else round_base * 10)


def frequency_histogram(values):
    """_compute_frequency_histogram (:62-78) + _compute_frequency_histogram_helper
    (:105-132) + _convert_frequency_bins_into_histogram (:176-195): per bin
    count = #elements, sum = sum of elements, max = max element."""
    values = np.asarray(values, dtype=np.int64)
    if values.size == 0:
        return []
    uniq, freq = np.unique(values, return_counts=True)
    bins = {}
    for v, f in zip(uniq.tolist(), freq.tolist()):
        lo, up = log_bin(v)
        b = bins.get(lo)
        bins[lo] = (lo, up, f, f * v, v) if b is None else (lo, up, b[2] + f, b[3] + f * v, max(b[4], v))
    return [bins[k] for k in sorted(bins)]


def min_max_lowers(values, number_of_buckets=NUMBER_OF_BUCKETS_SUM_HISTOGRAM):
    """_min_max_lowers (:346-370)."""
    mn, mx = float(np.min(values)), float(np.max(values))
    if mn == mx:
        return [mn, mn]
    return list(np.linspace(mn, mx, number_of_buckets + 1))


def float_histogram(values):
    """_compute_frequency_histogram_helper_with_lowers (:135-173) with
    _bin_lower_index (:50-59): bisect_right over the lowers, the maximum goes
    to the last bin."""
    values = np.asarray(values, dtype=np.float64)
    if values.size == 0:
        return []
    lowers = np.asarray(min_max_lowers(values))
    idx = np.searchsorted(lowers, values, side="right") - 1
    idx[values == lowers[-1]] = len(lowers) - 2
    out = []
    for i in np.unique(idx).tolist():
        sel = values[idx == i]
        out.append((float(lowers[i]), float(lowers[i + 1]), int(sel.size), float(sel.sum()), float(sel.max())))
    return out


def dataset_histograms(pid, pk, value):
    """compute_dataset_histograms (computing_histograms.py:456-513) over
    columns of dense codes (pid, pk) and fp64 values: {field: [bins]}."""
    pid = np.asarray(pid, dtype=np.int64)
    pk = np.asarray(pk, dtype=np.int64)
    value = np.asarray(value, dtype=np.float64)
    if pid.size == 0:
        return {f: [] for f in HIST_FIELDS}
    pairs, pair_of_row = np.unique(np.stack([pid, pk], 1), axis=0, return_inverse=True)
    pair_of_row = pair_of_row.reshape(-1)
    pair_rows = np.bincount(pair_of_row)
    pair_sum = np.bincount(pair_of_row, weights=value)
    _, l0 = np.unique(pairs[:, 0], return_counts=True)          # distinct pks per pid
    _, l1 = np.unique(pid, return_counts=True)                  # rows per pid
    pks, pk_rows = np.unique(pk, return_counts=True)            # rows per pk
    _, pk_pids = np.unique(pairs[:, 1], return_counts=True)     # distinct pids per pk
    pk_sum = np.bincount(np.searchsorted(pks, pk), weights=value)
    return {
        "l0_contributions_histogram": frequency_histogram(l0),
        "l1_contributions_histogram": frequency_histogram(l1),
        "linf_contributions_histogram": frequency_histogram(pair_rows),
        "linf_sum_contributions_histogram": float_histogram(pair_sum),
        "count_per_partition_histogram": frequency_histogram(pk_rows),
        "count_privacy_id_per_partition": frequency_histogram(pk_pids),
        "sum_per_partition_histogram": float_histogram(pk_sum),
    }


def weighted_frequency_histogram(values, weights):
    """_compute_weighted_frequency_histogram (:81-102): per distinct value,
    int(round(sum of its weights)) (Python's round half to even; the weights
    summed in row order, as sum_per_key does), then the frequency helper's
    bins (:105-132): a value whose weight rounds to 0 still makes a bin with
    count 0 and max = value."""
    sums = {}
    for v, w in zip(np.asarray(values, dtype=np.int64).tolist(), np.asarray(weights, dtype=np.float64).tolist()):
        sums[v] = sums.get(v, 0.0) + w
    bins = {}
    for v in sorted(sums):
        f = int(round(sums[v]))
        lo, up = log_bin(v)
        b = bins.get(lo)
        bins[lo] = (lo, up, f, f * v, v) if b is None else (lo, up, b[2] + f, b[3] + f * v, max(b[4], v))
    return [bins[k] for k in sorted(bins)]


def preaggregated_histograms(pk, count, total, n_partitions, n_contributions):
    """compute_dataset_histograms_on_preaggregated_data
    (computing_histograms.py:713-758) over pre-aggregated columns, one row
    per (privacy id, partition) pair: {field: [bins]}.  L0 weighs
    n_partitions by 1 / n_partitions (:520-543), L1 n_contributions by
    1 / n_partitions (:546-568), Linf is the frequency of count (:571-591),
    Linf-sum the float histogram of sum (:594-625), and the partition
    histograms sum count / count rows / sum sum per partition (:628-710)."""
    pk = np.asarray(pk, dtype=np.int64)
    count = np.asarray(count, dtype=np.int64)
    total = np.asarray(total, dtype=np.float64)
    npart = np.asarray(n_partitions, dtype=np.int64)
    ncontr = np.asarray(n_contributions, dtype=np.int64)
    if pk.size == 0:
        return {f: [] for f in HIST_FIELDS}
    w = np.array([1.0 / v for v in npart.tolist()], dtype=np.float64)
    pks, inv = np.unique(pk, return_inverse=True)
    inv = inv.reshape(-1)
    pk_count = np.bincount(inv, weights=count.astype(np.float64)).astype(np.int64)
    pk_rows = np.bincount(inv)
    pk_sum = np.bincount(inv, weights=total)
    return {
        "l0_contributions_histogram": weighted_frequency_histogram(npart, w),
        "l1_contributions_histogram": weighted_frequency_histogram(ncontr, w),
        "linf_contributions_histogram": frequency_histogram(count),
        "linf_sum_contributions_histogram": float_histogram(total),
        "count_per_partition_histogram": frequency_histogram(pk_count),
        "count_privacy_id_per_partition": frequency_histogram(pk_rows),
        "sum_per_partition_histogram": float_histogram(pk_sum),
    }
