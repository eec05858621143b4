"""TEST INFRASTRUCTURE — regenerate tests/golden/histograms/*.json by
running the reference's compute_dataset_histograms.

Runs only in the build container (it reads /root/reference, which never travels
to the GPU box).  The reference imports with the python-dp stand-in in
oracle/pydp_standin (PyDP is not installed; no permission denial was involved).

Each case runs pipeline_dp.dataset_histograms.computing_histograms.
compute_dataset_histograms (computing_histograms.py:456-513) on LocalBackend
over rows (pid, pk, value) and stores the inputs plus every bin
(lower, upper, count, sum, max) of the seven histograms.

Pre-aggregated cases (dataset_histograms_pre_*.json): the reference's own
analysis.pre_aggregation.preaggregate (analysis/pre_aggregation.py:19-58)
turns the raw rows into (partition_key, (count, sum, n_partitions,
n_contributions)) rows, and compute_dataset_histograms_on_preaggregated_data
(computing_histograms.py:713-758) produces the bins; a hand-made case with
inconsistent n_partitions pins the weighted bins' rounding (round half to
even of the summed 1/n_partitions weights, :81-102).

Usage: python -m oracle.gen_golden_hist   (from the repo root)
"""
import json
import os

import numpy as np

from oracle.gen_golden import OUT, _import_reference, _py

HIST_FIELDS = ("l0_contributions_histogram", "l1_contributions_histogram",
               "linf_contributions_histogram", "linf_sum_contributions_histogram",
               "count_per_partition_histogram", "count_privacy_id_per_partition",
               "sum_per_partition_histogram")


def _run_reference(rows):
    pipeline_dp = _import_reference()
    from pipeline_dp.dataset_histograms import computing_histograms as ch
    ext = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                                     partition_extractor=lambda r: r[1],
                                     value_extractor=lambda r: r[2])
    out = list(ch.compute_dataset_histograms(rows, ext, pipeline_dp.LocalBackend()))
    assert len(out) == 1
    h = out[0]
    res = {}
    for f in HIST_FIELDS:
        hist = getattr(h, f)
        res[f] = {"name": hist.name.value,
                  "bins": [[_py(b.lower), _py(b.upper), _py(b.count), _py(b.sum), _py(b.max)]
                           for b in hist.bins]}
    return res


def _hist_json(h):
    res = {}
    for f in HIST_FIELDS:
        hist = getattr(h, f)
        res[f] = {"name": hist.name.value,
                  "bins": [[_py(b.lower), _py(b.upper), _py(b.count), _py(b.sum), _py(b.max)]
                           for b in hist.bins]}
    return res


def _preaggregate_reference(rows):
    pipeline_dp = _import_reference()
    from analysis import pre_aggregation
    ext = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                                     partition_extractor=lambda r: r[1],
                                     value_extractor=lambda r: r[2])
    out = list(pre_aggregation.preaggregate(rows, pipeline_dp.LocalBackend(), ext))
    return [(pk, tuple(x)) for pk, x in out]


def _run_reference_pre(pre_rows):
    pipeline_dp = _import_reference()
    from pipeline_dp.dataset_histograms import computing_histograms as ch
    ext = pipeline_dp.PreAggregateExtractors(partition_extractor=lambda r: r[0],
                                             preaggregate_extractor=lambda r: r[1])
    out = list(ch.compute_dataset_histograms_on_preaggregated_data(pre_rows, ext, pipeline_dp.LocalBackend()))
    assert len(out) == 1
    return _hist_json(out[0])


def _case_pre(name, pre_rows, note):
    expected = _run_reference_pre(pre_rows)
    path = os.path.join(OUT, "histograms", f"dataset_histograms_pre_{name}.json")
    with open(path, "w") as f:
        json.dump({"note": note, "rows": [[_py(pk)] + [_py(v) for v in x] for pk, x in pre_rows],
                   "expected": expected}, f)
    print("wrote", path, len(pre_rows), "pre-aggregated rows")


def _case(name, rows, note):
    expected = _run_reference(rows)
    os.makedirs(os.path.join(OUT, "histograms"), exist_ok=True)
    path = os.path.join(OUT, "histograms", f"dataset_histograms_{name}.json")
    with open(path, "w") as f:
        json.dump({"note": note, "rows": [[_py(v) for v in r] for r in rows], "expected": expected}, f)
    print("wrote", path, len(rows), "rows")


def main():
    rng = np.random.default_rng(11)
    # 1. random ints, dyadic fp64 values (every sum exact in any order)
    n = 3000
    pid = rng.integers(0, 150, n)
    pk = rng.integers(0, 40, n)
    val = np.round(rng.normal(2.0, 3.0, n) * 8) / 8
    dyadic = list(zip(pid.tolist(), pk.tolist(), val.tolist()))
    _case("dyadic", dyadic, "uniform pid in [0,150), pk in [0,40), values k/8")
    # 2. heavy contributors: logarithmic bins above 1000 (pair 0/0 has 12,345
    # rows, pid 1 spreads 2,500 rows over 5 partitions, partition 3 gets 1,000)
    rows = [(0, 0, 1.0)] * 12345 + [(1, k % 5, 0.5) for k in range(2500)]
    rows += [(2 + (i % 700), 3, float(i % 7)) for i in range(1000)]
    rows += [(int(u), int(k), float(v)) for u, k, v in
             zip(rng.integers(5000, 5100, 800), rng.integers(0, 30, 800), rng.integers(-3, 9, 800))]
    _case("heavy", rows, "log bins above 1000: 12,345-row pair, 2,500-row pid, 1,000-row partition")
    heavy = rows
    # 3. string keys, general fp64 values
    rows = [(f"user{int(u)}", f"pk{int(k)}", float(v)) for u, k, v in
            zip(rng.integers(0, 90, 1500), rng.integers(0, 25, 1500), rng.normal(0.0, 10.0, 1500))]
    _case("strings", rows, "string privacy ids and partition keys, N(0,10) values")
    strings = rows
    # 4. every pair and partition sum equal: min == max, lowers = [m, m]
    rows = [(u, u % 3, 2.0) for u in range(30)]
    _case("constant", rows, "one row per pid: all pair sums 2.0, partition sums equal (min == max)")
    # pre-aggregated: the reference's preaggregate of the raw cases above
    for name, raw in (("dyadic", dyadic), ("heavy", heavy), ("strings", strings), ("constant", rows)):
        _case_pre(name, _preaggregate_reference(raw), f"preaggregate() of the raw '{name}' case")
    # rounding of the weighted L0 / L1 bins: n_partitions disagrees with the
    # rows present, so the summed 1/n_partitions weights are not integers
    # (5 x 1/2 = 2.5 -> 2, 6 x 1/4 = 1.5 -> 2, 3 x 1/8 = 0.375 -> 0, 7 x 1/2 = 3.5 -> 4)
    pre = [(k % 4, (1 + k % 3, float(k % 5) - 1.5, 2, 3)) for k in range(5)]
    pre += [(k % 6, (2, 0.25 * k, 4, 1200 + k % 2)) for k in range(6)]
    pre += [(7, (1, 1.0, 8, 5))] * 3
    pre += [(8 + k, (3, -2.0, 2, 2500)) for k in range(7)]
    _case_pre("weights", pre, "inconsistent n_partitions: non-integer weight sums, round half to even")


if __name__ == "__main__":
    main()
