"""Dataset histograms, CPU side: the oracle against the
reference's own outputs (golden fixtures), the integer-bin index mapping of
the kernels, and the host mirror of histograms.py against the reference
tests' known answers (tests/dataset_histograms/histograms_test.py)."""
import pytest

from oracle import histograms as OH
from pipelinedp_amd.dataset_histograms import computing_histograms as CH
from pipelinedp_amd.dataset_histograms import histograms as hist
from tests import hist_util as HU


@pytest.mark.parametrize("fx", HU.fixtures(), ids=lambda f: f["name"])
def test_oracle_matches_reference_golden(fx):
    pid, pk, val = HU.codes(fx["rows"])
    got = OH.dataset_histograms(pid, pk, val)
    for field, exp in fx["expected"].items():
        HU.assert_bins_equal(got[field], exp["bins"], f"{fx['name']}/{field}")


def _index_of(v):
    """the kernels' dense index (pdp_hist.hip log_bin_index), restated"""
    bound = 1000
    while v > bound:
        bound *= 10
    q = v // (bound // 1000) * (bound // 1000)
    if q < 1000:
        return q
    e = 0
    while q >= 1000:
        q //= 10
        e += 1
    return 1000 + (e - 1) * 900 + q - 100


def test_log_bin_index_round_trip():
    for v in list(range(0, 3000)) + [9999, 10000, 10001, 99999, 100000, 100001, 123456789,
                                     10**9, 10**9 + 1, 2**31 - 1, 2**32 - 1, 10**12, 10**15 + 7]:
        lo, up = OH.log_bin(v)
        assert CH.log_bin_bounds(_index_of(v)) == (lo, up), v
        assert _index_of(v) < 16384


def test_log_bin_index_is_monotone():
    idx = [_index_of(v) for v in range(1, 200000, 7)]
    assert idx == sorted(idx)


# histograms_test.py known answers
@pytest.mark.parametrize("bins,q,expected", [
    ([hist.FrequencyBin(1, 2, 2, 2, 1), hist.FrequencyBin(2, 3, 1, 2, 2), hist.FrequencyBin(3, 4, 1, 3, 3),
      hist.FrequencyBin(4, 5, 2, 8, 4), hist.FrequencyBin(5, 6, 2, 10, 5), hist.FrequencyBin(6, 7, 1, 6, 6),
      hist.FrequencyBin(10, 12, 1, 11, 11)], [0.001, 0.05, 0.1, 0.5, 0.8, 0.9], [1, 1, 1, 4, 6, 10]),
    ([hist.FrequencyBin(1000, 1010, 10, 10100, 1009)], [0.05, 0.1, 0.5, 0.8, 0.9], [1000] * 5),
])
def test_quantiles_known_answers(bins, q, expected):
    assert hist.Histogram(hist.HistogramType.L0_CONTRIBUTIONS, bins).quantiles(q) == expected


def test_ratio_dropped_known_answers():
    assert hist.compute_ratio_dropped(hist.Histogram(hist.HistogramType.L0_CONTRIBUTIONS, [])) == []
    h = hist.Histogram(hist.HistogramType.L0_CONTRIBUTIONS, [hist.FrequencyBin(1000, 1021, 10, 10100, 1020)])
    assert hist.compute_ratio_dropped(h) == [(0, 1), (1000, 100 / 10100), (1020, 0.0)]
    bins = [hist.FrequencyBin(1, 2, 8, 8, 1), hist.FrequencyBin(2, 3, 2, 4, 2), hist.FrequencyBin(3, 4, 1, 3, 3),
            hist.FrequencyBin(4, 5, 2, 8, 4), hist.FrequencyBin(5, 6, 2, 10, 5), hist.FrequencyBin(6, 7, 1, 6, 6),
            hist.FrequencyBin(11, 12, 1, 11, 11)]
    got = hist.compute_ratio_dropped(hist.Histogram(hist.HistogramType.L0_CONTRIBUTIONS, bins))
    want = [(0, 1), (1, 0.66), (2, 0.48), (3, 0.34), (4, 0.22), (5, 0.14), (6, 0.1), (11, 0.0)]
    assert [a for a, _ in got] == [a for a, _ in want]
    assert all(abs(x - y) < 1e-12 for (_, x), (_, y) in zip(got, want))


@pytest.mark.parametrize("name,bins,lower,upper", [
    (hist.HistogramType.L0_CONTRIBUTIONS, [], None, None),
    (hist.HistogramType.LINF_SUM_CONTRIBUTIONS, [], None, None),
    (hist.HistogramType.L0_CONTRIBUTIONS, [hist.FrequencyBin(4, 5, 1, 4, 4)], 1, None),
    (hist.HistogramType.LINF_SUM_CONTRIBUTIONS, [hist.FrequencyBin(0.1, 0.2, 1, 0.1, 0.1)], 0.1, 0.2),
    (hist.HistogramType.LINF_SUM_CONTRIBUTIONS, [hist.FrequencyBin(0.1, 0.1, 1, 0.1, 0.1)], 0.1, 0.1),
    (hist.HistogramType.SUM_PER_PARTITION, [hist.FrequencyBin(0.1, 0.2, 1, 0.1, 0.1),
                                            hist.FrequencyBin(0.3, 0.4, 1, 0.3, 0.3)], 0.1, 0.4),
])
def test_lower_and_upper(name, bins, lower, upper):
    h = hist.Histogram(name, bins)
    assert (h.lower, h.upper) == (lower, upper)
    assert h.is_integer == (name not in (hist.HistogramType.LINF_SUM_CONTRIBUTIONS,
                                         hist.HistogramType.SUM_PER_PARTITION))


def test_frequency_bin_add_and_eq():
    a = hist.FrequencyBin(10, 11, 2, 20, 10)
    assert a + hist.FrequencyBin(10, 11, 3, 30, 10) == hist.FrequencyBin(10, 11, 5, 50, 10)
    with pytest.raises(AssertionError):
        a + hist.FrequencyBin(11, 12, 1, 11, 11)


def test_compute_dataset_histograms_needs_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pipelinedp_amd import DataExtractors
    ext = DataExtractors(lambda r: r[0], lambda r: r[1], lambda r: r[2])
    with pytest.raises(RuntimeError):
        CH.compute_dataset_histograms([(1, 2, 3.0)], ext)


@pytest.mark.parametrize("field,rows,expected", HU.kat_cases())
def test_oracle_reference_test_known_answers(field, rows, expected):
    pid, pk, _ = HU.codes([(u, k, 0.0) for u, k in rows])
    got = OH.dataset_histograms(pid, pk, [0.0] * len(rows))[field]
    HU.assert_bins_equal(got, expected, field, exact=True)


# ---------------------------------------------- pre-aggregated (:713-758) --
@pytest.mark.parametrize("fx", HU.pre_fixtures(), ids=lambda f: f["name"])
def test_preaggregated_oracle_matches_reference_golden(fx):
    got = OH.preaggregated_histograms(*HU.pre_columns(fx["rows"]))
    for field, exp in fx["expected"].items():
        HU.assert_bins_equal(got[field], exp["bins"], f"pre_{fx['name']}/{field}")


@pytest.mark.parametrize("fx", HU.fixtures(), ids=lambda f: f["name"])
def test_preaggregated_equals_raw_histograms(fx):
    """the reference test's premise (computing_histograms_test.py:820-875,
    pre_aggregated=(False, True)): histograms of preaggregate(rows) equal
    those of the rows, here through the oracle on both sides"""
    pid, pk, val = HU.codes(fx["rows"])
    got = OH.preaggregated_histograms(*HU.preaggregate(pid, pk, val))
    for field, exp in fx["expected"].items():
        HU.assert_bins_equal(got[field], exp["bins"], f"{fx['name']}/{field}")


def test_preaggregated_weights_fixture_pins_rounding():
    """the inconsistent fixture's L0 / L1: half-to-even rounding and a
    count-0 bin that keeps its max"""
    fx = [f for f in HU.pre_fixtures() if f["name"] == "weights"][0]
    l0 = [tuple(b) for b in fx["expected"]["l0_contributions_histogram"]["bins"]]
    assert (8, 9, 0, 0, 8) in l0 and (2, 3, 6, 12, 2) in l0
    l1 = [tuple(b) for b in fx["expected"]["l1_contributions_histogram"]["bins"]]
    assert (2500, 2510, 4, 10000, 2500) in l1
