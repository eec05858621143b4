"""GPU parity of the dataset histograms (csrc/pdp_hist.hip,
compute_dataset_histograms) against the reference's own outputs (golden
fixtures, oracle/gen_golden_hist.py) and the NumPy oracle (oracle/histograms.py).

Bin bounds, counts, integer sums and maxima are exact; fp64 sums within 1e-9
relative (the reference sums in insertion order, the GPU in atomic order).
With dyadic values every sum is exact in any order, so bin membership of the
float histograms is pinned exactly too."""
import numpy as np
import pytest

from oracle import histograms as OH
from pipelinedp_amd import ColumnExtractor, ColumnTable, DataExtractors
from pipelinedp_amd import executor as X
from pipelinedp_amd.dataset_histograms import computing_histograms as CH
from tests import hist_util as HU

pytestmark = pytest.mark.gpu


def _dev():
    import torch
    return torch.device("cuda", 0)


def _check_all(got, want, what, exact=False):
    for field in OH.HIST_FIELDS:
        HU.assert_bins_equal(getattr(got, field).bins, want[field], f"{what}/{field}", exact=exact)


def _run_codes(pid, pk, val, U=None, P=None, mode="auto"):
    import torch
    d = _dev()
    U = int(pid.max()) + 1 if U is None else U
    P = int(pk.max()) + 1 if P is None else P
    vt = None if val is None else torch.as_tensor(val, device=d)
    raw = X.dataset_histograms(torch.as_tensor(pid, device=d), torch.as_tensor(pk, device=d), vt,
                               n_privacy_ids=U, n_partitions=P, force_pair_table=mode == "pair_table",
                               force_pair_hash=mode == "pair_hash")
    return CH.histograms_from_device(raw)


@pytest.mark.parametrize("case", ["uniform", "zipf_pids", "heavy_pairs", "int_values", "no_values",
                                  "wide_partitions", "zipf_partitions", "clipped"])
def test_pair_phases_agree_with_oracle(case):
    """The three pairs phases of pdp_hist.hip -- rows hashed into privacy-id
    buckets (default; pid counters in LDS, partition records summed per
    2,048-partition range by k_hb_prange, or partition atomics above 262,144
    partitions: "wide_partitions"), into pair buckets (PDP_HIST_FORCE_PAIR_HASH)
    and the HBM pair table (PDP_HIST_FORCE_PAIR_TABLE) -- give the oracle's
    bins; 3e6 rows, so the buckets span two levels (1,954 buckets in 8
    super-buckets).  "zipf_pids" has privacy ids with 10^4..10^6 rows, whose
    privacy-id buckets overflow: the default call falls back to pair buckets."""
    rng = np.random.default_rng({"uniform": 11, "zipf_pids": 12, "heavy_pairs": 13, "int_values": 14,
                                 "no_values": 15, "wide_partitions": 16, "zipf_partitions": 17, "clipped": 18}[case])
    n = 3_000_000
    pid = rng.integers(0, 200_000, n)
    pk = rng.integers(0, 40_000, n)
    if case == "zipf_pids":    # privacy ids with 10^4..10^6 rows
        pid = np.minimum(rng.zipf(1.4, n) - 1, 99_999)
    if case == "heavy_pairs":  # a few pairs with 10^5 rows each (one bucket holds them all)
        pid[:400_000] = rng.integers(0, 4, 400_000)
        pk[:400_000] = rng.integers(0, 2, 400_000)
    if case == "wide_partitions":
        pk = rng.integers(0, 300_000, n)
    if case == "zipf_partitions":  # hot partitions: LDS atomics on one range word
        pk = np.minimum(rng.zipf(1.1, n) - 1, 99_999)
    val = np.round(rng.normal(1, 3, n) * 8) / 8
    if case == "int_values":
        val = rng.integers(-20, 60, n)
    if case == "no_values":
        val = None
    if case == "clipped":  # the bench's values: ~5 % of the pair sums tie at each end
        val = np.clip(np.round(rng.normal(5, 3, n) * 8) / 8, 0.0, 10.0)
    want = OH.dataset_histograms(pid, pk, np.zeros(n) if val is None else val)
    for mode in ("auto", "pair_hash", "pair_table"):
        got = _run_codes(pid, pk, val, mode=mode)
        _check_all(got, want, f"{case}/{mode}", exact=True)


def test_pid_bucket_overflow_falls_back_to_pair_buckets():
    """One privacy id with 6,000 distinct partitions (and 3,000 light ones):
    its bucket's LDS table (kHbPidFill = 3,628 pairs) overflows, so the call
    redoes the pairs with pair-keyed buckets -- same bins."""
    rng = np.random.default_rng(21)
    heavy_pk = rng.permutation(8_192)[:6_000]
    pid = np.concatenate([np.zeros(6_000, np.int64), rng.integers(1, 1_000, 3_000)])
    pk = np.concatenate([heavy_pk, rng.integers(0, 8_192, 3_000)])
    val = np.round(rng.normal(0, 2, len(pid)) * 4) / 4
    got = _run_codes(pid, pk, val, U=1_000, P=8_192)
    _check_all(got, OH.dataset_histograms(pid, pk, val), "pid-overflow", exact=True)


def test_pair_bucket_overflow_falls_back():
    """3,000 distinct pairs that all hash into pair bucket 0 of 2 (crafted with
    the kernel's bucket hash): with the pair-keyed buckets
    (PDP_HIST_FORCE_PAIR_HASH) more than one LDS table holds (kHbFill =
    2,760), so the call redoes the pairs on the HBM pair table -- same bins;
    the default privacy-id buckets hold them."""
    from oracle.columnar import mix64
    U, P = 5_000, 64
    cand_pid = np.repeat(np.arange(U, dtype=np.int64), P)
    cand_pk = np.tile(np.arange(P, dtype=np.int64), U)
    pk_bits = max(1, int(np.ceil(np.log2(P))))
    x = (cand_pid.astype(np.uint64) << np.uint64(pk_bits)) | cand_pk.astype(np.uint64)
    h = (mix64(x ^ np.uint64(0x2545F4914F6CDD1D)) >> np.uint64(32)).astype(np.uint64)
    b = (h * np.uint64(2)) >> np.uint64(32)
    pick = np.flatnonzero(b == 0)[:3000]
    assert len(pick) == 3000
    pid, pk = cand_pid[pick], cand_pk[pick]
    val = np.round(np.random.default_rng(7).normal(0, 2, len(pid)) * 4) / 4
    want = OH.dataset_histograms(pid, pk, val)
    for mode in ("pair_hash", "auto"):
        got = _run_codes(pid, pk, val, U=U, P=P, mode=mode)
        _check_all(got, want, f"overflow/{mode}", exact=True)


@pytest.mark.parametrize("fx", HU.fixtures(), ids=lambda f: f["name"])
def test_reference_golden_rows(fx):
    rows = [tuple(r) for r in fx["rows"]]
    ext = DataExtractors(lambda r: r[0], lambda r: r[1], lambda r: r[2])
    (got,) = CH.compute_dataset_histograms(rows, ext)
    for field, exp in fx["expected"].items():
        h = getattr(got, field)
        assert h.name.value == exp["name"]
        HU.assert_bins_equal(h.bins, exp["bins"], f"{fx['name']}/{field}", exact=fx["name"] != "strings")


def test_reference_golden_column_table():
    fx = [f for f in HU.fixtures() if f["name"] == "dyadic"][0]
    rows = fx["rows"]
    t = ColumnTable({"pid": np.asarray([r[0] for r in rows], dtype=np.int64),
                     "pk": np.asarray([r[1] for r in rows], dtype=np.int64),
                     "v": np.asarray([r[2] for r in rows], dtype=np.float64)})
    ext = DataExtractors(ColumnExtractor("pid"), ColumnExtractor("pk"), ColumnExtractor("v"))
    (got,) = CH.compute_dataset_histograms(t, ext)
    for field, exp in fx["expected"].items():
        HU.assert_bins_equal(getattr(got, field).bins, exp["bins"], field, exact=True)


@pytest.mark.parametrize("case", ["uniform_dyadic", "zipf_heavy", "int_values", "no_values", "sparse_codes"])
def test_against_oracle(case):
    rng = np.random.default_rng({"uniform_dyadic": 1, "zipf_heavy": 2, "int_values": 3, "no_values": 4,
                                 "sparse_codes": 5}[case])
    n = 400_000
    if case == "zipf_heavy":   # partitions with 10^3..10^5 rows: logarithmic bins above 1000
        pid = rng.integers(0, 20_000, n)
        pk = np.minimum(rng.zipf(1.3, n) - 1, 49_999)
        val = rng.normal(5, 3, n)
    elif case == "sparse_codes":  # declared ranges much larger than the codes used
        pid = rng.integers(0, 1000, n) * 997
        pk = rng.integers(0, 50, n) * 31
        val = np.round(rng.normal(0, 4, n) * 4) / 4
    else:
        pid = rng.integers(0, 30_000, n)
        pk = rng.integers(0, 3_000, n)
        val = np.round(rng.normal(1, 2, n) * 16) / 16
    if case == "int_values":
        val = rng.integers(-50, 100, n)
    if case == "no_values":
        got = _run_codes(pid, pk, None)
        want = OH.dataset_histograms(pid, pk, np.zeros(n))
    else:
        got = _run_codes(pid, pk, val, U=int(pid.max()) + 7, P=int(pk.max()) + 3)
        want = OH.dataset_histograms(pid, pk, val)
    _check_all(got, want, case, exact=case != "zipf_heavy")


def test_single_row_and_constant_sums():
    got = _run_codes(np.array([3]), np.array([1]), np.array([2.5]), U=5, P=2)
    _check_all(got, OH.dataset_histograms([3], [1], [2.5]), "single")
    assert got.linf_sum_contributions_histogram.bins[0].lower == got.linf_sum_contributions_histogram.bins[0].upper


def test_subnormal_value_range():
    """Pair and partition sums that span a few subnormals: np.linspace's step
    (delta / 10,000) underflows to 0, so the lowers take numpy's other form,
    (i / 10,000) * delta + start (k_h_lowers and the float passes' STEP0
    path), and the bin guess's 1 / delta overflows; bins must still equal the
    oracle's exactly."""
    rng = np.random.default_rng(11)
    n = 50_000
    pid = rng.integers(0, 5_000, n)
    pk = rng.integers(0, 500, n)
    val = rng.integers(0, 4, n) * 5e-324
    got = _run_codes(pid, pk, val, U=5_000, P=500)
    _check_all(got, OH.dataset_histograms(pid, pk, val), "subnormal")


def test_empty_input():
    got = _run_codes(np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0), U=4, P=4)
    for field in OH.HIST_FIELDS:
        h = getattr(got, field)
        assert h.bins == [] and h.lower is None and h.upper is None


def test_out_of_range_codes_raise():
    """device-resident dense codes are taken as declared; one outside
    [0, n) sets the kernel's error bit and the API raises"""
    import torch
    d = _dev()
    t = ColumnTable({"pid": torch.tensor([0, 1], device=d), "pk": torch.tensor([0, 5], device=d),
                     "v": torch.tensor([1.0, 1.0], device=d, dtype=torch.float64)},
                    n_privacy_ids=2, n_partitions=3)
    ext = DataExtractors(ColumnExtractor("pid"), ColumnExtractor("pk"), ColumnExtractor("v"))
    with pytest.raises(ValueError):
        CH.compute_dataset_histograms(t, ext)
    pid = torch.tensor([0, 1, 2], device=d)
    pk = torch.tensor([0, 9, 1], device=d)
    raw = X.dataset_histograms(pid, pk, None, n_privacy_ids=3, n_partitions=2)
    flags = np.zeros(1, np.uint32)
    import ctypes
    from pipelinedp_amd import _native as N
    N.check(N.lib().pdp_bound_error_flags(X._ptr(raw["workspace"]), flags.ctypes.data_as(
        ctypes.POINTER(ctypes.c_uint32)), X._stream()), "flags")
    assert flags[0] & 1
    h = CH.histograms_from_device(raw)   # the bad row is skipped, never read out of bounds
    assert h.l1_contributions_histogram.total_sum() == 2


def test_full_size_invariants():
    """1e8 rows (C2's shape, the bench's hist workload): totals every
    histogram must satisfy, checked against torch group-bys on the device;
    and the default privacy-id buckets give exactly the bins of the HBM pair
    table (PDP_HIST_FORCE_PAIR_TABLE), which the small cases pin to the
    oracle (quarter-integer values: every sum exact in any order)."""
    import torch
    d = _dev()
    n, U, P = 100_000_000, 1_000_000, 100_000
    g = torch.Generator(device=d).manual_seed(5)
    pid = torch.randint(0, U, (n,), device=d, generator=g)
    pk = torch.randint(0, P, (n,), device=d, generator=g)
    val = torch.randint(-8, 9, (n,), device=d, generator=g).to(torch.float64) / 4
    raw = X.dataset_histograms(pid, pk, val, n_privacy_ids=U, n_partitions=P)
    h = CH.histograms_from_device(raw)
    del raw
    ref = CH.histograms_from_device(X.dataset_histograms(pid, pk, val, n_privacy_ids=U, n_partitions=P,
                                                         force_pair_table=True))
    for field in OH.HIST_FIELDS:
        got = [(b.lower, b.upper, b.count, b.sum, b.max) for b in getattr(h, field).bins]
        want = [(b.lower, b.upper, b.count, b.sum, b.max) for b in getattr(ref, field).bins]
        assert got == want, field
    n_pairs = int(torch.unique(pid * P + pk).numel())
    n_pids = int(torch.unique(pid).numel())
    total = float(val.sum().item())
    del pid, pk
    assert h.l1_contributions_histogram.total_sum() == n
    assert h.l1_contributions_histogram.total_count() == n_pids
    assert h.linf_contributions_histogram.total_sum() == n
    assert h.count_per_partition_histogram.total_sum() == n
    assert h.count_per_partition_histogram.total_count() == P
    assert h.l0_contributions_histogram.total_sum() == n_pairs
    assert h.linf_contributions_histogram.total_count() == n_pairs
    assert h.count_privacy_id_per_partition.total_sum() == n_pairs
    assert h.linf_sum_contributions_histogram.total_count() == n_pairs
    assert h.sum_per_partition_histogram.total_count() == P
    assert h.sum_per_partition_histogram.total_sum() == total  # quarter-integers: exact
    assert h.linf_sum_contributions_histogram.total_sum() == total
    assert len(h.linf_sum_contributions_histogram.bins) <= CH.NUMBER_OF_BUCKETS_SUM_HISTOGRAM


def _two_rank_data():
    rng = np.random.default_rng(21)
    n = 300_000
    pid = rng.integers(0, 50_000, n)
    pk = np.minimum(rng.zipf(1.4, n) - 1, 1999)
    val = np.round(rng.normal(2, 5, n) * 8) / 8
    return pid, pk, val


def _hist_worker(rank, port, results):
    import os
    import torch.distributed as dist
    from pipelinedp_amd import parallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        pid, pk, val = _two_rank_data()
        mine = parallel.shard_by_privacy_id(pid, 2, rank)
        h = _run_codes(pid[mine], pk[mine], val[mine], U=50_000, P=2000)
        results[rank] = {f: [tuple(map(float, (b.lower, b.upper, b.count, b.sum, b.max)))
                             for b in getattr(h, f).bins] for f in OH.HIST_FIELDS}
    except Exception as e:
        results[rank] = repr(e)
    finally:
        dist.destroy_process_group()


def test_two_ranks_match_single_process():
    """rows sharded by privacy id over two ranks (gloo exchange, both on this
    GPU): every rank's merged histograms equal the single-process ones
    (dyadic values: exact)."""
    import socket
    import torch.multiprocessing as mp
    pid, pk, val = _two_rank_data()
    single = _run_codes(pid, pk, val, U=50_000, P=2000)
    _check_all(single, OH.dataset_histograms(pid, pk, val), "single", exact=True)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.spawn(_hist_worker, args=(port, results), nprocs=2, join=True)
    res = dict(results)
    assert all(isinstance(res[r], dict) for r in (0, 1)), res
    for r in (0, 1):
        for f in OH.HIST_FIELDS:
            HU.assert_bins_equal(res[r][f], getattr(single, f).bins, f"rank{r}/{f}", exact=True)


@pytest.mark.parametrize("field,rows,expected", HU.kat_cases())
def test_reference_test_known_answers(field, rows, expected):
    """the reference tests' expected L0 / L1 bins, through the HIP path"""
    ext = DataExtractors(lambda r: r[0], lambda r: r[1], lambda r: 0)
    (got,) = CH.compute_dataset_histograms(rows, ext)
    HU.assert_bins_equal(getattr(got, field).bins, expected, field, exact=True)


def test_many_partition_regions():
    """P = 7e7 partitions: more regions (P / 4096) than the LDS region-count
    histogram holds, so rows are counted per region with global atomics"""
    rng = np.random.default_rng(31)
    n = 200_000
    pid = rng.integers(0, 5_000, n)
    pk = rng.integers(0, 70_000_000, n)
    pk[:50_000] = rng.integers(0, 40, 50_000)  # a few hot partitions in region 0 as well
    val = np.round(rng.normal(0, 3, n) * 4) / 4
    got = _run_codes(pid, pk, val, U=5_000, P=70_000_000)
    _check_all(got, OH.dataset_histograms(pid, pk, val), "many_regions", exact=True)


# ---------------------------------------------- pre-aggregated (:713-758) --
def _run_pre(pk, cnt, tot, npart, ncontr, P=None):
    import torch
    d = _dev()
    P = int(pk.max()) + 1 if P is None else P
    cols = [torch.as_tensor(np.ascontiguousarray(c), device=d) for c in (pk, cnt, tot, npart, ncontr)]
    raw = X.dataset_histograms_preaggregated(*cols, n_partitions=P)
    return CH.histograms_from_device(raw)


@pytest.mark.parametrize("fx", HU.pre_fixtures(), ids=lambda f: f["name"])
def test_preaggregated_reference_golden_rows(fx):
    """the reference's compute_dataset_histograms_on_preaggregated_data bins,
    from rows (pk, (count, sum, n_partitions, n_contributions)) as
    preaggregate() emits them, through PreAggregateExtractors"""
    from pipelinedp_amd.data_extractors import PreAggregateExtractors
    rows = [(r[0], tuple(r[1:])) for r in fx["rows"]]
    ext = PreAggregateExtractors(partition_extractor=lambda r: r[0], preaggregate_extractor=lambda r: r[1])
    (got,) = CH.compute_dataset_histograms_on_preaggregated_data(rows, ext)
    for field, exp in fx["expected"].items():
        h = getattr(got, field)
        assert h.name.value == exp["name"]
        HU.assert_bins_equal(h.bins, exp["bins"], f"pre_{fx['name']}/{field}",
                             exact=fx["name"] not in ("strings", "weights"))


def test_preaggregated_column_table():
    from pipelinedp_amd.data_extractors import PreAggregateExtractors
    fx = [f for f in HU.pre_fixtures() if f["name"] == "heavy"][0]
    pk, cnt, tot, npart, ncontr = HU.pre_columns(fx["rows"])
    t = ColumnTable({"pk": pk, "c": cnt, "s": tot, "np": npart, "nc": ncontr})
    ext = PreAggregateExtractors(partition_extractor=ColumnExtractor("pk"),
                                 preaggregate_extractor=lambda r: (r["c"], r["s"], r["np"], r["nc"]))
    (got,) = CH.compute_dataset_histograms_on_preaggregated_data(t, ext)
    for field, exp in fx["expected"].items():
        HU.assert_bins_equal(getattr(got, field).bins, exp["bins"], field, exact=True)


@pytest.mark.parametrize("case", ["uniform", "zipf_heavy", "big_values"])
def test_preaggregated_against_oracle_and_raw(case):
    """pre-aggregated columns of seeded raw data: the HIP bins equal the
    oracle's, and equal the raw-data HIP histograms (the reference test's
    premise, computing_histograms_test.py:820-875)"""
    rng = np.random.default_rng({"uniform": 41, "zipf_heavy": 42, "big_values": 43}[case])
    n = 300_000
    if case == "zipf_heavy":
        pid = np.minimum(rng.zipf(1.5, n) - 1, 9_999)   # pids with 10^3..10^5 rows: L1 above 1000
        pk = np.minimum(rng.zipf(1.3, n) - 1, 19_999)
    elif case == "big_values":
        pid = rng.integers(0, 30, n)                    # ~10^4 rows and ~10^3 partitions per pid
        pk = rng.integers(0, 2_500, n)
    else:
        pid = rng.integers(0, 40_000, n)
        pk = rng.integers(0, 3_000, n)
    val = np.round(rng.normal(1, 3, n) * 8) / 8
    pre = HU.preaggregate(pid, pk, val)
    got = _run_pre(*pre)
    _check_all(got, OH.preaggregated_histograms(*pre), f"pre_{case}", exact=True)
    raw = _run_codes(pid, pk, val)
    for field in OH.HIST_FIELDS:
        HU.assert_bins_equal(getattr(got, field).bins, HU.as_tuples(getattr(raw, field).bins), f"raw/{field}",
                             exact=True)


def test_preaggregated_invalid_rows_raise():
    from pipelinedp_amd.data_extractors import PreAggregateExtractors
    ext = PreAggregateExtractors(partition_extractor=lambda r: r[0], preaggregate_extractor=lambda r: r[1])
    with pytest.raises(ValueError):
        CH.compute_dataset_histograms_on_preaggregated_data([(0, (1, 1.0, 0, 1))], ext)  # n_partitions 0
    with pytest.raises(ValueError):
        CH.compute_dataset_histograms_on_preaggregated_data([(0, (0, 1.0, 1, 1))], ext)  # count 0


def test_preaggregated_empty_input():
    import torch
    d = _dev()
    e = torch.empty(0, dtype=torch.int64, device=d)
    raw = X.dataset_histograms_preaggregated(e, e, torch.empty(0, dtype=torch.float64, device=d), e, e,
                                             n_partitions=0)
    got = CH.histograms_from_device(raw)
    assert all(not getattr(got, f).bins for f in OH.HIST_FIELDS)


def _pre_data(split):
    if split == "pid":
        return _two_rank_data()
    # privacy ids with 10^3..10^5 rows (L0 / L1 values above 1000: the weight
    # table, not only the dense sums)
    rng = np.random.default_rng(22)
    n = 300_000
    pid = np.minimum(rng.zipf(1.5, n) - 1, 9_999)
    pk = np.minimum(rng.zipf(1.3, n) - 1, 1_999)
    val = np.round(rng.normal(1, 3, n) * 8) / 8
    return pid, pk, val


def _pre_worker(rank, port, results, split):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        pid, pk, val = _pre_data(split)
        pre = HU.preaggregate(pid, pk, val)
        if split == "pid":
            # shard the pre-aggregated rows by privacy id: rows of one pid on one rank
            pairs_pid = np.unique(np.stack([pid, pk], 1), axis=0)[:, 0]
            keep = pairs_pid % 2 == rank
        else:
            # every other (pid, pk) row: a privacy id's rows span both ranks,
            # which pre-aggregated input (no privacy-id column) cannot rule out;
            # its 1 / n_partitions weights must be summed over ranks before
            # rounding, not rounded per rank
            keep = np.arange(len(pre[0])) % 2 == rank
        h = _run_pre(*(c[keep] for c in pre), P=2000)
        results[rank] = {f: [tuple(map(float, (b.lower, b.upper, b.count, b.sum, b.max)))
                             for b in getattr(h, f).bins] for f in OH.HIST_FIELDS}
    except Exception as e:
        results[rank] = repr(e)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("split", ["pid", "row"])
def test_preaggregated_two_ranks_match_single_process(split):
    import socket
    import torch.multiprocessing as mp
    pid, pk, val = _pre_data(split)
    single = _run_pre(*HU.preaggregate(pid, pk, val), P=2000)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.spawn(_pre_worker, args=(port, results, split), nprocs=2, join=True)
    res = dict(results)
    assert all(isinstance(res[r], dict) for r in (0, 1)), res
    for r in (0, 1):
        for f in OH.HIST_FIELDS:
            HU.assert_bins_equal(res[r][f], getattr(single, f).bins, f"rank{r}/{f}", exact=True)
