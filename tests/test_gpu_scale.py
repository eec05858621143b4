"""GPU parity at the BASELINE workload sizes.

Every test runs the HIP path (pdp_bound_contributions + pdp_reduce_partitions
through the C ABI) on a BASELINE-shaped input and checks it against the CPU
oracle, not against another HIP path:
* C2 (1e8 rows, U = 1e6, P = 1e5, L0 = 8, Linf = 2, sampling fires) against
  the oracle's identical counter-based samples, and its "parity variant"
  (L0 / Linf taken from the data, nothing sampled) against an exact group-by;
* C3 at 1e9 rows on one GPU through size-independent identities (kept pairs
  = sum over privacy ids of min(L0, distinct partitions); one row per kept
  pair), plus the oracle on C3-shaped inputs in the record format C3 runs in
  (PACKED) and, forced, the wide format;
* C4's shape (P = 1e7, U = 1e8, 1e8 rows, VARIANCE + PRIVACY_ID_COUNT flags,
  L0 = 4, Linf = 2) including selection and noise for the kept partitions;
* C5's shape (heavy-tailed Pareto(1.5) rows per privacy id with a 1e6-row
  privacy id, Zipf partitions, lognormal values).
Integers (privacy-id counts, counts) bit-exact; fp64 sums within 1e-9 of the
per-partition sum of |terms| (summation order differs).  The oracle runs on
privacy-id shards over host processes (oracle/parallel_oracle.py), which
keeps integer results identical to the single-process oracle.
"""
import numpy as np
import pytest

from oracle import columnar as O
from oracle import parallel_oracle as PO

pytestmark = pytest.mark.gpu

FLOAT_RTOL = 1e-9


def _spec(l0, linf, vk, flags, lo=0.0, hi=10.0):
    from pipelinedp_amd import executor as X
    return X.BoundingSpec(l0=l0, linf=linf, value_kind=vk, flags=flags, min_value=lo, max_value=hi,
                          middle=lo + (hi - lo) / 2)


def _gpu(device, pid, pk, val, U, P, spec, seed, key_format=0, algorithm=0, row_offset=0):
    import torch
    from pipelinedp_amd import executor as X
    tp = torch.as_tensor(pid).to(device)
    tk = torch.as_tensor(pk).to(device)
    tv = None if val is None else torch.as_tensor(val).to(device)
    acc = X.bound_and_reduce(tp, tk, tv, n_privacy_ids=U, n_partitions=P, bounding=spec, seed=seed,
                             key_format=key_format, algorithm=algorithm, row_offset=row_offset)
    torch.cuda.synchronize()
    out = {k: (None if v is None else v.cpu().numpy()) for k, v in acc.items()}
    del tp, tk, tv, acc
    torch.cuda.empty_cache()
    return out


def _oracle(pid, pk, val, U, P, spec, seed, rand_shift, row_offset=0):
    return PO.bound_and_reduce(pid, pk, val, n_privacy_ids=U, n_partitions=P, l0=spec.l0, linf=spec.linf,
                               value_kind=spec.value_kind, flags=spec.flags, min_value=spec.min_value,
                               max_value=spec.max_value, middle=spec.middle, seed=seed, rand_shift=rand_shift,
                               row_offset=row_offset)


def _scale(pk, val, P, spec):
    s = np.ones(P)
    if val is not None:
        w = np.abs(np.clip(val.astype(np.float64), spec.min_value, spec.max_value)) + abs(spec.middle) + 1.0
        s += np.bincount(pk, weights=w, minlength=P)
    return s


def _compare(got, want, scale):
    np.testing.assert_array_equal(got["privacy_id_count"], want["privacy_id_count"])
    np.testing.assert_array_equal(got["count"], want["count"])
    for k in ("sum", "normalized_sum", "normalized_sum_sq"):
        if got[k] is None:
            continue
        sc = scale if k != "normalized_sum_sq" else scale * scale
        bad = np.abs(got[k] - want[k]) > FLOAT_RTOL * sc
        assert not bad.any(), (k, np.flatnonzero(bad)[:5])


def _plan(n, U, P, spec, key_format=0, algorithm=0):
    from pipelinedp_amd import executor as X
    return X.bound_plan(n, U, P, spec, algorithm=algorithm, key_format=key_format)


def _zipf_pk(rng, n, P, a):
    w = np.arange(1, P + 1, dtype=np.float64) ** -a
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.minimum(np.searchsorted(cdf, rng.random(n)), P - 1).astype(np.int64)


# ----------------------------------------------------------- record formats --
@pytest.mark.parametrize("l0,linf,flags", [(2, 1, O.ACC_NSUM), (3, 2, O.ACC_SUM | O.ACC_NSUM),
                                           (8, 2, O.ACC_SUM | O.ACC_NSUM | O.ACC_NSUM2)])
@pytest.mark.parametrize("skew", [False, True])
def test_packed_records_match_oracle(device, l0, linf, flags, skew):
    """PDP_KEYS_PACKED (level-1 u64 record, tile-relative row; C3's format)
    keeps exactly the oracle's samples across many 65,536-row tiles."""
    rng = np.random.default_rng(40 + l0 + skew)
    n, U, P = 700_000, 300_000, 100_000
    pid = rng.integers(0, U, n)
    if skew:  # a third of the rows on 64 privacy ids: dense and sparse super-buckets
        pid[: n // 3] = rng.integers(0, 64, n // 3)
    pk = _zipf_pk(rng, n, P, 1.1) if skew else rng.integers(0, P, n)
    val = rng.uniform(-1.0, 11.0, n)
    spec = _spec(l0, linf, O.VALUE_F64, flags)
    plan = _plan(n, U, P, spec, key_format=3)
    assert plan.key_format == 3 and plan.n_buckets > 64  # two partition levels
    got = _gpu(device, pid, pk, val, U, P, spec, 77, key_format=3, row_offset=123)
    want = _oracle(pid, pk, val, U, P, spec, 77, plan.rand_shift, row_offset=123)
    _compare(got, want, _scale(pk, val, P, spec))


def test_packed_sparse_super_bucket_spans_many_tiles(device):
    """A super-bucket with one row per 65,536-row tile: its level-2 window spans
    more tiles than the LDS table holds (256), so rows beyond it find their
    tile by the global search."""
    rng = np.random.default_rng(41)
    n, U, P = 17_500_000, 300_000, 100_000
    spec = _spec(2, 1, O.VALUE_F64, O.ACC_NSUM)
    plan = _plan(n, U, P, spec, key_format=3)
    per_super = 1 << (plan.bucket_bits + 2)  # 37 super-buckets of 4 buckets (asserted below)
    sparse = 5
    pid = rng.integers(0, U - per_super, n)
    pid = np.where(pid >= sparse * per_super, pid + per_super, pid)  # no row in super-bucket 5 ...
    tiles = np.arange(0, n, 65536)
    pid[tiles] = sparse * per_super + rng.integers(0, per_super, len(tiles))  # ... except one per tile
    assert len(tiles) > 256
    pk = rng.integers(0, P, n)
    val = rng.uniform(0.0, 10.0, n)
    got = _gpu(device, pid, pk, val, U, P, spec, 5, key_format=3)
    want = _oracle(pid, pk, val, U, P, spec, 5, plan.rand_shift)
    _compare(got, want, _scale(pk, val, P, spec))


# ---------------------------------------------------------------------- C1 --
def test_c1_movie_view_matches_oracle(device):
    """BASELINE config 1 itself: 1e6 movie_view rows
    (oracle/local_backend_port.movie_view_rows, the CPU baseline's input),
    COUNT + SUM of int ratings clipped to [1, 5], L0 = 2, Linf = 1 (both
    samplings fire: ~10 rows per user, Zipf movies).  Movie ids are dense
    codes (17,771 partitions, code 0 unused).  Counts, privacy-id counts and
    the int64 SUM bit-exact against the oracle (the auto plan)."""
    from oracle.local_backend_port import movie_view_rows
    from pipelinedp_amd import executor as X
    rows = np.asarray(movie_view_rows(1_000_000, seed=0), dtype=np.int64)
    pid, pk, val = rows[:, 0].copy(), rows[:, 1].copy(), rows[:, 2].copy()
    U, P = 100_000, 17_771
    spec = X.BoundingSpec(l0=2, linf=1, value_kind=O.VALUE_I64, flags=O.ACC_SUM | O.SUM_INT, min_value=1,
                          max_value=5, middle=3.0)
    plan = _plan(len(pid), U, P, spec)
    want = _oracle(pid, pk, val, U, P, spec, 1234, plan.rand_shift)
    got = _gpu(device, pid, pk, val, U, P, spec, 1234)
    for k in ("privacy_id_count", "count", "sum"):
        np.testing.assert_array_equal(got[k], want[k])
    assert (got["count"] == got["privacy_id_count"]).all()  # Linf = 1: one row per kept pair
    assert got["privacy_id_count"].sum() < len(pid)  # cross-partition sampling fired


# ---------------------------------------------------------------------- C2 --
def _c2(seed=1):
    rng = np.random.default_rng(seed)
    n, U, P = 100_000_000, 1_000_000, 100_000
    pid = rng.integers(0, U, n)
    pk = rng.integers(0, P, n)
    val = np.clip(rng.normal(5.0, 3.0, n), 0.0, 10.0)
    return pid, pk, val, U, P


@pytest.mark.timeout(900)
def test_c2_full_scale_sampling_matches_oracle(device):
    """C2 throughput variant (L0 = 8, Linf = 2: both samplings fire) at the
    full 1e8 rows, COUNT + SUM + MEAN accumulators."""
    pid, pk, val, U, P = _c2()
    spec = _spec(8, 2, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM)
    plan = _plan(len(pid), U, P, spec)
    assert plan.algorithm == 2 and plan.key_format == 3  # the bench's plan: bucketed, packed level-1 records
    got = _gpu(device, pid, pk, val, U, P, spec, 0xC2)
    want = _oracle(pid, pk, val, U, P, spec, 0xC2, plan.rand_shift)
    _compare(got, want, _scale(pk, val, P, spec))
    assert got["count"].sum() < len(pid)  # sampling fired


@pytest.mark.timeout(900)
def test_c2_full_scale_parity_variant_exact_groupby(device):
    """C2 parity variant: L0 := max distinct partitions per privacy id, Linf :=
    max rows per (pid, pk) from the data, so nothing is sampled: counts and
    privacy-id counts equal an exact group-by; sums within 1e-9."""
    pid, pk, val, U, P = _c2()
    key = pid * P + pk
    pairs, rows_per_pair = np.unique(key, return_counts=True)
    l0 = int(np.bincount(pairs // P, minlength=U).max())
    linf = int(rows_per_pair.max())
    spec = _spec(l0, linf, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM)
    got = _gpu(device, pid, pk, val, U, P, spec, 3)
    np.testing.assert_array_equal(got["count"], np.bincount(pk, minlength=P))
    np.testing.assert_array_equal(got["privacy_id_count"], np.bincount(pairs % P, minlength=P))
    sc = _scale(pk, val, P, spec)
    assert np.all(np.abs(got["sum"] - np.bincount(pk, weights=val, minlength=P)) <= FLOAT_RTOL * sc)
    assert np.all(np.abs(got["normalized_sum"] - np.bincount(pk, weights=val - 5.0, minlength=P)) <= FLOAT_RTOL * sc)


# ---------------------------------------------------------------------- C3 --
@pytest.mark.timeout(900)
def test_c3_full_scale_identities(device):
    """C3 at 1e9 rows on one GPU (the bench's workload and plan): with Linf = 1
    every kept pair keeps one row; the kept pairs number exactly
    sum over privacy ids of min(L0, distinct partitions) (torch group-by on
    the device); normalized sums are bounded by the clipping."""
    import torch
    from pipelinedp_amd import executor as X
    import bench
    n, U, P = bench.C3["rows"], bench.C3["privacy_ids"], bench.C3["partitions"]
    pid, pk, val = bench.gen_c3(n, U, P, 0, 1, device, 2000)
    bounding, _, _ = bench.build_plan(bench.C3["l0"], bench.C3["linf"])
    plan = X.bound_plan(n, U, P, bounding)
    assert plan.key_format == 3  # PACKED
    acc = X.bound_and_reduce(pid, pk, val, n_privacy_ids=U, n_partitions=P, bounding=bounding, seed=99)
    pidc = acc["privacy_id_count"]
    kept_pairs = int(pidc.sum())
    assert int(acc["count"].sum()) == kept_pairs
    assert bool((acc["count"] == pidc).all())
    assert float(acc["normalized_sum"].abs().max()) <= 5.0 * float(acc["count"].max()) + 1e-6
    del acc, val
    key = pid * P + pk
    del pk
    distinct = torch.unique(key)  # sorted distinct (pid, pk) pairs
    del key
    per_pid = torch.bincount(distinct // P, minlength=U)
    del distinct
    assert kept_pairs == int(torch.clamp(per_pid, max=bench.C3["l0"]).sum())
    del pid, per_pid
    torch.cuda.empty_cache()


def _c3_shape(n, seed):
    rng = np.random.default_rng(seed)
    U, P = n // 100, 1_000_000
    return rng.integers(0, U, n), _zipf_pk(rng, n, P, 1.1), rng.random(n) * 10.0, U, P


@pytest.mark.timeout(600)
def test_c3_shape_packed_matches_oracle(device):
    """C3-shaped 5e7 rows (Zipf(1.1) over 1e6 partitions, 100 rows per privacy
    id, L0 = 2, Linf = 1): AUTO picks the PACKED records, as at 1e9."""
    pid, pk, val, U, P = _c3_shape(50_000_000, 2)
    spec = _spec(2, 1, O.VALUE_F64, O.ACC_NSUM)
    plan = _plan(len(pid), U, P, spec)
    assert plan.algorithm == 2 and plan.key_format == 3
    got = _gpu(device, pid, pk, val, U, P, spec, 17)
    want = _oracle(pid, pk, val, U, P, spec, 17, plan.rand_shift)
    _compare(got, want, _scale(pk, val, P, spec))


@pytest.mark.timeout(600)
def test_c3_slice_wide_records_match_oracle(device):
    """A 1e7-row C3 slice with the wide (u64 key + row) records forced."""
    pid, pk, val, U, P = _c3_shape(10_000_000, 3)
    spec = _spec(2, 1, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM)
    plan = _plan(len(pid), U, P, spec, key_format=1)
    got = _gpu(device, pid, pk, val, U, P, spec, 18, key_format=1)
    want = _oracle(pid, pk, val, U, P, spec, 18, plan.rand_shift)
    _compare(got, want, _scale(pk, val, P, spec))


# ---------------------------------------------------------------------- C4 --
@pytest.mark.timeout(900)
def test_c4_shape_matches_oracle_with_selection_and_noise(device):
    """C4's shape on one GPU: P = 1e7 uniform partitions, U = 1e8 privacy ids,
    1e8 rows, VARIANCE + PRIVACY_ID_COUNT accumulators, L0 = 4, Linf = 2; then
    truncated-geometric selection and secure Gaussian VARIANCE / PID noise on
    the 1e7 partitions, all against the oracle."""
    import torch
    from pipelinedp_amd import dp_computations as dpc
    from pipelinedp_amd import executor as X
    rng = np.random.default_rng(4)
    n, U, P = 100_000_000, 100_000_000, 10_000_000
    pid = rng.integers(0, U, n)
    pk = rng.integers(0, P, n)
    val = rng.random(n) * 10.0
    spec = _spec(4, 2, O.VALUE_F64, O.ACC_NSUM | O.ACC_NSUM2)
    plan = _plan(n, U, P, spec)
    got = _gpu(device, pid, pk, val, U, P, spec, 0xC4)
    want = _oracle(pid, pk, val, U, P, spec, 0xC4, plan.rand_shift)
    _compare(got, want, _scale(pk, val, P, spec))
    del pid, pk, val
    # selection + noise on the device accumulators vs the oracle
    acc = {k: (None if v is None else torch.as_tensor(v).to(device)) for k, v in got.items()}
    table = dpc.truncated_geometric_keep_table(4.0, 1e-6, 4)
    sel = X.SelectionSpec(strategy=O.SELECT_TRUNCATED_GEOMETRIC, keep_prob=table)
    ops = [X.MetricOpSpec(kind=O.OP_VARIANCE, out_col=(0, 1, 2, 3),
                          noise=tuple(dpc.gaussian_noise_params(s) for s in (3.0, 20.0, 150.0)), middle=5.0),
           X.MetricOpSpec(kind=O.OP_PRIVACY_ID_COUNT, out_col=(4,), noise=(dpc.gaussian_noise_params(2.5),))]
    index, out, n_kept = X.select_and_noise(acc, selection=sel, ops=ops, n_cols=5, seed_select=5, seed_noise=6)
    keep, _ = O.select(want["privacy_id_count"], O.SELECT_TRUNCATED_GEOMETRIC, keep_prob=table, seed=5)
    want_index = np.flatnonzero(keep)
    np.testing.assert_array_equal(index.cpu().numpy(), want_index)
    assert n_kept > 0
    wm = O.noise_metrics([o.as_dict() for o in ops], want_index, want, False, None, 6, n_cols=5)
    np.testing.assert_allclose(out.cpu().numpy()[:, :n_kept], wm, rtol=1e-9, atol=1e-9)
    # the same accumulators under GAUSSIAN_THRESHOLDING (SURVEY §8(d) C4's
    # second strategy; partition_selection.py:29-44, dp_engine.py:315-371):
    # sigma / threshold as DPEngine derives them for eps = 1/3, delta = 1e-6,
    # L0 = 4; kept set, noised privacy-id counts and metrics vs the oracle
    sigma, threshold = dpc.gaussian_thresholding_params(1.0 / 3, 1e-6, 4)
    gsel = X.SelectionSpec(strategy=O.SELECT_GAUSSIAN, noise=dpc.gaussian_noise_params(sigma),
                           threshold=threshold, want_noised_count=True)
    gops = ops + [X.MetricOpSpec(kind=O.OP_THRESHOLDED_PID, out_col=(5,))]
    gindex, gout, g_kept = X.select_and_noise(acc, selection=gsel, ops=gops, n_cols=6, seed_select=7,
                                              seed_noise=8)
    gkeep, gnoised = O.select(want["privacy_id_count"], O.SELECT_GAUSSIAN,
                              noise=dpc.gaussian_noise_params(sigma).as_dict(), threshold=threshold, seed=7)
    g_want_index = np.flatnonzero(gkeep)
    np.testing.assert_array_equal(gindex.cpu().numpy(), g_want_index)
    assert 0 < g_kept < int((want["privacy_id_count"] > 0).sum())  # the threshold drops some partitions
    gwm = O.noise_metrics([o.as_dict() for o in gops], g_want_index, want, False, gnoised, 8, n_cols=6)
    np.testing.assert_allclose(gout.cpu().numpy()[:, :g_kept], gwm, rtol=1e-9, atol=1e-9)


def test_c4_bucketing_packed_wide_records_match_oracle(device):
    """C4's per-GPU bucketing (U = 1.25e7 privacy ids -> 12,208 buckets of
    1,024, P = 1e7): PACKED level-1 records and WIDE ones from level 2 on
    (bucket + partition bits > 31), the tile-local level 1 counting buckets in
    u16 halves; 2e7 rows against the oracle, sampling firing."""
    rng = np.random.default_rng(44)
    n, U, P = 20_000_000, 12_500_000, 10_000_000
    pid = rng.integers(0, U, n)
    pid[:300_000] = rng.integers(0, 2_000, 300_000)  # a few heavy privacy ids
    pk = rng.integers(0, P, n)
    val = rng.random(n) * 10.0
    spec = _spec(4, 2, O.VALUE_F64, O.ACC_NSUM | O.ACC_NSUM2)
    plan = _plan(n, U, P, spec)
    assert plan.algorithm == 2 and plan.key_format == 5 and plan.n_buckets > 10_000  # PACKED64
    want = _oracle(pid, pk, val, U, P, spec, 0x4C4, plan.rand_shift)
    _compare(_gpu(device, pid, pk, val, U, P, spec, 0x4C4), want, _scale(pk, val, P, spec))
    assert _plan(n, U, P, spec, key_format=4).key_format == 4  # and PACKED_WIDE, asked for
    _compare(_gpu(device, pid, pk, val, U, P, spec, 0x4C4, key_format=4), want, _scale(pk, val, P, spec))


def test_many_buckets_wide_level2_fanout_matches_oracle(device):
    """34,180 buckets (U = 7e7 privacy ids, 2,048 per bucket): level 1 counts
    them in u16 halves and level 2 fans each super-bucket out to 512 buckets
    (the 1,024-destination LDS stage); 3e6 rows, mostly one per privacy id,
    plus a heavy id, against the oracle."""
    rng = np.random.default_rng(34)
    n, U, P = 3_000_000, 70_000_000, 100_000
    pid = rng.integers(0, U, n)
    pid[:50_000] = 123_456_789 % U
    pk = _zipf_pk(rng, n, P, 1.1)
    val = rng.random(n) * 10.0
    spec = _spec(2, 1, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM)
    plan = _plan(n, U, P, spec)
    assert plan.algorithm == 2 and plan.key_format == 3 and plan.n_buckets > 32_768
    got = _gpu(device, pid, pk, val, U, P, spec, 0x34)
    want = _oracle(pid, pk, val, U, P, spec, 0x34, plan.rand_shift)
    _compare(got, want, _scale(pk, val, P, spec))


# ---------------------------------------------------------------------- C5 --
@pytest.mark.timeout(900)
def test_c5_shape_heavy_tailed_privacy_ids_match_oracle(device):
    """C5's shape: rows per privacy id ~ discrete Pareto(1.5) capped at 1e6,
    privacy id 0 with exactly 1e6 rows (sample_fixed_per_key on a giant key,
    pipeline_backend.py:531-547), Zipf(1.1) partitions folded into 1e6,
    lognormal(1, 1) values clipped to [0, 20]; COUNT + SUM + MEAN, L0 = 4,
    Linf = 2."""
    rng = np.random.default_rng(5)
    U, P = 200_000, 1_000_000
    per = np.minimum(np.floor(rng.pareto(1.5, U) * 20 + 1), 1_000_000).astype(np.int64)
    per[0] = 1_000_000
    pid = np.repeat(np.arange(U, dtype=np.int64), per)
    pid = pid[rng.permutation(len(pid))]
    n = len(pid)
    pk = _zipf_pk(rng, n, P, 1.1)
    val = np.clip(rng.lognormal(1.0, 1.0, n), 0.0, 20.0)
    spec = _spec(4, 2, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM, 0.0, 20.0)
    plan = _plan(n, U, P, spec)
    assert plan.algorithm == 2
    got = _gpu(device, pid, pk, val, U, P, spec, 0xC5)
    want = _oracle(pid, pk, val, U, P, spec, 0xC5, plan.rand_shift)
    _compare(got, want, _scale(pk, val, P, spec))


@pytest.mark.timeout(900)
def test_c5_shard_plan_matches_oracle(device):
    """The plan the C5 bench times on each GPU (bench.py C5: P = 1e7 Zipf(1.1),
    U = 1.25e7): PACKED_WIDE records and the two-level range merge (coarse
    ranges, then k_split_* / k_fine_reduce), on 5e7 rows with rows per privacy
    id ~ discrete Pareto(1.5), privacy id 0 holding 1e6 rows (sample_fixed_per_key
    on a giant key, pipeline_backend.py:531-547), lognormal(1, 1) values
    clipped to [0, 20]; COUNT + SUM + MEAN accumulators, L0 = 4, Linf = 2,
    against the oracle (VERDICT r02 missing #2)."""
    from pipelinedp_amd import _native as N
    rng = np.random.default_rng(55)
    U, P, n_target = 12_500_000, 10_000_000, 50_000_000
    per = np.floor(rng.pareto(1.5, U) + 1.0)
    per = np.minimum(per * (n_target / per.sum()), 1_000_000)
    per = np.maximum(np.floor(per), 0).astype(np.int64)
    per[0] = 1_000_000
    pid = np.repeat(np.arange(U, dtype=np.int64), per)
    pid = pid[rng.permutation(len(pid))]
    n = len(pid)
    assert n >= n_target * 0.9
    pk = _zipf_pk(rng, n, P, 1.1)
    val = np.clip(rng.lognormal(1.0, 1.0, n), 0.0, 20.0)
    spec = _spec(4, 2, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM, 0.0, 20.0)
    plan = _plan(n, U, P, spec)
    assert plan.algorithm == N.ALGO_BUCKETED and plan.key_format == N.KEYS_PACKED64
    assert plan.merge == N.MERGE_RANGES and plan.n_ranges < -(-P // 2048)  # coarse ranges: two-level merge
    got = _gpu(device, pid, pk, val, U, P, spec, 0x5C5)
    want = _oracle(pid, pk, val, U, P, spec, 0x5C5, plan.rand_shift)
    _compare(got, want, _scale(pk, val, P, spec))
    assert got["privacy_id_count"].sum() > 0
