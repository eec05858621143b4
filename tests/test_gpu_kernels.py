"""GPU parity of the HIP kernels (through the C ABI) against the CPU oracle.

The oracle (oracle/columnar.py) reproduces the kernels' counter-based
sampling priorities and Philox streams, so integer outputs (privacy-id counts,
counts, int sums, keep decisions) must match bit-exactly and fp64 sums/noised
metrics within 1e-9 relative (tolerance stated per assertion).
"""
import numpy as np
import pytest

from oracle import columnar as O

pytestmark = pytest.mark.gpu

FLOAT_RTOL = 1e-9  # fp64 sums: relative to the sum of |terms| (order-dependent rounding)


def _gen(seed, n, U, P, value_kind, skew=False):
    rng = np.random.default_rng(seed)
    pid = rng.integers(0, U, n, dtype=np.int64)
    if skew:
        pk = np.minimum(rng.zipf(1.3, n) - 1, P - 1).astype(np.int64)
    else:
        pk = rng.integers(0, P, n, dtype=np.int64)
    if value_kind == O.VALUE_F64:
        val = rng.normal(5.0, 3.0, n)
    elif value_kind == O.VALUE_I64:
        val = rng.integers(-3, 12, n, dtype=np.int64)
    else:
        val = None
    return pid, pk, val


def _rand_shift(n, U, P, spec, algorithm=0, bucket_threads=0):
    from pipelinedp_amd import executor as X
    return X.bound_plan(n, U, P, spec, algorithm, bucket_threads=bucket_threads).rand_shift


def _run_gpu(device, pid, pk, val, U, P, spec, seed, allowed=None, row_offset=0, algorithm=0, merge=0,
             key_format=0, bucket_threads=0):
    import torch
    from pipelinedp_amd import executor as X
    tp = torch.as_tensor(pid).to(device)
    tk = torch.as_tensor(pk).to(device)
    tv = None if val is None else torch.as_tensor(val).to(device)
    ta = None if allowed is None else torch.as_tensor(allowed.astype(np.uint8)).to(device)
    acc = X.bound_and_reduce(tp, tk, tv, n_privacy_ids=U, n_partitions=P, bounding=spec, seed=seed,
                             allowed=ta, row_offset=row_offset, algorithm=algorithm, merge=merge,
                             key_format=key_format, bucket_threads=bucket_threads)
    torch.cuda.synchronize()
    return {k: (None if v is None else v.cpu().numpy()) for k, v in acc.items()}


def _oracle(pid, pk, val, U, P, spec, seed, allowed=None, row_offset=0, algorithm=0, bucket_threads=0):
    return O.bound_and_reduce(pid, pk, val, n_privacy_ids=U, n_partitions=P, l0=spec.l0,
                              linf=spec.linf, value_kind=spec.value_kind, flags=spec.flags,
                              min_value=spec.min_value, max_value=spec.max_value,
                              middle=spec.middle, min_sum=spec.min_sum, max_sum=spec.max_sum,
                              seed=seed, row_offset=row_offset, allowed=allowed,
                              rand_shift=_rand_shift(len(pid), U, P, spec, algorithm, bucket_threads))


def _abs_scale(pid, pk, val, P, lo, hi, mid):
    """Per-partition sum of |terms| for the fp tolerance."""
    s = np.zeros(P)
    if val is not None:
        np.add.at(s, pk, np.abs(np.clip(val.astype(np.float64), lo, hi)) + abs(mid) + 1.0)
    return s + 1.0


def _compare(got, want, scale):
    np.testing.assert_array_equal(got["privacy_id_count"], want["privacy_id_count"])
    np.testing.assert_array_equal(got["count"], want["count"])
    for k in ("sum", "normalized_sum", "normalized_sum_sq"):
        if got[k] is None:
            continue
        if got[k].dtype == np.int64:
            np.testing.assert_array_equal(got[k], want[k])
        else:
            sc = scale if k != "normalized_sum_sq" else scale * scale
            assert np.all(np.abs(got[k] - want[k]) <= FLOAT_RTOL * sc), k


CASES = [
    # (l0, linf, value_kind, flags, lo, hi, per-partition bounds)
    (1, 1, O.VALUE_NONE, 0, 0, 0, None),
    (2, 1, O.VALUE_F64, O.ACC_SUM, 0.0, 10.0, None),
    (3, 2, O.VALUE_F64, O.ACC_NSUM, 0.0, 10.0, None),
    (4, 3, O.VALUE_F64, O.ACC_NSUM | O.ACC_NSUM2, -1.0, 8.0, None),
    (8, 2, O.VALUE_I64, O.ACC_SUM | O.SUM_INT, 0, 7, None),
    (5, 0, O.VALUE_F64, O.SUM_PER_PARTITION, 0, 0, (-3.0, 20.0)),
    (2, 0, O.VALUE_I64, O.SUM_PER_PARTITION | O.SUM_INT, 0, 0, (-3, 9)),
    (2, 2, O.VALUE_I64, O.SUM_PER_PARTITION | O.SUM_INT, 0, 0, (0, 5)),
    (16, 4, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM | O.ACC_NSUM2, 1.0, 6.0, None),
    (256, 256, O.VALUE_F64, O.ACC_SUM, 0.0, 10.0, None),
]


# name -> (PDP_ALGO_*, PDP_MERGE_*, PDP_KEYS_*)
ALGOS = {"global": (1, 0, 0), "bucketed-atomic-wide": (2, 1, 1), "bucketed-ranges-wide": (2, 2, 1),
         "bucketed-atomic-compact": (2, 1, 2), "bucketed-ranges-compact": (2, 2, 2)}


@pytest.mark.parametrize("case", CASES, ids=[f"l0={c[0]}-linf={c[1]}-f={c[3]}" for c in CASES])
@pytest.mark.parametrize("skew", [False, True])
@pytest.mark.parametrize("algo", list(ALGOS))
def test_bound_and_reduce_matches_oracle(device, case, skew, algo):
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import executor as X
    l0, linf, vk, flags, lo, hi, pp = case
    U, P, n = 700, 257, 40000
    pid, pk, val = _gen(11 + l0 + linf, n, U, P, vk, skew)
    mid = lo + (hi - lo) / 2 if vk != O.VALUE_NONE else 0.0
    spec = X.BoundingSpec(l0=l0, linf=linf, value_kind=vk, flags=flags, min_value=lo, max_value=hi,
                          middle=mid, min_sum=pp[0] if pp else 0.0, max_sum=pp[1] if pp else 0.0)
    seed = 0x1234_5678_9ABC_DEF0 + l0
    try:
        X.bound_plan(n, U, P, spec, *ALGOS[algo])
    except N.NativeLibraryError:
        pytest.skip(f"{algo} infeasible for l0={l0}, linf={linf}")
    got = _run_gpu(device, pid, pk, val, U, P, spec, seed, row_offset=77, algorithm=ALGOS[algo][0],
                   merge=ALGOS[algo][1], key_format=ALGOS[algo][2])
    want = _oracle(pid, pk, val, U, P, spec, seed, row_offset=77, algorithm=ALGOS[algo][0])
    _compare(got, want, _abs_scale(pid, pk, val, P, lo, hi, mid))


def test_no_sampling_keeps_everything(device):
    """When l0 >= distinct partitions per pid and linf >= rows per pair nothing
    is dropped: counts are the raw group counts (exact)."""
    from pipelinedp_amd import executor as X
    rng = np.random.default_rng(3)
    U, P, n = 300, 50, 6000
    pid = rng.integers(0, U, n)
    pk = rng.integers(0, P, n)
    val = rng.normal(2, 1, n)
    spec = X.BoundingSpec(l0=64, linf=64, value_kind=O.VALUE_F64, flags=O.ACC_SUM, min_value=-100,
                          max_value=100, middle=0.0)
    got = _run_gpu(device, pid, pk, val, U, P, spec, 5)
    cnt = np.bincount(pk, minlength=P)
    np.testing.assert_array_equal(got["count"], cnt)
    pairs = np.unique(pid * P + pk)
    np.testing.assert_array_equal(got["privacy_id_count"], np.bincount(pairs % P, minlength=P))
    ref = np.zeros(P)
    np.add.at(ref, pk, val)
    assert np.allclose(got["sum"], ref, rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("algo", list(ALGOS))
def test_public_filter(device, algo):
    from pipelinedp_amd import executor as X
    U, P, n = 200, 40, 5000
    pid, pk, val = _gen(7, n, U, P, O.VALUE_F64)
    allowed = np.zeros(P, dtype=bool)
    allowed[::3] = True
    spec = X.BoundingSpec(l0=2, linf=1, value_kind=O.VALUE_F64, flags=O.ACC_SUM, min_value=0, max_value=10)
    got = _run_gpu(device, pid, pk, val, U, P, spec, 99, allowed=allowed, algorithm=ALGOS[algo][0],
                   merge=ALGOS[algo][1], key_format=ALGOS[algo][2])
    want = _oracle(pid, pk, val, U, P, spec, 99, allowed=allowed, algorithm=ALGOS[algo][0])
    _compare(got, want, _abs_scale(pid, pk, val, P, 0, 10, 0))
    assert np.all(got["count"][~allowed] == 0)


@pytest.mark.parametrize("algo", list(ALGOS))
@pytest.mark.parametrize("bad", ["pid", "pk"])
def test_out_of_range_keys_raise(device, algo, bad):
    import torch
    from pipelinedp_amd import executor as X
    pid = torch.tensor([0, 1, 5 if bad == "pid" else 2], dtype=torch.int64, device=device)
    pk = torch.tensor([0, 1, 7 if bad == "pk" else 1], dtype=torch.int64, device=device)
    spec = X.BoundingSpec(l0=1, linf=1, value_kind=O.VALUE_NONE, flags=0)
    with pytest.raises(ValueError):
        X.bound_and_reduce(pid, pk, None, n_privacy_ids=3, n_partitions=2, bounding=spec, seed=1,
                           algorithm=ALGOS[algo][0], merge=ALGOS[algo][1], key_format=ALGOS[algo][2])


@pytest.mark.parametrize("heavy", [False, True])
def test_algorithms_agree_at_scale(device, heavy):
    """Bucketed and global paths keep the same samples on a larger skewed input
    (one privacy id with 200k rows when heavy)."""
    import torch
    from pipelinedp_amd import executor as X
    rng = np.random.default_rng(8)
    n, U, P = 2_000_000, 50_000, 30_000
    pid = rng.integers(0, U, n)
    if heavy:
        pid[:200_000] = 17
    pk = np.minimum(rng.zipf(1.2, n) - 1, P - 1)
    val = rng.normal(5, 3, n)
    spec = X.BoundingSpec(l0=4, linf=2, value_kind=O.VALUE_F64, flags=O.ACC_SUM | O.ACC_NSUM,
                          min_value=0.0, max_value=10.0, middle=5.0)
    a = _run_gpu(device, pid, pk, val, U, P, spec, 3, algorithm=1)
    sc = _abs_scale(pid, pk, val, P, 0.0, 10.0, 5.0)
    for merge, keys in ((1, 1), (2, 1), (1, 2), (2, 2)):  # 30k partitions = 15 merge ranges
        b = _run_gpu(device, pid, pk, val, U, P, spec, 3, algorithm=2, merge=merge, key_format=keys)
        np.testing.assert_array_equal(a["privacy_id_count"], b["privacy_id_count"])
        np.testing.assert_array_equal(a["count"], b["count"])
        assert np.all(np.abs(a["sum"] - b["sum"]) <= FLOAT_RTOL * sc)
        assert np.all(np.abs(a["normalized_sum"] - b["normalized_sum"]) <= FLOAT_RTOL * sc)


@pytest.mark.parametrize("P", [2047, 2048, 2049, 100_000, 2_000_000])
def test_range_merge_matches_oracle_many_ranges(device, P):
    """Range merge at range boundaries and up to the 1024-range limit (P = 2M)."""
    from pipelinedp_amd import executor as X
    n, U = 300_000, 20_000
    pid, pk, val = _gen(P, n, U, P, O.VALUE_I64)
    spec = X.BoundingSpec(l0=3, linf=2, value_kind=O.VALUE_I64, flags=O.ACC_SUM | O.SUM_INT | O.ACC_NSUM,
                          min_value=0, max_value=9, middle=4.5)
    info = X.bound_plan(n, U, P, spec, 2, 2)
    assert info.merge == 2 and info.n_ranges == (P + 2047) // 2048
    got = _run_gpu(device, pid, pk, val, U, P, spec, 21, algorithm=2, merge=2)
    want = _oracle(pid, pk, val, U, P, spec, 21, algorithm=2)
    _compare(got, want, _abs_scale(pid, pk, val, P, 0, 9, 4.5))


@pytest.mark.parametrize("P,skew", [(2_097_153, False), (10_000_000, False), (10_000_000, True),
                                     (40_000_000, False)])
def test_two_level_range_merge_matches_oracle(device, P, skew):
    """More than 1024 ranges of 2,048 partitions: kept pairs grouped by <= 256
    coarse ranges in the bucket kernel, re-sorted by fine range (k_split_*),
    summed per fine range (k_fine_reduce); Zipf-hot partitions included."""
    from pipelinedp_amd import executor as X
    n, U = 400_000, 30_000
    rng = np.random.default_rng(P % 1000 + skew)
    pid = rng.integers(0, U, n)
    pk = (np.minimum(rng.zipf(1.2, n) - 1, P - 1) if skew else rng.integers(0, P, n)).astype(np.int64)
    val = rng.normal(4.0, 3.0, n)
    spec = X.BoundingSpec(l0=3, linf=2, value_kind=O.VALUE_F64,
                          flags=O.ACC_SUM | O.ACC_NSUM | O.ACC_NSUM2, min_value=0.0, max_value=9.0, middle=4.5)
    info = X.bound_plan(n, U, P, spec)
    assert info.merge == 2 and info.n_ranges <= 256 and (P + 2047) // 2048 > 1024
    got = _run_gpu(device, pid, pk, val, U, P, spec, 33)
    want = _oracle(pid, pk, val, U, P, spec, 33)
    _compare(got, want, _abs_scale(pid, pk, val, P, 0.0, 9.0, 4.5))


@pytest.mark.parametrize("P,keys", [(5_000, 3), (5_000, 5), (10_000_000, 0), (1_500_000, 0)])
def test_half_size_buckets_match_oracle(device, P, keys):
    """bucket_threads = 512: buckets of half as many privacy ids (two
    workgroups per CU), single-level and two-level range merges, a heavy id."""
    from pipelinedp_amd import executor as X
    rng = np.random.default_rng(P + keys)
    n, U = 1_200_000, 200_000
    pid = rng.integers(0, U, n)
    pid[:30_000] = 4_321
    pk = np.minimum(rng.zipf(1.3, n) - 1, P - 1).astype(np.int64)
    val = rng.normal(4.0, 3.0, n)
    spec = X.BoundingSpec(l0=3, linf=2, value_kind=O.VALUE_F64,
                          flags=O.ACC_SUM | O.ACC_NSUM | O.ACC_NSUM2, min_value=0.0, max_value=9.0, middle=4.5)
    full = X.bound_plan(n, U, P, spec, 2, 2, keys)
    half = X.bound_plan(n, U, P, spec, 2, 2, keys, bucket_threads=512)
    assert full.bucket_threads == 1024
    if 512 < half.n_ranges <= 1024:  # one thread per range: no half-size buckets
        assert half.bucket_threads == 1024
        return
    assert half.bucket_threads == 512 and half.bucket_bits == full.bucket_bits - 1 and half.lds_bytes <= 80 * 1024
    got = _run_gpu(device, pid, pk, val, U, P, spec, 91, algorithm=2, merge=2, key_format=keys, bucket_threads=512)
    want = _oracle(pid, pk, val, U, P, spec, 91, algorithm=2, bucket_threads=512)
    _compare(got, want, _abs_scale(pid, pk, val, P, 0.0, 9.0, 4.5))


@pytest.mark.parametrize("keys", [1, 2, 3, 4, 5], ids=["wide", "compact", "packed", "packed-wide", "packed64"])
@pytest.mark.parametrize("public", [False, True])
def test_tile_local_partition_matches_oracle(device, keys, public):
    """The tile-local level 1 (stage blocks + per-stage super-bucket offsets,
    bucket counts from its LDS) and the level 2 that gathers those runs, for
    every record format: 23 tiles (two level-2 groups, a partial last stage),
    37 super-buckets, a heavy privacy id, dead (non-public) rows."""
    from pipelinedp_amd import executor as X
    rng = np.random.default_rng(21 + keys)
    n, U, P = 1_500_123, 300_000, 5_000
    pid = rng.integers(0, U, n)
    pid[:40_000] = 12_345
    pk = np.minimum(rng.zipf(1.3, n) - 1, P - 1).astype(np.int64)
    val = rng.normal(4.0, 3.0, n)
    allowed = (np.arange(P) % 5 != 1) if public else None
    spec = X.BoundingSpec(l0=3, linf=2, value_kind=O.VALUE_F64, flags=O.ACC_SUM | O.ACC_NSUM,
                          min_value=0.0, max_value=9.0, middle=4.5)
    info = X.bound_plan(n, U, P, spec, 2, 2, keys)
    assert info.algorithm == 2 and info.n_buckets > 64 and info.key_format == keys
    got = _run_gpu(device, pid, pk, val, U, P, spec, 71, allowed=allowed, algorithm=2, merge=2, key_format=keys)
    want = _oracle(pid, pk, val, U, P, spec, 71, allowed=allowed, algorithm=2)
    _compare(got, want, _abs_scale(pid, pk, val, P, 0.0, 9.0, 4.5))


@pytest.mark.parametrize("n", [1, 1000, 65_535, 65_537, 8 * 65_536 + 8_191])
def test_tile_local_partition_edge_sizes(device, n):
    """Tile-local partition passes at sizes around their stage / tile /
    level-2 group boundaries, with many more buckets than rows (empty runs)."""
    from pipelinedp_amd import executor as X
    rng = np.random.default_rng(n)
    U, P = 300_000, 5_000
    pid = rng.integers(0, U, n)
    pk = rng.integers(0, P, n)
    val = rng.normal(4.0, 3.0, n)
    spec = X.BoundingSpec(l0=3, linf=2, value_kind=O.VALUE_F64, flags=O.ACC_SUM | O.ACC_NSUM,
                          min_value=0.0, max_value=9.0, middle=4.5)
    info = X.bound_plan(n, U, P, spec)
    assert info.algorithm == 2 and info.n_buckets > 64 and info.key_format == 3
    got = _run_gpu(device, pid, pk, val, U, P, spec, 5)
    want = _oracle(pid, pk, val, U, P, spec, 5)
    _compare(got, want, _abs_scale(pid, pk, val, P, 0.0, 9.0, 4.5))


def test_tile_local_partition_unaligned_columns(device):
    """Key columns that do not start on a 16-byte boundary (views one element
    in) take the scalar-load path of level 1."""
    import torch
    from pipelinedp_amd import executor as X
    rng = np.random.default_rng(17)
    n, U, P = 700_001, 300_000, 5_000
    pid = rng.integers(0, U, n + 1)
    pk = rng.integers(0, P, n + 1)
    val = rng.normal(4.0, 3.0, n + 1)
    spec = X.BoundingSpec(l0=3, linf=2, value_kind=O.VALUE_F64, flags=O.ACC_SUM | O.ACC_NSUM,
                          min_value=0.0, max_value=9.0, middle=4.5)
    tp = torch.as_tensor(pid).to(device)[1:]
    tk = torch.as_tensor(pk).to(device)[1:]
    tv = torch.as_tensor(val).to(device)[1:]
    assert tp.data_ptr() % 16 != 0
    acc = X.bound_and_reduce(tp, tk, tv, n_privacy_ids=U, n_partitions=P, bounding=spec, seed=9)
    torch.cuda.synchronize()
    got = {k: (None if v is None else v.cpu().numpy()) for k, v in acc.items()}
    want = _oracle(pid[1:], pk[1:], val[1:], U, P, spec, 9)
    _compare(got, want, _abs_scale(pid[1:], pk[1:], val[1:], P, 0.0, 9.0, 4.5))


def test_compact_records_chosen_when_they_fit():
    """C2 (U = 1e6, P = 1e5, L0 = 8, Linf = 2) moves 8-byte records: PACKED
    (one u64 per row) through the tile-local level 1, then COMPACT pairs; at
    P = 1e7 the level-1 record stays PACKED and level 2 on moves PACKED64
    records (row, bucket-local pid and partition in one u64) -- 8 bytes, not
    the 12 of PACKED_WIDE's u64 key + row."""
    from pipelinedp_amd import executor as X
    spec = X.BoundingSpec(l0=8, linf=2, value_kind=O.VALUE_F64, flags=O.ACC_NSUM, min_value=0.0,
                          max_value=10.0, middle=5.0)
    assert X.bound_plan(100_000_000, 1_000_000, 100_000, spec).key_format == 3
    assert X.bound_plan(100_000_000, 1_000_000, 10_000_000, spec).key_format == 5
    assert X.bound_plan(100_000_000, 1_000_000, 10_000_000, spec, key_format=4).key_format == 4


def test_empty_input(device):
    import torch
    from pipelinedp_amd import executor as X
    e = torch.zeros(0, dtype=torch.int64, device=device)
    spec = X.BoundingSpec(l0=2, linf=1, value_kind=O.VALUE_F64, flags=O.ACC_SUM, min_value=0, max_value=1)
    acc = X.bound_and_reduce(e, e, torch.zeros(0, dtype=torch.float64, device=device), n_privacy_ids=4,
                             n_partitions=3, bounding=spec, seed=1)
    assert int(acc["count"].sum()) == 0


@pytest.mark.parametrize("strategy", [O.SELECT_TRUNCATED_GEOMETRIC, O.SELECT_LAPLACE,
                                      O.SELECT_GAUSSIAN, O.SELECT_ALL_NONEMPTY, O.SELECT_PUBLIC])
@pytest.mark.parametrize("pre_threshold", [0, 3])
def test_select_and_noise_matches_oracle(device, strategy, pre_threshold):
    import torch
    from pipelinedp_amd import executor as X
    rng = np.random.default_rng(strategy * 10 + pre_threshold)
    P = 5000
    rc = rng.integers(0, 40, P).astype(np.int64)
    rc[rng.random(P) < 0.2] = 0
    acc_np = {
        "privacy_id_count": rc,
        "count": rc * 2,
        "sum": rng.normal(0, 10, P),
        "normalized_sum": rng.normal(0, 10, P),
        "normalized_sum_sq": np.abs(rng.normal(0, 10, P)),
    }
    acc = {k: torch.as_tensor(v).to(device) for k, v in acc_np.items()}
    table = np.minimum(1.0, 1e-3 * (np.exp(0.3 * np.arange(40)) - 1))
    table[0] = 0.0
    pub = (rng.random(P) < 0.5).astype(np.uint8)
    from pipelinedp_amd import dp_computations as dpc
    lap, gau = dpc.laplace_noise_params, dpc.gaussian_noise_params
    sel_noise = gau(2.5) if strategy == O.SELECT_GAUSSIAN else lap(0.4, 1.0)
    sel = X.SelectionSpec(strategy=strategy, max_rows_per_privacy_id=1, pre_threshold=pre_threshold,
                          keep_prob=table, noise=sel_noise, threshold=12.0,
                          want_noised_count=True)
    ops = [
        X.MetricOpSpec(kind=O.OP_COUNT, out_col=(0,), noise=(lap(2.0, 3.0),)),
        X.MetricOpSpec(kind=O.OP_SUM, out_col=(1,), noise=(gau(3.0),)),
        X.MetricOpSpec(kind=O.OP_MEAN, out_col=(2, 3, 4), noise=(lap(1.0, 1.0), lap(0.5, 1.0)), middle=5.0),
        X.MetricOpSpec(kind=O.OP_VARIANCE, out_col=(5, 6, 7, 8), noise=(gau(1.0), gau(2.0), gau(3.0)),
                       middle=5.0),
        X.MetricOpSpec(kind=O.OP_PRIVACY_ID_COUNT, out_col=(9,), noise=(gau(0.7),)),
    ]
    if strategy in (O.SELECT_LAPLACE, O.SELECT_GAUSSIAN):
        ops.append(X.MetricOpSpec(kind=O.OP_THRESHOLDED_PID, out_col=(10,)))
    n_cols = 1 + max(c for o in ops for c in o.out_col)
    index, out, n_kept = X.select_and_noise(acc, selection=sel, ops=ops, n_cols=n_cols, seed_select=42,
                                            seed_noise=4242, partition_offset=1000,
                                            public_mask=torch.as_tensor(pub).to(device))
    keep, noised = O.select(rc, strategy, max_rows_per_privacy_id=1, pre_threshold=pre_threshold,
                            keep_prob=table, noise=sel_noise.as_dict(), threshold=12.0, public_mask=pub, seed=42,
                            partition_offset=1000)
    want_index = np.flatnonzero(keep)
    np.testing.assert_array_equal(index.cpu().numpy(), want_index)
    want = O.noise_metrics([o.as_dict() for o in ops], want_index, acc_np, False, noised, 4242,
                           partition_offset=1000, n_cols=n_cols)
    got = out.cpu().numpy()[:, :n_kept]
    # the secure samplers' draws are grid integers (bit-exact); the metrics
    # built from them (mean, variance) divide in fp64 the same way
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)


def test_single_hip_runtime_loaded(device):
    """The library must bind to torch's libamdhip64 (one HIP runtime per process)."""
    from pipelinedp_amd import _native
    _native.lib()
    with open("/proc/self/maps") as f:
        paths = {line.split()[-1] for line in f if "libamdhip64" in line}
    assert len(paths) == 1, paths
