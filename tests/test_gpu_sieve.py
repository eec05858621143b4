"""GPU parity of the threshold sieve (pdp_bound.hip, Plan.sieve) against the oracle.

The sieve changes data movement only: k_sieve_l1 keeps the rows whose pair
hash is below t = sieve / 2^16, the bucket kernel marks privacy ids with
fewer than l0 candidate pairs, and the fix-up (k_sieve_rescan ->
k_fix_scatter -> k_bucket_fix) recomputes those ids from all of their rows.
Kept pairs and rows must therefore equal the oracle's exactly (the oracle has
no sieve: oracle/columnar.py bound_and_reduce follows
contribution_bounders.py:72-111 with the kernels' priorities), at every t:
t ~ 0 (nearly every id unresolved: the fix-up does all the work, the Bloom
filter saturates), intermediate t, and t = 1/2.  Integer outputs bit-exact;
fp64 sums within 1e-9 of the sum of |terms| (FLOAT_RTOL).
"""
import numpy as np
import pytest

from oracle import columnar as O
from tests.test_gpu_kernels import _abs_scale, _compare, _gen, _rand_shift

pytestmark = pytest.mark.gpu

SIEVES = [1, 64, 4096, 16384, 32768]  # t = sieve / 2^16

# (l0, linf, value_kind, flags, lo, hi, per-partition bounds, U): U large
# enough for two partition levels (the sieve's precondition)
CASES = [
    (2, 1, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM, 0.0, 10.0, None, 200_000),
    (4, 2, O.VALUE_I64, O.ACC_SUM | O.SUM_INT, 0, 7, None, 90_000),
    (16, 4, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM | O.ACC_NSUM2, 1.0, 6.0, None, 20_000),
    (3, 0, O.VALUE_F64, O.SUM_PER_PARTITION, 0, 0, (-3.0, 20.0), 120_000),
    (1, 1, O.VALUE_NONE, 0, 0, 0, None, 300_000),
]


def _spec(case):
    from pipelinedp_amd import executor as X
    l0, linf, vk, flags, lo, hi, pp, _ = case
    mid = lo + (hi - lo) / 2 if vk != O.VALUE_NONE else 0.0
    return X.BoundingSpec(l0=l0, linf=linf, value_kind=vk, flags=flags, min_value=lo, max_value=hi,
                          middle=mid, min_sum=pp[0] if pp else 0.0, max_sum=pp[1] if pp else 0.0)


def _run(device, pid, pk, val, U, P, spec, seed, sieve, allowed=None, key_format=0, row_offset=0, band=0,
         workspace=None, threads=0, bucket_threads=0):
    import torch
    from pipelinedp_amd import executor as X
    tv = None if val is None else torch.as_tensor(val).to(device)
    ta = None if allowed is None else torch.as_tensor(allowed.astype(np.uint8)).to(device)
    acc = X.bound_and_reduce(torch.as_tensor(pid).to(device), torch.as_tensor(pk).to(device), tv,
                             n_privacy_ids=U, n_partitions=P, bounding=spec, seed=seed, allowed=ta,
                             key_format=key_format, sieve=sieve, row_offset=row_offset, sieve_band=band,
                             workspace=workspace, sieve_threads=threads, bucket_threads=bucket_threads)
    torch.cuda.synchronize()
    return {k: (None if v is None else v.cpu().numpy()) for k, v in acc.items()}


def _want(pid, pk, val, U, P, spec, seed, allowed=None, row_offset=0, bucket_threads=0):
    return O.bound_and_reduce(pid, pk, val, n_privacy_ids=U, n_partitions=P, l0=spec.l0, linf=spec.linf,
                              value_kind=spec.value_kind, flags=spec.flags, min_value=spec.min_value,
                              max_value=spec.max_value, middle=spec.middle, min_sum=spec.min_sum,
                              max_sum=spec.max_sum, seed=seed, allowed=allowed, row_offset=row_offset,
                              rand_shift=_rand_shift(len(pid), U, P, spec, bucket_threads=bucket_threads))


@pytest.mark.parametrize("case", CASES, ids=[f"l0={c[0]}-linf={c[1]}-f={c[3]}" for c in CASES])
def test_sieve_matches_oracle_at_every_threshold(device, case):
    from pipelinedp_amd import executor as X
    spec = _spec(case)
    U, P = case[7], 3001
    n = 2_000_000 + 12_345  # a ragged last tile
    pid, pk, val = _gen(77 + spec.l0, n, U, P, spec.value_kind, skew=True)
    seed = 0xA5A5_0000_1111 + spec.l0
    want = _want(pid, pk, val, U, P, spec, seed)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    for sieve in SIEVES:
        plan = X.bound_plan(n, U, P, spec, sieve=sieve)
        assert plan.sieve == sieve, (sieve, plan.sieve)
        assert plan.band == (min(2 * sieve, 32768) if sieve < 32768 else 0)
        for band in (0, -1):  # the side band (ids with < l0 pairs below 2t: the rescan), and without it
            # both level-1 workgroup shapes (512 threads, 16 flush slots per
            # tile; 1,024 threads, 8 slots)
            for threads in (512, 1024):
                got = _run(device, pid, pk, val, U, P, spec, seed, sieve, band=band, threads=threads)
                _compare(got, want, scale)
    off = _run(device, pid, pk, val, U, P, spec, seed, -1)
    assert X.bound_plan(n, U, P, spec, sieve=-1).sieve == 0
    _compare(off, want, scale)


@pytest.mark.parametrize("key_format", [2, 3])  # COMPACT, PACKED
def test_sieve_key_formats_public_filter_and_offset(device, key_format):
    """Dead (non-public) rows are dropped by the sieve and marked dead in the
    fix-up; row priorities follow row_offset in both."""
    spec = _spec(CASES[0])
    U, P, n = 200_000, 1000, 1_500_000
    pid, pk, val = _gen(5, n, U, P, spec.value_kind, skew=True)
    allowed = np.random.default_rng(3).random(P) < 0.7
    seed, off = 991, 123_456_789
    want = _want(pid, pk, val, U, P, spec, seed, allowed=allowed, row_offset=off)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    for sieve in (64, 8192):
        got = _run(device, pid, pk, val, U, P, spec, seed, sieve, allowed=allowed, key_format=key_format,
                   row_offset=off)
        _compare(got, want, scale)
        assert (got["privacy_id_count"][~allowed] == 0).all()


@pytest.mark.parametrize("key_format", [4, 5], ids=["packed-wide", "packed64"])
def test_sieve_packed_wide(device, key_format):
    """P = 1e7 (bucket + partition bits > 31): PACKED_WIDE records, 8-byte
    fix-up keys, rand_shift > 32 (the threshold is a multiple of the masked
    hash grain)."""
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import executor as X
    spec = _spec((4, 2, O.VALUE_F64, O.ACC_NSUM, 0.0, 20.0, None, 0))
    U, P, n = 400_000, 10_000_000, 2_000_000
    rng = np.random.default_rng(8)
    pid = rng.integers(0, U, n)
    pk = np.minimum(rng.zipf(1.1, n) - 1, P - 1).astype(np.int64)
    val = np.clip(rng.lognormal(1.0, 1.0, n), 0, 20)
    plan = X.bound_plan(n, U, P, spec, sieve=4096, key_format=key_format)
    assert plan.key_format == key_format and plan.rand_shift > 32 and plan.sieve == 4096
    seed = 4242
    want = _want(pid, pk, val, U, P, spec, seed)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    for sieve in (64, 4096, 32768):
        _compare(_run(device, pid, pk, val, U, P, spec, seed, sieve, key_format=key_format), want, scale)


def test_sieve_c3_shape_slice(device):
    """A C3-shaped slice (uniform ids, ~100 rows each, Zipf(1.1) keys folded
    into 1e6, L0 = 2, Linf = 1, COUNT+SUM+MEAN) with the AUTO threshold."""
    from pipelinedp_amd import executor as X
    spec = _spec((2, 1, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM, 0.0, 10.0, None, 0))
    U, P = 150_000, 1_000_000
    n = 100 * U
    rng = np.random.default_rng(2)
    pid = rng.integers(0, U, n)
    pk = np.minimum(rng.zipf(1.1, n) - 1, P - 1).astype(np.int64)
    val = rng.random(n) * 10.0
    plan = X.bound_plan(n, U, P, spec)
    assert 0 < plan.sieve < 16384 and plan.band == 2 * plan.sieve  # auto: t ~ 0.15, band to 2t
    seed = 77
    want = _want(pid, pk, val, U, P, spec, seed)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    ws = X.BoundWorkspace()
    _compare(_run(device, pid, pk, val, U, P, spec, seed, 0, workspace=ws), want, scale)
    st = ws.stats()
    # ~t of the rows went on as candidates and ~t more to the band; ids
    # short of l0 candidate pairs are finished from the band (at C3's ~100
    # rows per id none is short of l0 pairs below 2t: no rescan)
    assert 0.1 * n < st["rows_partitioned"] < 0.2 * n and 0.1 * n < st["band_rows"] < 0.2 * n, st
    assert st["unresolved_ids"] > 0 and st["unresolved2_ids"] == 0 and st["fixup2_rows"] == 0, st
    _compare(_run(device, pid, pk, val, U, P, spec, seed, 0, band=-1), want, scale)


def test_band_with_ids_short_of_pairs(device):
    """Ids with one to three rows next to ~100-row ids: the short ones stay
    unresolved after the band (fewer than l0 distinct pairs below 2t, or at
    all), so the band's fix-up launch marks them and the privacy-id column is
    re-read for them (the third bucket launch); equal to the oracle."""
    from pipelinedp_amd import executor as X
    spec = _spec((3, 2, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM, 0.0, 10.0, None, 0))
    U, P = 120_000, 50_000
    rng = np.random.default_rng(31)
    big = rng.integers(0, 100_000, 100 * 100_000)
    small = np.repeat(np.arange(100_000, U), rng.integers(1, 4, U - 100_000))
    pid = rng.permutation(np.concatenate([big, small]))
    n = len(pid)
    pk = rng.integers(0, P, n)
    val = rng.random(n) * 10.0
    plan = X.bound_plan(n, U, P, spec, sieve=6000)
    assert plan.sieve == 6000 and plan.band == 12000
    seed = 5150
    want = _want(pid, pk, val, U, P, spec, seed)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    ws = X.BoundWorkspace()
    _compare(_run(device, pid, pk, val, U, P, spec, seed, 6000, workspace=ws), want, scale)
    st = ws.stats()
    assert st["unresolved2_ids"] > 10_000 and st["fixup2_rows"] >= st["unresolved2_ids"], st


@pytest.mark.parametrize("threads", [512, 1024])
def test_sieve_every_row_a_candidate(device, threads):
    """Tiles whose every row is a candidate (each row's pair hash below t =
    1/2): the stage flushes at every chance, so a tile fills all of its
    flush slots (16 for 512 threads, 8 for 1,024); equal to the oracle."""
    from pipelinedp_amd import executor as X
    spec = _spec((2, 1, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM, 0.0, 10.0, None, 0))
    U, P = 300_000, 4096  # > 64 buckets: two partition levels, the sieve's precondition
    seed = 8080
    rng = np.random.default_rng(12)
    cu = rng.integers(0, U, 400_000)
    ck = rng.integers(0, P, 400_000)
    low = O.pair_hash(seed, cu, ck) < np.uint32(1 << 31)
    cu, ck = cu[low], ck[low]
    idx = rng.integers(0, len(cu), 3 * 65536 + 999)
    pid, pk = cu[idx], ck[idx]
    n = len(pid)
    val = rng.random(n) * 10.0
    plan = X.bound_plan(n, U, P, spec, sieve=32768, sieve_threads=threads)
    assert plan.sieve == 32768 and plan.sieve_threads == threads
    want = _want(pid, pk, val, U, P, spec, seed)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    ws = X.BoundWorkspace()
    _compare(_run(device, pid, pk, val, U, P, spec, seed, 32768, workspace=ws, threads=threads), want, scale)
    assert ws.stats()["rows_partitioned"] == n


@pytest.mark.parametrize("key_format", [0, 5], ids=["auto", "packed64"])
@pytest.mark.parametrize("sieve", [-1, 4096])
def test_malformed_records_are_flagged_not_read(device, sieve, key_format, monkeypatch):
    """PDP_DEBUG_CORRUPT_RECORDS overwrites bucket 0's level-2 records with
    the all-ones partition (>= P) and bucket 1's with an out-of-range row: the
    bucket kernel sets the error word (bound_and_reduce raises) instead of
    dereferencing them (the r02 illegal-address fault)."""
    import torch
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import executor as X
    base = _spec(CASES[0])
    spec = X.BoundingSpec(l0=base.l0, linf=base.linf, value_kind=base.value_kind,
                          flags=base.flags | N.DEBUG_CORRUPT_RECORDS, min_value=base.min_value,
                          max_value=base.max_value, middle=base.middle)
    U, P, n = 200_000, 3001, 1_000_000
    pid, pk, val = _gen(1, n, U, P, spec.value_kind)
    monkeypatch.delenv("PIPELINEDP_AMD_TEST_HOOKS", raising=False)
    with pytest.raises(RuntimeError, match="test hook"):  # rejected outside test mode
        _run(device, pid, pk, val, U, P, spec, 5, sieve, key_format=key_format)
    monkeypatch.setenv("PIPELINEDP_AMD_TEST_HOOKS", "1")
    with pytest.raises(ValueError, match="outside the dense key range"):
        _run(device, pid, pk, val, U, P, spec, 5, sieve, key_format=key_format)
    torch.cuda.synchronize()  # the device is still healthy
    ok = _run(device, pid, pk, val, U, P, base, 5, sieve, key_format=key_format)
    assert ok["privacy_id_count"].sum() > 0


@pytest.mark.parametrize("sieve", [6000, 10096])
def test_sieve_with_half_size_buckets(device, sieve):
    """bucket_threads = 512 under the sieve and its band: the candidate
    records, the fix-up launches and the range merge over twice the buckets."""
    from pipelinedp_amd import executor as X
    spec = _spec(CASES[0])
    U, P, n = 400_000, 100_003, 4_000_000
    pid, pk, val = _gen(5, n, U, P, spec.value_kind, skew=True)
    plan = X.bound_plan(n, U, P, spec, sieve=sieve, bucket_threads=512)
    assert plan.sieve == sieve and plan.bucket_threads == 512
    got = _run(device, pid, pk, val, U, P, spec, 19, sieve, bucket_threads=512)
    want = _want(pid, pk, val, U, P, spec, 19, bucket_threads=512)
    _compare(got, want, _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle))


@pytest.mark.parametrize("threads", [512, 1024])
def test_persistent_level1_loops_over_tiles(device, threads, monkeypatch):
    """The persistent level 1 with few workgroups (test hook
    PIPELINEDP_AMD_L1_GRID): each workgroup runs several whole tiles, so the
    next tile's chunks are prefetched across the tile boundary and the LDS
    state (bucket counts, band queues, flush slots) is reset between tiles;
    with the band on and off, equal to the oracle."""
    from pipelinedp_amd import executor as X
    spec = _spec(CASES[0])
    U, P = 200_000, 3001
    n = 40 * 65536 + 777  # 40 whole tiles and a ragged one
    pid, pk, val = _gen(41, n, U, P, spec.value_kind, skew=True)
    seed = 6060
    want = _want(pid, pk, val, U, P, spec, seed)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    monkeypatch.setenv("PIPELINEDP_AMD_TEST_HOOKS", "1")
    for grid in ("3", "7"):  # 13-14 and 5-6 tiles per workgroup
        monkeypatch.setenv("PIPELINEDP_AMD_L1_GRID", grid)
        for band in (0, -1):
            got = _run(device, pid, pk, val, U, P, spec, seed, 4096, band=band, threads=threads)
            _compare(got, want, scale)


def test_plan_feedback_runs_light_user_tables_unsieved(device):
    """Light users: half the privacy ids hold 1-3 rows, so the
    sieve leaves more than RESCAN_BLOOM_MAX ids for the whole-column re-read.
    The first auto call runs sieved and leaves its fix-up counters behind
    (pdp_bound_stats_async); the next call on the same columns runs the
    unsieved plan.  Both equal the oracle; another table keeps the sieve."""
    import torch
    from pipelinedp_amd import executor as X
    spec = _spec((2, 1, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM, 0.0, 10.0, None, 0))
    rng = np.random.default_rng(77)
    heavy, light = 80_000, 80_000  # > 64 buckets of 2,048 ids: two partition levels, the sieve's precondition
    U, P = heavy + light, 50_000
    big = rng.integers(0, heavy, 100 * heavy)
    small = np.repeat(np.arange(heavy, U), rng.integers(1, 4, light))
    pid = rng.permutation(np.concatenate([big, small]))
    n = len(pid)
    pk = rng.integers(0, P, n)
    val = rng.random(n) * 10.0
    assert X.bound_plan(n, U, P, spec).sieve > 0  # the auto plan sieves this shape
    seed = 4321
    want = _want(pid, pk, val, U, P, spec, seed)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    tp, tk, tv = (torch.as_tensor(a).to(device) for a in (pid, pk, val))
    ws = X.BoundWorkspace()

    def call():
        acc = X.bound_and_reduce(tp, tk, tv, n_privacy_ids=U, n_partitions=P, bounding=spec, seed=seed,
                                 workspace=ws)
        torch.cuda.synchronize()
        return {k: (None if v is None else v.cpu().numpy()) for k, v in acc.items()}

    _compare(call(), want, scale)
    st1 = ws.stats()
    assert st1["sieve"] > 0 and st1["unresolved_ids"] > X.RESCAN_BLOOM_MAX, st1
    _compare(call(), want, scale)
    assert ws.stats()["sieve"] == 0  # measured slow: unsieved now
    assert X.plan_feedback_state(tp, tk, n_privacy_ids=U, n_partitions=P, bounding=spec)["unsieved"]
    # the decision belongs to these tensor objects and their contents: a copy
    # (as a new table allocated at a freed one's address would be) starts
    # fresh, and an in-place write through torch re-measures
    tp2, tk2 = tp.clone(), tk.clone()
    assert X.plan_feedback_state(tp2, tk2, n_privacy_ids=U, n_partitions=P, bounding=spec) is None
    tk.add_(0)
    assert X.plan_feedback_state(tp, tk, n_privacy_ids=U, n_partitions=P, bounding=spec) is None
    _compare(call(), want, scale)  # measured again: sieved, equal to the oracle
    assert ws.stats()["sieve"] > 0
    # a table of heavy users only keeps the sieved plan
    pid2 = rng.integers(0, U, 100 * U)
    pk2 = rng.integers(0, P, len(pid2))
    val2 = rng.random(len(pid2)) * 10.0
    t2 = [torch.as_tensor(a).to(device) for a in (pid2, pk2, val2)]
    for _ in range(2):
        X.bound_and_reduce(*t2, n_privacy_ids=U, n_partitions=P, bounding=spec, seed=seed, workspace=ws)
        torch.cuda.synchronize()
        assert ws.stats()["sieve"] > 0


@pytest.mark.parametrize("sieve,U,u16", [(-1, 300_000, 0), (32768, 300_000, 0), (-1, 40_000_000, 1),
                                         (16384, 20_000_000, 1)],
                         ids=["tile-local", "sieve", "tile-local-u16", "sieve-band-u16"])
def test_tile_with_every_row_in_one_bucket(device, sieve, U, u16):
    """Level 1 keeps a tile's bucket counts as u16 (flush_counts16); a bucket
    holding all 65,536 rows of a tile (counted 65,536, stored as 0 with the
    bucket in tile_over) must still get all of them.  Tile 0 here: every row
    from the first 2,048 privacy ids (bucket 0 at b = 11), and with the sieve
    every such row a candidate (pair hash below t); equal to the oracle.
    u16: so many buckets that level 1 counts each half tile in u16 lanes
    (counts_tm / counts_tm2, Plan.hist_u16): the bucket's two halves are
    32,768 each and their sum 65,536 carries out of its lane in the column
    scan unless the lanes are added apart (k_gscan_sums)."""
    from pipelinedp_amd import executor as X
    spec = _spec((2, 1, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM, 0.0, 10.0, None, 0))
    P = 4096
    seed = 9191
    plan = X.bound_plan(3 * 65536 + 321, U, P, spec, sieve=sieve)
    assert plan.bucket_bits == 11 and (plan.sieve > 0) == (sieve > 0) and plan.hist_u16 == u16, \
        (plan.bucket_bits, plan.sieve, plan.hist_u16)
    rng = np.random.default_rng(5)
    cu = rng.integers(0, 2048, 200_000)
    ck = rng.integers(0, P, 200_000)
    if sieve > 0:
        low = O.pair_hash(seed, cu, ck) < np.uint32(sieve << 16)
        cu, ck = cu[low], ck[low]
    idx = rng.integers(0, len(cu), 65536)
    pid = np.concatenate([cu[idx], rng.integers(0, U, 2 * 65536 + 321)])
    pk = np.concatenate([ck[idx], rng.integers(0, P, 2 * 65536 + 321)])
    n = len(pid)
    val = rng.random(n) * 10.0
    want = _want(pid, pk, val, U, P, spec, seed)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    _compare(_run(device, pid, pk, val, U, P, spec, seed, sieve), want, scale)


def test_fixup_list_capacity_guard_raises(device, monkeypatch):
    """The fix-up row list's writes are guarded by its capacity and an
    overflow sets bit 1 of the error word, which bound_and_reduce raises
    (the guard was untested).  The region cannot overflow
    for real (each list holds distinct rows), so the test hook
    PIPELINEDP_AMD_FIX_CAP shrinks it to 64 entries under a table whose
    fix-up lists thousands of rows; afterwards the device is healthy and the
    full region gives the oracle's result."""
    from pipelinedp_amd import _native as N
    spec = _spec((3, 2, O.VALUE_F64, O.ACC_SUM | O.ACC_NSUM, 0.0, 10.0, None, 0))
    U, P = 120_000, 50_000
    rng = np.random.default_rng(31)
    big = rng.integers(0, 100_000, 100 * 100_000)
    small = np.repeat(np.arange(100_000, U), rng.integers(1, 4, U - 100_000))
    pid = rng.permutation(np.concatenate([big, small]))
    n = len(pid)
    pk = rng.integers(0, P, n)
    val = rng.random(n) * 10.0
    seed = 5150
    monkeypatch.setenv("PIPELINEDP_AMD_TEST_HOOKS", "1")
    monkeypatch.setenv("PIPELINEDP_AMD_FIX_CAP", "64")
    for band in (0, -1):  # the band's lists and the whole-column re-read both fill the list
        with pytest.raises(N.NativeLibraryError, match="outgrew its workspace region"):
            _run(device, pid, pk, val, U, P, spec, seed, 6000, band=band)
    monkeypatch.delenv("PIPELINEDP_AMD_FIX_CAP")
    want = _want(pid, pk, val, U, P, spec, seed)
    _compare(_run(device, pid, pk, val, U, P, spec, seed, 6000), want,
             _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle))


def test_workspace_placement_probe_keeps_results(device, monkeypatch):
    """A workspace placed by measurement (executor._place: level-1 passes
    with PDP_PROBE_LEVEL1 into candidate workspaces, the fastest kept; here
    forced at test size) gives the oracle's result, and the probe passes
    leave nothing behind that the real call reads."""
    import torch
    from pipelinedp_amd import executor as X
    spec = _spec(CASES[0])
    U, P, n = 200_000, 3001, 1_500_000
    pid, pk, val = _gen(61, n, U, P, spec.value_kind, skew=True)
    seed = 808
    want = _want(pid, pk, val, U, P, spec, seed)
    scale = _abs_scale(pid, pk, val, P, spec.min_value, spec.max_value, spec.middle)
    monkeypatch.setattr(X, "PLACEMENT_PROBE_MIN", 0)
    monkeypatch.setattr(X, "PLACEMENT_PROBE", 3)
    before = len(X._placement_log)
    ws = X.BoundWorkspace()
    for sieve in (4096, -1):  # sieved (level 1 = k_sieve_l1) and tile-local (k_scatter_l1_local)
        ws.buf = None  # a new workspace: placed again
        _compare(_run(device, pid, pk, val, U, P, spec, seed, sieve, workspace=ws), want, scale)
    log = X._placement_log[before:]
    assert len(log) == 2 and all(len(e["candidates_ms"]) == 3 for e in log), log
    torch.cuda.synchronize()
