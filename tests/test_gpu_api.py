"""End-to-end GPU tests through the drop-in API: DPEngine.aggregate on
ColumnarBackend (HIP kernels via the C ABI).

* pre-noise accumulators equal the reference's golden accumulators
  (tests/golden, made by running the reference's DPEngine on LocalBackend);
* noise added to exactly-known aggregates follows the calibrated Laplace /
  Gaussian distributions (KS, p > 1e-4, the reference's own gate in
  dp_computations_test.py:472-545);
* private partition selection keeps partitions at the truncated-geometric
  rate pi(n) (binomial bound per n);
* two ranks (gloo, sharing the one GPU) give the single-process result.
"""
import math
import os
import socket

import numpy as np
import pytest

import pipelinedp_amd as pdp
from pipelinedp_amd import _native as N
from pipelinedp_amd import columnar_backend as CB
from pipelinedp_amd import dp_computations as dpc
from tests import golden_util as G

pytestmark = pytest.mark.gpu


def _ext():
    return pdp.DataExtractors(privacy_id_extractor=pdp.ColumnExtractor("pid"),
                              partition_extractor=pdp.ColumnExtractor("pk"),
                              value_extractor=pdp.ColumnExtractor("v"))


def _aggregate(table, params, eps, delta, public=None, seed=None):
    backend = CB.ColumnarBackend(seed=seed)
    acc = pdp.NaiveBudgetAccountant(total_epsilon=eps, total_delta=delta)
    engine = pdp.DPEngine(acc, backend)
    sink = engine.aggregate(table, params, _ext(), public_partitions=public)
    acc.compute_budgets()
    return sink, backend


@pytest.mark.parametrize("fx", G.fixtures(), ids=G.fixture_ids())
def test_backend_accumulators_match_reference_golden(device, fx):
    case = fx["case"]
    rows = [tuple(r) for r in fx["rows"]]
    backend = CB.ColumnarBackend(device=device, seed=5)
    acc = pdp.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
    engine = pdp.DPEngine(acc, backend)
    sink = engine.aggregate(rows, G.aggregate_params(case), G.extractors(case),
                            public_partitions=case.get("public"))
    acc.compute_budgets()
    got = backend.accumulators(sink)
    want = G.expected_map(fx)
    assert set(G._key(k) for k in got) == set(want)
    for k, v in got.items():
        G.assert_acc_equal(want[G._key(k)], v, f"{fx['name']}[{k}]")


def _public_table(P, per_partition, value):
    """Partition p holds `per_partition` rows from distinct privacy ids, each
    with value `value` (no sampling fires with L0 = Linf = 1)."""
    pid = np.arange(P * per_partition, dtype=np.int64)
    pk = pid // per_partition
    v = np.full(pid.shape[0], value, dtype=np.float64)
    return pdp.ColumnTable({"pid": pid, "pk": pk, "v": v})


def _ks(samples, cdf):
    from scipy.stats import kstest
    return kstest(samples, cdf).pvalue


def test_laplace_count_and_sum_noise_distribution(device):
    from scipy.stats import laplace
    P, c, v = 6000, 5, 3.0
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM], noise_kind=pdp.NoiseKind.LAPLACE,
                                 max_partitions_contributed=1, max_contributions_per_partition=1,
                                 min_value=0.0, max_value=4.0)
    sink, _ = _aggregate(_public_table(P, c, v), params, eps=1.0, delta=0.0, public=list(range(P)), seed=11)
    out = list(sink)
    assert len(out) == P
    count = np.array([m.count for _, m in out])
    s = np.array([m.sum for _, m in out])
    b_count = dpc.laplace_diversity(0.5, 1)       # eps split between COUNT and SUM
    b_sum = dpc.laplace_diversity(0.5, 4.0)
    assert _ks(count - c, laplace(scale=b_count).cdf) > 1e-4
    assert _ks(s - c * v, laplace(scale=b_sum).cdf) > 1e-4
    assert not np.any(count == np.round(count))  # continuous noise: non-integers (dp_computations_test.py:162)


def test_gaussian_sum_noise_distribution(device):
    from scipy.stats import norm
    P, c, v = 6000, 3, 1.5
    params = pdp.AggregateParams(metrics=[pdp.Metrics.SUM], noise_kind=pdp.NoiseKind.GAUSSIAN,
                                 max_partitions_contributed=1, max_contributions_per_partition=1,
                                 min_value=-2.0, max_value=2.0)
    sink, _ = _aggregate(_public_table(P, c, v), params, eps=1.0, delta=1e-5, public=list(range(P)), seed=12)
    s = np.array([m.sum for _, m in sink])
    sigma = dpc.compute_sigma(1.0, 1e-5, 2.0)
    assert _ks(s - c * v, norm(scale=sigma).cdf) > 1e-4


def test_truncated_geometric_keep_rates(device):
    """Partitions with n = 1..7 privacy ids are kept with probability pi(n)."""
    per_n, ns = 3000, list(range(1, 8))
    pid, pk = [], []
    nxt, part = 0, 0
    for n in ns:
        for _ in range(per_n):
            pid.extend(range(nxt, nxt + n))
            pk.extend([part] * n)
            nxt += n
            part += 1
    table = pdp.ColumnTable({"pid": np.asarray(pid, np.int64), "pk": np.asarray(pk, np.int64),
                             "v": np.zeros(len(pid))})
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT], noise_kind=pdp.NoiseKind.LAPLACE,
                                 max_partitions_contributed=1, max_contributions_per_partition=1)
    sink, _ = _aggregate(table, params, eps=2.0, delta=0.01, seed=13)
    plan = CB.recognise(sink)
    keep = np.asarray(CB.AggregateRun(CB.ColumnarBackend(), plan)._selection().keep_prob)
    kept = np.zeros(part, dtype=bool)
    for k, _ in sink:
        kept[int(k)] = True
    for i, n in enumerate(ns):
        p = float(keep[min(n, len(keep) - 1)])
        k = int(kept[i * per_n:(i + 1) * per_n].sum())
        sd = math.sqrt(per_n * p * (1 - p))
        assert abs(k - per_n * p) <= 5 * sd + 1, (n, k, per_n * p)


def test_mean_metrics_consistent(device):
    """MEAN output: mean = middle + noisy_nsum / max(1, noisy_count) and
    sum = mean * noisy_count (MeanMechanism, dp_computations.py:562-568), with
    enormous epsilon so the noise is negligible."""
    rng = np.random.default_rng(4)
    n, U, P = 50_000, 2_000, 40
    pid = rng.integers(0, U, n)
    pk = rng.integers(0, P, n)
    v = rng.uniform(0, 10, n)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.MEAN, pdp.Metrics.COUNT, pdp.Metrics.SUM],
                                 noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=P,
                                 max_contributions_per_partition=64, min_value=0.0, max_value=10.0)
    table = pdp.ColumnTable({"pid": pid, "pk": pk, "v": v})
    sink, _ = _aggregate(table, params, eps=1e9, delta=1e-6, public=list(range(P)), seed=14)
    out = dict(sink)
    for p in range(P):
        m = out[p]
        sel = pk == p
        assert m.count == pytest.approx(sel.sum(), abs=1e-3)
        assert m.mean == pytest.approx(v[sel].mean(), rel=1e-6)
        assert m.sum == pytest.approx(v[sel].sum(), rel=1e-6)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_data():
    rng = np.random.default_rng(21)
    n, U, P = 40_000, 3_000, 500
    pid = rng.integers(0, U, n)
    pk = rng.integers(0, P, n)
    v = rng.normal(4, 2, n)
    owner = pid % 2  # privacy ids never span ranks
    order = np.argsort(owner, kind="stable")  # rank 0's rows first, then rank 1's
    return pid[order], pk[order], v[order], owner[order], P


def _params_2rank():
    return pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
                               noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=3,
                               max_contributions_per_partition=2, min_value=0.0, max_value=8.0)


def _two_rank_worker(rank, port, results):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        pid, pk, v, owner, P = _rank_data()
        mine = owner == rank
        table = pdp.ColumnTable({"pid": pid[mine], "pk": pk[mine], "v": v[mine]},
                                n_privacy_ids=int(pid.max()) + 1, n_partitions=P)
        sink, _ = _aggregate(table, _params_2rank(), eps=1.0, delta=1e-6, seed=99)
        results[rank] = [(int(k), tuple(m)) for k, m in sink]
    except Exception as e:
        results[rank] = repr(e)
    finally:
        dist.destroy_process_group()


def test_two_ranks_match_single_process(device):
    """Rows sharded by privacy id over two ranks (gloo exchange, both on this
    GPU): the union of the ranks' partitions equals the single-process result
    (same samples, same selection, same noise streams; fp sums within 1e-9)."""
    import torch.multiprocessing as mp
    pid, pk, v, owner, P = _rank_data()
    table = pdp.ColumnTable({"pid": pid, "pk": pk, "v": v}, n_privacy_ids=int(pid.max()) + 1, n_partitions=P)
    sink, _ = _aggregate(table, _params_2rank(), eps=1.0, delta=1e-6, seed=99)
    single = {int(k): tuple(m) for k, m in sink}
    ctx = mp.get_context("spawn")
    manager = ctx.Manager()
    results = manager.dict()
    mp.spawn(_two_rank_worker, args=(_free_port(), results), nprocs=2, join=True)
    res = dict(results)
    assert all(isinstance(res[r], list) for r in (0, 1)), res
    merged = {}
    for r in (0, 1):
        for k, m in res[r]:
            assert k not in merged
            merged[k] = m
    assert set(merged) == set(single)
    for k in single:
        np.testing.assert_allclose(merged[k], single[k], rtol=1e-9, atol=1e-6)


def _row_sharded_worker(rank, port, mode, results):
    """Rows split by ROW index over two ranks (privacy ids span ranks)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        pid, pk, v, _, P = _rank_data()
        half = len(pid) // 2
        sl = slice(0, half) if rank == 0 else slice(half, None)
        table = pdp.ColumnTable({"pid": pid[sl], "pk": pk[sl], "v": v[sl]}, n_privacy_ids=int(pid.max()) + 1,
                                n_partitions=P)
        params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.PRIVACY_ID_COUNT],
                                     noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=64,
                                     max_contributions_per_partition=64)
        backend = CB.ColumnarBackend(seed=7, privacy_id_sharding=mode)
        acc = pdp.NaiveBudgetAccountant(total_epsilon=1e6, total_delta=1e-6)
        sink = pdp.DPEngine(acc, backend).aggregate(table, params, _ext(), public_partitions=list(range(P)))
        acc.compute_budgets()
        results[rank] = [(int(k), m.count, m.privacy_id_count) for k, m in sink]
    except ValueError as e:
        results[rank] = "ValueError: " + str(e)
    except Exception as e:
        results[rank] = repr(e)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["verify", "shuffle"])
def test_two_ranks_privacy_ids_spanning_ranks(device, mode):
    """Rows sharded by row, not by privacy id: "verify" (the default) raises on
    every rank; "shuffle" exchanges the rows to the privacy ids' owner ranks,
    after which the result (no sampling fires: L0 = Linf = 64, eps = 1e6) is
    the exact group-by of all rows."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.spawn(_row_sharded_worker, args=(_free_port(), mode, results), nprocs=2, join=True)
    res = dict(results)
    if mode == "verify":
        assert all(isinstance(res[r], str) and "more than one rank" in res[r] for r in (0, 1)), res
        return
    assert all(isinstance(res[r], list) for r in (0, 1)), res
    pid, pk, v, _, P = _rank_data()
    cnt = np.bincount(pk, minlength=P)
    pids = np.bincount(np.unique(pid * P + pk) % P, minlength=P)
    merged = {}
    for r in (0, 1):
        for k, c, u in res[r]:
            assert k not in merged
            merged[k] = (c, u)
    assert set(merged) == set(range(P))
    for k, (c, u) in merged.items():
        assert abs(c - cnt[k]) < 0.5 and abs(u - pids[k]) < 0.5, (k, c, cnt[k], u, pids[k])  # b = 0.008


def test_select_partitions_matches_reference_golden(device):
    """DPEngine.select_partitions on ColumnarBackend returns the reference's
    kept keys (tests/golden/select_partitions.json, eps = 1e4)."""
    import json
    with open(os.path.join(G.GOLDEN, "select_partitions.json")) as f:
        fx = json.load(f)
    acc = pdp.NaiveBudgetAccountant(total_epsilon=fx["eps"], total_delta=fx["delta"])
    engine = pdp.DPEngine(acc, CB.ColumnarBackend(device=device, seed=11))
    ext = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1])
    sink = engine.select_partitions([tuple(r) for r in fx["rows"]],
                                    pdp.SelectPartitionsParams(max_partitions_contributed=3), ext)
    acc.compute_budgets()
    assert sorted(sink) == fx["expected_keys"]


@pytest.mark.parametrize("strategy", [pdp.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC,
                                      pdp.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING])
def test_select_partitions_matches_oracle_with_sampling(device, strategy):
    """200k rows where L0 sampling fires: the kept keys equal the oracle's
    (same pair priorities, same Philox selection stream)."""
    from oracle import columnar as O
    rng = np.random.default_rng(4)
    n, U, P = 200_000, 5_000, 3_000
    pid = rng.integers(0, U, n)
    pk = np.minimum(rng.zipf(1.2, n) - 1, P - 1)
    table = pdp.ColumnTable({"pid": pid, "pk": pk}, n_privacy_ids=U, n_partitions=P)
    backend = CB.ColumnarBackend(device=device, seed=21)
    acc = pdp.NaiveBudgetAccountant(total_epsilon=2.0, total_delta=1e-5)
    engine = pdp.DPEngine(acc, backend)
    ext = pdp.DataExtractors(privacy_id_extractor=pdp.ColumnExtractor("pid"),
                             partition_extractor=pdp.ColumnExtractor("pk"))
    sink = engine.select_partitions(table, pdp.SelectPartitionsParams(
        max_partitions_contributed=3, partition_selection_strategy=strategy), ext)
    acc.compute_budgets()
    got = sorted(sink)
    run = CB.AggregateRun(backend, CB.recognise(sink))
    seed_bound, seed_select, _ = run._seeds
    sel = run._selection()
    spec = run._bounding_spec(N.VALUE_NONE)
    oacc = O.bound_and_reduce(pid, pk, None, n_privacy_ids=U, n_partitions=P, l0=3, linf=0,
                              value_kind=O.VALUE_NONE, flags=0, seed=seed_bound,
                              rand_shift=__import__("pipelinedp_amd.executor", fromlist=["x"]).bound_plan(
                                  n, U, P, spec).rand_shift)
    keep, _ = O.select(oacc["privacy_id_count"], sel.strategy, keep_prob=sel.keep_prob,
                       noise=None if sel.noise is None else sel.noise.as_dict(), threshold=sel.threshold,
                       seed=seed_select)
    assert got == np.flatnonzero(keep).tolist()
    assert 0 < len(got) < P


def _add_noise(pairs_or_table, kind, eps, delta, l0, linf, seed):
    backend = CB.ColumnarBackend(seed=seed)
    acc = pdp.NaiveBudgetAccountant(total_epsilon=eps, total_delta=delta)
    engine = pdp.DPEngine(acc, backend)
    nk = pdp.NoiseKind.LAPLACE if kind == "laplace" else pdp.NoiseKind.GAUSSIAN
    sink = engine.add_dp_noise(pairs_or_table, pdp.AddDPNoiseParams(noise_kind=nk, l0_sensitivity=l0,
                                                                     linf_sensitivity=linf))
    acc.compute_budgets()
    return sink, backend


@pytest.mark.parametrize("kind", ["laplace", "gaussian"])
def test_add_dp_noise_matches_oracle_and_distribution(device, kind):
    """add_dp_noise (dp_engine.py:551-607) through the HIP kernel: keys kept
    in order, values = oracle (same Philox stream, fp64 within 1e-12), noise
    KS-distributed as the calibrated mechanism (p > 1e-4)."""
    from scipy.stats import laplace, norm
    from oracle import columnar as O
    n = 30001  # odd: exercises the tail element
    rng = np.random.default_rng(5)
    vals = rng.integers(-50, 50, n).astype(np.float64)
    keys = [f"k{i}" for i in range(n)]
    sink, backend = _add_noise(list(zip(keys, vals.tolist())), kind, 1.0, 1e-6, 2, 3.0, seed=21)
    out = list(sink)
    assert [k for k, _ in out] == keys
    got = np.array([v for _, v in out])
    noise = CB.noise_mechanism_of(CB.recognise(sink).noise_fn)
    scale = noise.scale
    _, _, seed_noise = backend._seeds()
    want = O.add_noise(vals, noise.as_dict(), seed_noise)
    np.testing.assert_array_equal(got, want)  # grid-valued draws: bit-exact
    # every output lies on the mechanism's power-of-two grid
    g = noise.granularity
    assert g > 0 and math.log2(g).is_integer()
    assert np.all(np.fmod(got, g) == 0.0)
    dist = laplace(scale=6.0 / 1.0) if kind == "laplace" else norm(scale=dpc.compute_sigma(1.0, 1e-6, math.sqrt(2) * 3.0))
    assert math.isclose(scale, dist.std() / (math.sqrt(2) if kind == "laplace" else 1.0), rel_tol=1e-12)
    assert _ks(got - vals, dist.cdf) > 1e-4


def test_add_dp_noise_device_columns(device):
    """A (keys, values) ColumnTable of device tensors is noised in place on
    the GPU; int64 values are converted as float(value)."""
    import torch
    from oracle import columnar as O
    n = 4096
    keys = torch.arange(n, device=device)
    vals = torch.arange(n, device=device, dtype=torch.int64) * 3
    sink, backend = _add_noise(pdp.ColumnTable({"pk": keys, "v": vals}), "laplace", 0.5, 0.0, 1, 1.0, seed=22)
    out = list(sink)
    assert [k for k, _ in out] == list(range(n))
    _, _, seed_noise = backend._seeds()
    want = O.add_noise(np.arange(n) * 3, dpc.laplace_noise_params(0.5, 1.0).as_dict(), seed_noise)
    np.testing.assert_array_equal(np.array([v for _, v in out]), want)


def test_add_noise_kernel_sharded_offsets_equal_whole(device):
    """Shards noised with their global offsets equal the unsharded column."""
    import torch
    from pipelinedp_amd import executor as X
    x = torch.randn(10001, dtype=torch.float64, device=device)
    nz = dpc.gaussian_noise_params(2.5)
    whole = X.add_noise(x, noise=nz, seed=77)
    a = X.add_noise(x[:4000].clone(), noise=nz, seed=77)
    b = X.add_noise(x[4000:].clone(), noise=nz, seed=77, index_offset=4000)
    assert torch.equal(torch.cat([a, b]), whole)


@pytest.mark.parametrize("name", ["string_keys", "count_sum_int_movie", "count_sum_mean_f64"])
def test_parquet_ingest_matches_reference_golden(device, tmp_path, name):
    """Columnar ingest: the golden rows written to
    Parquet and read back as dictionary / numeric Arrow columns give the
    reference's golden accumulators through the same GPU path."""
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    fx = [f for f in G.fixtures() if f["name"] == name][0]
    case = fx["case"]
    rows = [tuple(r) for r in fx["rows"]]
    path = tmp_path / "rows.parquet"
    pq.write_table(pa.table({"pid": [r[0] for r in rows], "pk": [r[1] for r in rows],
                             "v": [r[2] for r in rows]}), path)
    table = pdp.ColumnTable.from_parquet(path, key_columns=["pid", "pk"])
    backend = CB.ColumnarBackend(device=device, seed=5)
    acc = pdp.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
    engine = pdp.DPEngine(acc, backend)
    sink = engine.aggregate(table, G.aggregate_params(case), _ext(), public_partitions=case.get("public"))
    acc.compute_budgets()
    got = backend.accumulators(sink)
    want = G.expected_map(fx)
    assert set(G._key(k) for k in got) == set(want)
    for k, v in got.items():
        G.assert_acc_equal(want[G._key(k)], v, f"{name}[{k}]")


def test_out_of_range_keys_raise_when_the_result_is_read(device):
    """The key-range check of the API path is deferred (the error word is
    copied to pinned memory behind the bounding launches):
    an out-of-range partition code still raises ValueError, at the first read
    of the result, and the same backend then aggregates a valid table."""
    import torch
    rng = np.random.default_rng(3)
    n, U, P = 100_000, 5_000, 100
    pid = torch.as_tensor(rng.integers(0, U, n)).to(device)
    pk = torch.as_tensor(rng.integers(0, P, n)).to(device)
    v = torch.as_tensor(rng.random(n)).to(device)
    bad = pk.clone()
    bad[777] = P + 5
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM], noise_kind=pdp.NoiseKind.LAPLACE,
                                 max_partitions_contributed=2, max_contributions_per_partition=1,
                                 min_value=0.0, max_value=1.0)
    backend = CB.ColumnarBackend(device=device, seed=3)
    for col, raises in ((bad, True), (pk, False), (bad, True)):
        acc = pdp.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
        table = pdp.ColumnTable({"pid": pid, "pk": col, "v": v}, n_privacy_ids=U, n_partitions=P)
        sink = pdp.DPEngine(acc, backend).aggregate(table, params, _ext())
        acc.compute_budgets()
        if raises:
            with pytest.raises(ValueError, match="outside the dense key range"):
                list(sink)
        else:
            assert len(list(sink)) > 0
