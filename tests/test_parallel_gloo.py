"""Multi-rank path on the CPU (gloo, world_size 2): rows sharded by privacy id,
each rank bounds and reduces its own shard, one accumulator exchange.  The
per-rank bounding is the CPU oracle here (the kernels' restatement), so this
checks the sharding design: the exchanged slices equal the unsharded
aggregation of the concatenated shards bit-exactly for counts."""
import os
import socket

import numpy as np
import pytest

from oracle import columnar as O
from pipelinedp_amd import parallel

U, P, N_PER_RANK, WORLD = 400, 37, 6000, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(rank):
    """Rank r's rows: the privacy ids shard_by_privacy_id assigns to it."""
    rng = np.random.default_rng(100 + rank)
    pid = rng.integers(0, U, 4 * N_PER_RANK)
    mine = parallel.shard_by_privacy_id(pid, WORLD, rank)
    pid = pid[mine][:N_PER_RANK]
    pk = rng.integers(0, P, pid.shape[0])
    val = rng.normal(3.0, 2.0, pid.shape[0])
    return pid, pk, val


def _oracle(pid, pk, val, P_pad, row_offset):
    return O.bound_and_reduce(pid, pk, val, n_privacy_ids=U, n_partitions=P_pad, l0=3, linf=2,
                              value_kind=O.VALUE_F64, flags=O.ACC_SUM | O.ACC_NSUM, min_value=0.0,
                              max_value=6.0, middle=3.0, seed=77, row_offset=row_offset,
                              rand_shift=O.pk_bits(P_pad) + 8)


def _worker(rank, port, results):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        P_pad, slice_len = parallel.partition_slices(P, WORLD)
        shards = [_shard(r) for r in range(WORLD)]
        offsets = np.cumsum([0] + [s[0].shape[0] for s in shards])
        pid, pk, val = shards[rank]
        acc = _oracle(pid, pk, val, P_pad, int(offsets[rank]))
        tens = {k: (None if v is None else torch.as_tensor(v)) for k, v in acc.items()}
        mine, first = parallel.exchange_accumulators(tens)
        assert first == rank * slice_len
        full = _oracle(np.concatenate([s[0] for s in shards]), np.concatenate([s[1] for s in shards]),
                       np.concatenate([s[2] for s in shards]), P_pad, 0)
        sl = slice(first, first + slice_len)
        np.testing.assert_array_equal(mine["privacy_id_count"].numpy(), full["privacy_id_count"][sl])
        np.testing.assert_array_equal(mine["count"].numpy(), full["count"][sl])
        np.testing.assert_allclose(mine["sum"].numpy(), full["sum"][sl], rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(mine["normalized_sum"].numpy(), full["normalized_sum"][sl],
                                   rtol=1e-12, atol=1e-9)
        results[rank] = "ok"
    except Exception as e:  # reported to the parent
        results[rank] = repr(e)
    finally:
        dist.destroy_process_group()


def test_exchange_matches_unsharded_aggregation():
    import torch.multiprocessing as mp
    manager = mp.Manager()
    results = manager.dict()
    mp.spawn(_worker, args=(_free_port(), results), nprocs=WORLD, join=True)
    assert dict(results) == {0: "ok", 1: "ok"}


def test_partition_slices_and_validation():
    import torch
    assert parallel.partition_slices(100_000, 8) == (100_000, 12_500)
    assert parallel.partition_slices(37, 2) == (38, 19)
    assert parallel.partition_slices(5, 1) == (5, 5)
    acc = {"privacy_id_count": torch.zeros(5, dtype=torch.int64)}
    assert parallel.exchange_accumulators(acc) == (acc, 0)  # not initialised: one rank


def test_owner_of_numpy_matches_torch():
    """shard_by_privacy_id (NumPy) and the library's owner_of (torch; the
    kernel pdp_owner_mismatches) agree, negative and large ids included, so
    data sharded by the helper passes the "verify" fast path."""
    import torch
    rng = np.random.default_rng(9)
    ids = np.concatenate([rng.integers(-2**63, 2**63 - 1, 5000, dtype=np.int64), np.arange(-50, 50),
                          np.array([2**63 - 1, -2**63], dtype=np.int64)])
    for world in (2, 3, 8):
        np.testing.assert_array_equal(parallel.owner_of_np(ids, world),
                                      parallel.owner_of(torch.as_tensor(ids), world).numpy())
        m = parallel.shard_by_privacy_id(ids, world, 1)
        np.testing.assert_array_equal(m, parallel.owner_of_np(ids, world) == 1)


def test_shard_by_privacy_id_partitions_rows():
    pid = np.arange(10_000)
    masks = [parallel.shard_by_privacy_id(pid, 4, r) for r in range(4)]
    assert np.all(sum(m.astype(int) for m in masks) == 1)
    assert all(abs(m.sum() - 2500) < 300 for m in masks)
    keys = np.array(["a", "b", "c", "d"] * 10, dtype=object)
    m0 = parallel.shard_by_privacy_id(keys, 2, 0)
    m1 = parallel.shard_by_privacy_id(keys, 2, 1)
    assert np.all(m0 ^ m1)


def _dict_worker(rank, port, results):
    import torch.distributed as dist
    from pipelinedp_amd import columnar as C
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        # string partition keys, overlapping between ranks, in different orders
        keys = [["b", "a", "c", "a"], ["d", "c", "b"]][rank]
        enc = parallel.global_partition_keys(C.encode_keys(np.asarray(keys, dtype=object)))
        assert list(enc.decode) == ["b", "a", "c", "d"]
        assert [enc.key_of(c) for c in enc.codes] == keys
        # dense integer keys keep identity codes, range = max over ranks
        ids = parallel.global_partition_keys(C.encode_keys(np.arange(3 + 4 * rank)))
        assert ids.decode is None and ids.n == 7
        assert parallel.row_offset(10 + rank) == (0 if rank == 0 else 10)
        seeds = parallel.broadcast_seeds((rank + 1, rank + 2, rank + 3))
        assert seeds == (1, 2, 3)
        assert parallel.all_ranks_any(rank == 1) is True
        # int64 accumulators narrowed to int32 on the wire only when no sum
        # over ranks can reach 2^31: 2^30 on both ranks stays int64 (exact)
        import torch
        big = {"count": torch.full((4,), 2 ** 30, dtype=torch.int64),
               "privacy_id_count": torch.arange(4, dtype=torch.int64),
               "sum": torch.full((4,), -5, dtype=torch.int64), "normalized_sum": None}
        got, first = parallel.exchange_accumulators(big)
        assert got["count"].dtype == torch.int64 and got["count"].tolist() == [2 ** 31] * 2
        assert got["privacy_id_count"].tolist() == [2 * (first + i) for i in range(2)]
        assert got["sum"].tolist() == [-10, -10] and got["normalized_sum"] is None
        results[rank] = "ok"
    except Exception as e:
        results[rank] = repr(e)
    finally:
        dist.destroy_process_group()


def test_global_partition_dictionary_and_offsets():
    import torch.multiprocessing as mp
    manager = mp.Manager()
    results = manager.dict()
    mp.spawn(_dict_worker, args=(_free_port(), results), nprocs=WORLD, join=True)
    assert dict(results) == {0: "ok", 1: "ok"}


def _pid_worker(rank, port, results):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        # disjoint privacy ids: accepted
        parallel.check_privacy_ids_disjoint(torch.arange(rank, 1000, WORLD))
        # one shared id among many: rejected on every rank
        ids = torch.arange(rank * 500, rank * 500 + 500)
        ids = torch.cat([ids, torch.tensor([123_456])])
        try:
            parallel.check_privacy_ids_disjoint(ids)
            results[rank] = "overlap not detected"
            return
        except ValueError as e:
            assert "more than one rank" in str(e)
        # string ids: identities are a fixed-key hash, equal across ranks
        a = parallel.key_identities(np.asarray(["u1", "u2", f"only{rank}"], dtype=object))
        b = parallel.key_identities(np.asarray(["u2", "u1"], dtype=object))
        assert list(a[:2]) == list(b[::-1])
        assert list(parallel.key_identities(np.asarray([5, 7], dtype=object))) == [5, 7]
        # shuffle: every privacy id's rows end on its owner rank, rows preserved
        rng = np.random.default_rng(rank)
        pid = torch.as_tensor(rng.integers(0, 300, 2000))
        pk = torch.as_tensor(rng.integers(0, 50, 2000))
        val = torch.as_tensor(rng.normal(size=2000))
        got_pid, (got_pk, got_val, none) = parallel.shuffle_by_privacy_id(pid, [pk, val, None])
        assert none is None
        assert bool((parallel._owner(got_pid, WORLD) == rank).all())
        parallel.check_privacy_ids_disjoint(torch.unique(got_pid))
        rows = sorted(zip(got_pid.tolist(), got_pk.tolist(), got_val.tolist()))
        objs = [None] * WORLD
        dist.all_gather_object(objs, rows)
        every = sorted(r for part in objs for r in part)
        mine = list(zip(pid.tolist(), pk.tolist(), val.tolist()))
        allin = [None] * WORLD
        dist.all_gather_object(allin, mine)
        assert every == sorted(r for part in allin for r in part)
        # the helper aggregate() and compute_dataset_histograms() share
        # (histograms of row-sharded input were silently wrong)
        from pipelinedp_amd import columnar as C
        from pipelinedp_amd.columnar_backend import shard_rows_by_privacy_id
        enc = C.EncodedKeys(pid, 300, None)
        try:
            shard_rows_by_privacy_id("verify", pid, pk, val, enc)
            results[rank] = "row-sharded ids not detected"
            return
        except ValueError as e:
            assert "more than one rank" in str(e)
        # the verify fast path: hash-owned ids pass with one flag all-reduce,
        # disjoint ids that are not hash-owned go through the id exchange
        assert parallel.verify_privacy_id_sharding(got_pid) == "owned"
        assert shard_rows_by_privacy_id("verify", got_pid, got_pk, got_val, enc)[0] is got_pid
        assert parallel.verify_privacy_id_sharding(torch.arange(rank * 700, rank * 700 + 700)) == "exchanged"
        try:  # one rank hash-owned, the other holding an id of rank 0's: still caught
            mine_ids = got_pid if rank == 0 else torch.cat([got_pid, got_pid.new_tensor([0, 1, 2, 3, 4, 5])])
            allin0 = [None] * WORLD
            dist.all_gather_object(allin0, sorted(set(got_pid.tolist())))
            if rank == 1:
                mine_ids = torch.cat([got_pid, torch.as_tensor(allin0[0][:3])])
            parallel.verify_privacy_id_sharding(mine_ids)
            results[rank] = "overlap behind the fast path not detected"
            return
        except ValueError as e:
            assert "more than one rank" in str(e)
        sp, spk, sval, senc = shard_rows_by_privacy_id("shuffle", pid, pk, val, enc)
        assert senc.n == int(torch.unique(sp).numel()) and len(spk) == len(sval) == len(sp)
        assert shard_rows_by_privacy_id("trusted", pid, pk, val, enc)[0] is pid
        results[rank] = "ok"
    except Exception as e:
        results[rank] = repr(e)
    finally:
        dist.destroy_process_group()


def test_privacy_ids_spanning_ranks_are_detected_and_shuffle_fixes_them():
    """rows sharded by row would let one privacy id contribute on
    several ranks (world x L0 partitions, breaking the sensitivity); the
    library detects it, or exchanges the rows by privacy-id owner."""
    import torch.multiprocessing as mp
    manager = mp.Manager()
    results = manager.dict()
    mp.spawn(_pid_worker, args=(_free_port(), results), nprocs=WORLD, join=True)
    assert dict(results) == {0: "ok", 1: "ok"}
