"""Multi-rank dataset histograms on the CPU (gloo, world_size 2): the
exchange between pdp_dataset_histograms_pairs and _finish, and the merge of
the ranks' bins (pipelinedp_amd.parallel).  The kernels themselves run in
tests/test_gpu_histograms.py (two ranks on one GPU)."""
import os
import socket
import struct

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pipelinedp_amd import parallel


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ord(x: float) -> int:
    """the kernels' order-preserving uint64 image of an fp64, as int64 bits"""
    b = struct.unpack("<Q", struct.pack("<d", x))[0]
    o = (~b & 0xFFFFFFFFFFFFFFFF) if b >> 63 else (b | (1 << 63))
    return struct.unpack("<q", struct.pack("<Q", o))[0]


def _worker(rank, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        pkstat = torch.tensor([(1 << 32) | 5, 0, (2 << 32) | 7][::1 if rank == 0 else -1], dtype=torch.int64)
        psum = torch.tensor([1.5, -2.0, 0.25], dtype=torch.float64) * (rank + 1)
        mins = [-3.5, 2.0] if rank == 0 else [0.5, 7.25]
        minmax = torch.tensor([_ord(mins[0]), _ord(mins[1])], dtype=torch.int64)
        parallel.exchange_histogram_stats(pkstat, psum, minmax, None)
        out = {
            "int_count": torch.tensor([[2, 0, 1]], dtype=torch.int64) * (rank + 1),
            "int_sum": torch.tensor([[4, 0, 9]], dtype=torch.int64),
            "int_max": torch.tensor([[2, 0, 9 - rank]], dtype=torch.int64),
            "float_count": torch.tensor([[1, 0], [1, 1]], dtype=torch.int64) if rank == 0 else
            torch.tensor([[1, 1], [0, 0]], dtype=torch.int64),
            "float_sum": torch.tensor([[-1.0, 0.0], [3.0, -4.0]], dtype=torch.float64) if rank == 0 else
            torch.tensor([[-2.0, 5.0], [0.0, 0.0]], dtype=torch.float64),
            "float_max": torch.tensor([[-1.0, 0.0], [3.0, -4.0]], dtype=torch.float64) if rank == 0 else
            torch.tensor([[-0.5, 5.0], [0.0, 0.0]], dtype=torch.float64),
            "float_lowers": torch.tensor([[-3.0, 0.0, 6.0], [1.0, 2.0, 4.0]], dtype=torch.float64) if rank == 0 else
            torch.tensor([[-3.0, 0.0, 6.0], [0.0, 0.0, 0.0]], dtype=torch.float64),
            "float_n_lowers": torch.tensor([3, 3 if rank == 0 else 0], dtype=torch.int32),
        }
        parallel.merge_histogram_bins(out, None)
        results[rank] = ({k: v.tolist() for k, v in out.items()}, pkstat.tolist(), psum.tolist(), minmax.tolist())
    except Exception as e:  # pragma: no cover - reported by the parent
        results[rank] = repr(e)
    finally:
        dist.destroy_process_group()


def test_exchange_and_merge_two_ranks():
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.spawn(_worker, args=(_free_port(), results), nprocs=2, join=True)
    assert all(isinstance(results[r], tuple) for r in (0, 1)), dict(results)
    out, pkstat, psum, minmax = results[0]
    assert results[1] == results[0]  # every rank holds the merged result
    assert pkstat == [(3 << 32) | 12, 0, (3 << 32) | 12]
    assert np.allclose(psum, [4.5, -6.0, 0.75])
    assert minmax == [_ord(-3.5), _ord(7.25)]  # global min of the mins, max of the maxes
    assert out["int_count"] == [[6, 0, 3]] and out["int_sum"] == [[8, 0, 18]] and out["int_max"] == [[2, 0, 9]]
    assert out["float_count"] == [[2, 1], [1, 1]]
    assert out["float_sum"] == [[-3.0, 5.0], [3.0, -4.0]]
    # bin maxima only over ranks whose bin holds elements (rank 1's empty
    # partition bins hold 0.0 and must not win over -4.0)
    assert out["float_max"] == [[-0.5, 5.0], [3.0, -4.0]]
    assert out["float_lowers"] == [[-3.0, 0.0, 6.0], [1.0, 2.0, 4.0]]
    assert out["float_n_lowers"] == [3, 3]


def _overflow_worker(rank, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        # rows of one partition: 2^31 + 5 on each rank -> 2^32 + 10 in total, which
        # would carry into the packed privacy-id count
        pkstat = torch.tensor([(1 << 32) | ((1 << 31) + 5), (1 << 32) | 3], dtype=torch.int64)
        psum = torch.zeros(2, dtype=torch.float64)
        minmax = torch.tensor([_ord(0.0), _ord(1.0)], dtype=torch.int64)
        try:
            parallel.exchange_histogram_stats(pkstat, psum, minmax, None)
            results[rank] = "no error"
        except ValueError as e:
            results[rank] = "ValueError" if "2^32" in str(e) else repr(e)
    finally:
        dist.destroy_process_group()


def test_partition_counter_overflow_across_ranks_raises():
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.spawn(_overflow_worker, args=(_free_port(), results), nprocs=2, join=True)
    assert dict(results) == {0: "ValueError", 1: "ValueError"}


def _weights_worker(rank, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        # L0/L1 weight sums that land exactly on x.5 only when the ranks' parts
        # are added before rounding: key 7 -> 1.25 + 1.25, key 9 -> 0.5 + 2.0,
        # key 11 only on rank 1 (3/8 + 1/8 in one part)
        wsmall = torch.zeros(2000, dtype=torch.float64)
        wsmall[3] = 0.75 if rank == 0 else 1.75
        keys = [7, 9] if rank == 0 else [9, 7, 11]
        ws = [1.25, 0.5] if rank == 0 else [2.0, 1.25, 0.5]
        wtab = torch.zeros((8, 2), dtype=torch.int64)
        for i, (k, w) in enumerate(zip(keys, ws)):
            wtab[2 * i, 0] = k
            wtab[2 * i, 1] = torch.tensor([w], dtype=torch.float64).view(torch.int64)[0]
        uk, uw = parallel.exchange_preaggregated_weights(wsmall, wtab, None)
        results[rank] = (dict(zip(uk.tolist(), uw.tolist())), wsmall[3].item(), int(wtab.abs().sum()))
    except Exception as e:  # pragma: no cover - reported by the parent
        results[rank] = repr(e)
    finally:
        dist.destroy_process_group()


def test_preaggregated_weights_summed_before_rounding():
    """2-rank pre-aggregated weights equal the 1-rank sums at a .5
    tie (dyadic weights: every addition order gives the same fp64 sum, so the
    2-rank and 1-rank bins round alike; non-dyadic ties such as 1/3 + 1/6 can
    differ by an ulp with the summation order -- as the reference's own Python
    sum order does -- and stay parity-unpinned)."""
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.spawn(_weights_worker, args=(_free_port(), results), nprocs=2, join=True)
    assert all(isinstance(results[r], tuple) for r in (0, 1)), dict(results)
    merged = {}
    for r in (0, 1):
        for k, w in results[r][0].items():
            assert k not in merged  # each key summed on exactly one (its owner) rank
            merged[k] = w
    assert merged == {7: 2.5, 9: 2.5, 11: 0.5}
    assert [round(merged[k]) for k in (7, 9)] == [2, 2]  # half to even, as one rank's 2.5
    assert results[0][1] == 2.5 and results[1][1] == 0.0  # small weights: rank 0 holds the sum
    assert results[0][2] == 0 and results[1][2] == 0       # the tables are zeroed
