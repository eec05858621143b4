"""TEST INFRASTRUCTURE — the NumPy oracle (oracle/columnar.py) on many host cores.

Bounding is a function of one privacy id's rows (contribution_bounders.py:
62-111), so the oracle's bound_and_reduce runs independently on privacy-id
shards (pid mod K) and the per-partition accumulators add up
(combine_accumulators_per_key, pipeline_backend.py:555-565).  Every shard
keeps its rows' indices in the full input (row_index), so the row priorities
are those of the unsharded oracle and of the kernels: integer outputs are
bit-identical to oracle.columnar.bound_and_reduce on the whole input; fp64
sums differ only in summation order.  Used by the at-scale GPU parity tests
(1e7-1e8 rows), where the single-process oracle would take minutes.

The columns are handed over as .npy files memory-mapped by the workers
(started with the 'spawn' method: children never inherit GPU state).
"""
import os
import tempfile

import numpy as np


def _worker(args):
    from oracle import columnar as O
    d, k, K, kw = args
    pid = np.load(os.path.join(d, "pid.npy"), mmap_mode="r")
    pk = np.load(os.path.join(d, "pk.npy"), mmap_mode="r")
    val = np.load(os.path.join(d, "val.npy"), mmap_mode="r") if os.path.exists(os.path.join(d, "val.npy")) else None
    rows = np.flatnonzero((pid % K) == k)
    return O.bound_and_reduce(np.asarray(pid[rows]), np.asarray(pk[rows]), val, row_index=rows, **kw)


def bound_and_reduce(pid, pk, value, workers=None, **kw):
    """oracle.columnar.bound_and_reduce over `workers` processes (same keyword
    arguments; the privacy ids must be non-negative)."""
    import multiprocessing as mp
    from oracle import columnar as O
    pid = np.ascontiguousarray(pid, dtype=np.int64)
    if workers is None:
        workers = max(1, min(16, (os.cpu_count() or 1)))
    if workers == 1 or len(pid) < 1_000_000:
        return O.bound_and_reduce(pid, pk, value, **kw)
    if np.any(pid < 0):
        raise ValueError("parallel oracle needs non-negative privacy ids")
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        np.save(os.path.join(d, "pid.npy"), pid)
        np.save(os.path.join(d, "pk.npy"), np.ascontiguousarray(pk, dtype=np.int64))
        if value is not None:
            np.save(os.path.join(d, "val.npy"), np.ascontiguousarray(value))
        with mp.get_context("spawn").Pool(workers) as pool:
            parts = pool.map(_worker, [(d, k, workers, kw) for k in range(workers)])
    out = {}
    for name in parts[0]:
        out[name] = np.sum([p[name] for p in parts], axis=0).astype(parts[0][name].dtype)
    return out
