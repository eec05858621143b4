"""TEST INFRASTRUCTURE — the "strong" CPU baseline of bench.py.

The vectorised NumPy oracle (oracle/columnar.py) run on many host cores at
once: the rows are sharded by privacy id over worker processes (each worker
bounds and reduces its own shard, like one GPU rank), the per-partition
accumulators are summed, then selection and noise run once.  This is what a
careful multi-core CPU implementation of the reference's LocalBackend path
(pipeline_backend.py:477-583) looks like; the reference itself is
single-threaded.  bench.py calls it on rank 0 before
any GPU work (the worker pool is started from a process with no GPU state).
"""
import os
import time

import numpy as np


def c3_shard(rows, privacy_ids, partitions, zipf_a, seed):
    """C3-shaped synthetic shard: uniform pid over its own
    privacy ids, Zipf(a) partition keys folded into `partitions`, U(0, 10)."""
    rng = np.random.default_rng(seed)
    pid = rng.integers(0, privacy_ids, rows)
    w = np.arange(1, partitions + 1, dtype=np.float64) ** -zipf_a
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    pk = np.minimum(np.searchsorted(cdf, rng.random(rows)), partitions - 1)
    val = rng.random(rows) * 10.0
    return pid, pk, val


def _worker(args):
    from oracle import columnar as O
    rows, privacy_ids, partitions, zipf_a, l0, linf, seed = args
    pid, pk, val = c3_shard(rows, privacy_ids, partitions, zipf_a, seed)
    t0 = time.perf_counter()
    acc = O.bound_and_reduce(pid, pk, val, n_privacy_ids=privacy_ids, n_partitions=partitions, l0=l0,
                             linf=linf, value_kind=O.VALUE_F64, flags=O.ACC_NSUM, min_value=0.0,
                             max_value=10.0, middle=5.0, seed=seed)
    dt = time.perf_counter() - t0
    return dt, acc["privacy_id_count"], acc["count"], acc["normalized_sum"]


def usable_cpus():
    """(workers, note): the CPUs this process may run on -- os.cpu_count(),
    bounded by its affinity mask and by a cgroup CPU quota (cpu.max) when one
    is set (a GPU box grants each GPU a share of a larger host's cores)."""
    total = os.cpu_count() or 1
    n, why = total, []
    try:
        aff = len(os.sched_getaffinity(0))
        if aff < n:
            n, why = aff, why + [f"affinity {aff}"]
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(quota) // int(period))
            if q < n:
                n, why = q, why + [f"cgroup quota {q}"]
    except (OSError, ValueError):
        pass
    return n, f"os.cpu_count() = {total}" + (f", usable {n} ({', '.join(why)})" if why else "")


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def run(workers, rows_per_worker, privacy_ids_per_worker, partitions, zipf_a, l0, linf, eps, delta):
    """Returns (rows/s, seconds, kept partitions): max-over-workers bounding
    time plus the merge, selection and noise on the summed accumulators."""
    import multiprocessing as mp
    from oracle import columnar as O
    from oracle import pydp_restatement as pydp
    jobs = [(rows_per_worker, privacy_ids_per_worker, partitions, zipf_a, l0, linf, 1000 + w)
            for w in range(workers)]
    with mp.get_context("spawn").Pool(workers) as pool:
        res = pool.map(_worker, jobs)
    t0 = time.perf_counter()
    pidc = np.sum([r[1] for r in res], axis=0)
    cnt = np.sum([r[2] for r in res], axis=0)
    nsum = np.sum([r[3] for r in res], axis=0)
    eps_each = eps / 3
    table = np.asarray(pydp.truncated_geometric_table(eps_each, delta, l0), dtype=np.float64)
    keep, _ = O.select(pidc, O.SELECT_TRUNCATED_GEOMETRIC, keep_prob=table, seed=7)
    idx = np.flatnonzero(keep)
    none = pydp.laplace_params(1.0, 0.0)
    ops = [dict(kind=O.OP_MEAN, out_col=[0, 1, 2, -1], middle=5.0,
                noise=[pydp.laplace_params(eps_each, l0 * linf), pydp.laplace_params(eps_each, l0 * linf * 5.0),
                       none])]
    O.noise_metrics(ops, idx, {"count": cnt, "normalized_sum": nsum, "privacy_id_count": pidc}, False,
                    None, seed=9)
    dt = max(r[0] for r in res) + (time.perf_counter() - t0)
    return workers * rows_per_worker / dt, dt, len(idx)


if __name__ == "__main__":
    print(run(usable_cpus()[0], 1_000_000, 10_000, 1_000_000, 1.1, 2, 1, 1.0, 1e-6))
