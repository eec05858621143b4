#!/usr/bin/env python3
"""Benchmark of the DPEngine.aggregate hot path on MI355X (BASELINE.json).

Workloads:
  c3 (default, BASELINE configs[2], the north-star target shape): 1e9 rows in
     total, privacy ids uniform over 1e7, partition keys Zipf(1.1) folded into
     1e6 partitions, values U(0, 10); COUNT + SUM + MEAN, Laplace,
     max_partitions_contributed = 2 (sampling fires), max_contributions_per_
     partition = 1, private partitions (truncated geometric), eps = 1,
     delta = 1e-6.  Strong scaling: N GPUs share the 1e9 rows, sharded by
     privacy id (rank r holds the privacy ids = r mod N).
  c2 (BASELINE configs[1]): 1e8 rows per GPU, 1e6 privacy ids, 1e5 uniform
     partitions, values N(5, 3) clipped to [0, 10], L0 = 8, Linf = 2.  Weak
     scaling.  At N = 1 with the default workload it also runs as the
     `secondary` object of the JSON line.
  c4 (BASELINE configs[3]): VARIANCE + PRIVACY_ID_COUNT,
     Gaussian noise, private partition selection, 1e7 uniform partitions,
     values U(0, 10), L0 = 4, Linf = 2; 1.25e8 rows and 1.25e7 privacy ids
     per GPU, so N = 8 is the 1e9-row, 1e8-id configuration.  Weak scaling.
  c5 (BASELINE configs[4]): COUNT + SUM + MEAN, no public
     partitions, rows per privacy id discrete Pareto(1.5) capped at 1e6 and
     rescaled to the row count (rows shuffled), partition keys Zipf(1.1)
     folded into 1e7, values lognormal(1, 1) clipped to [0, 20], L0 = 4,
     Linf = 2; 6.25e8 rows and 1.25e7 privacy ids per GPU, so N = 8 is the
     5e9-row, 1e8-id configuration.  Weak scaling.
  c4 and c5 time the public API: pipelinedp_amd.DPEngine.aggregate over a
  device-resident ColumnTable on ColumnarBackend (trusted privacy-id
  sharding), + compute_budgets() + the collected result, per step.

A step = one full aggregate over the resident batch: contribution bounding
(L0 + Linf sampling), per-partition reduction, [RCCL reduce-scatter of the
accumulators], partition selection, compaction and noisy metrics, ending with
the kept-partition count on the host.  Inputs are resident in HBM before
timing starts.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]
  With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts
  `python -m torch.distributed.run --nproc-per-node N` on itself as a child
  process (before touching the GPU) and exits with its status.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np


HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

# HBM bytes per launch from rocprofv3 PMC passes over this same bench command
# (tools/gpu_pmc.sh -> tools/pmc_summary.py: 2 x FETCH_SIZE for the gfx950
# wide-load under-count + WRITE_SIZE, MI355X_MICROARCH.md "HBM").  Valid for
# the workload and tree named in the file; None otherwise.
PMC_SUMMARY = {w: os.path.join(HERE, "profiles", "r06", f"{w}_pmc.json") for w in ("c3", "c2", "c4", "c5", "hist")}


# kernels whose work depends on the step's data (the sieve's fix-up: how many
# privacy ids stay unresolved, how many rows the band and the fix-up list hold)
# -> the bound_plan.stats fields that measure it.  Their PMC bytes are joined
# only when the profiled run's stats equal this run's on those fields and the
# profiled launches moved about the same bytes each.
DATA_DEPENDENT = {
    "k_band_scan": ("unresolved_ids", "band_rows"),
    "k_fix_filter": ("fixup_rows", "fixup2_rows"),
    "k_fix_scatter": ("fixup_rows", "fixup2_rows"),
    "k_fix_buckets": ("unresolved_ids", "unresolved2_ids"),
    "k_bucket_fix": ("unresolved_ids", "fixup_rows"),
    "k_sieve_rescan": ("unresolved_ids", "unresolved2_ids", "fixup2_rows"),
    "k_bucket_fix2": ("unresolved2_ids", "fixup2_rows"),
}


def join_pmc_entry(kernel, e, pmc_stats, stats):
    """Whether a PMC summary entry may stand for this run's launches of `kernel`."""
    keys = DATA_DEPENDENT.get(kernel)
    if keys is None:
        return True
    if not pmc_stats or not stats or any(pmc_stats.get(k) != stats.get(k) for k in keys):
        return False
    lo, hi = e.get("launch_hbm_bytes_min"), e.get("launch_hbm_bytes_max")
    return lo is not None and hi is not None and hi <= 1.25 * lo + 1e6


def load_pmc(pmc_file, workload, n, world, stats=None):
    """Per-kernel HBM bytes from a PMC summary, joined only when it was made
    from this workload at this size AND from these kernel sources (its "tree"
    equals tools/tree_id.py's id of the tree bench.py runs on); a
    data-dependent kernel's entry only when join_pmc_entry allows it.  Returns
    (traffic, source, refused): refused names why a file present was not used."""
    if world != 1 or not pmc_file or not os.path.exists(pmc_file):
        return {}, None, None
    sys.path.insert(0, os.path.join(HERE, "tools"))
    from tree_id import source_tree_id
    with open(pmc_file) as f:
        pmc = json.load(f)
    src = os.path.relpath(pmc_file, HERE)
    if not pmc.get("workload", "").startswith(f"{workload} n={n} "):
        return {}, None, f"{src}: workload {pmc.get('workload')!r}, not {workload} n={n}"
    tree = source_tree_id()
    if pmc.get("tree") != tree:
        return {}, None, f"{src}: profiled tree {pmc.get('tree')}, this tree {tree}"
    return ({k: v["hbm_bytes"] for k, v in pmc["kernels"].items()
             if "hbm_bytes" in v and join_pmc_entry(k, v, pmc.get("stats"), stats)}, src, None)


def pmc_entry(e, k, traffic, ms):
    """Adds a kernel's PMC bytes to its table entry -- unless they imply a rate
    above the HBM peak, which no launch can move (a figure from launches that
    did other work than these); returns whether they were added."""
    if k not in traffic:
        return False
    gbs = traffic[k] / (ms * 1e-3) / 1e9
    if gbs > HBM_PEAK_GBS:
        return False
    e["pmc_bytes"] = traffic[k]
    e["pmc_gbs"] = gbs
    return True

# workload constants
C2 = dict(rows=100_000_000, privacy_ids=1_000_000, partitions=100_000, l0=8, linf=2)
C3 = dict(rows=1_000_000_000, privacy_ids=10_000_000, partitions=1_000_000, l0=2, linf=1, zipf=1.1)
C4 = dict(rows=125_000_000, privacy_ids=12_500_000, partitions=10_000_000, l0=4, linf=2)
C5 = dict(rows=625_000_000, privacy_ids=12_500_000, partitions=10_000_000, l0=4, linf=2, pareto=1.5,
          max_rows_per_id=1_000_000, zipf=1.1, max_value=20.0)
MIN_VALUE, MAX_VALUE = 0.0, 10.0
EPS, DELTA = 1.0, 1e-6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--privacy-ids", type=int, default=0,
                    help="C3: privacy ids in total (default: the config's 1e7; with --rows, one rank's "
                         "share of an N-GPU run on one GPU); C4 / C5: privacy ids per rank")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("c3", "c2", "c4", "c5", "hist"), default="c3")
    ap.add_argument("--rows", type=int, default=0, help="override: rows in total (c3) / per GPU (c2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-secondary", action="store_true", help="skip the C2 secondary run at N = 1")
    ap.add_argument("--cpu-sample-rows", type=int, default=1_000_000)
    ap.add_argument("--key-format", type=int, default=0, help="PDP_KEYS_* (0 auto)")
    ap.add_argument("--sieve-band", type=int, default=0,
                    help="the sieve's side band (0 auto, -1 off; pdp_bound_config.sieve_band)")
    ap.add_argument("--sieve", type=int, default=0,
                    help="threshold sieve t * 2^16 (0 auto, -1 off; pdp_bound_config.sieve)")
    ap.add_argument("--sieve-threads", type=int, default=0,
                    help="the sieve's level-1 workgroup: 0 auto, 512 or 1024 (pdp_bound_config.sieve_threads)")
    ap.add_argument("--bucket-threads", type=int, default=0,
                    help="the bucket kernel's workgroup: 0 auto, 512 or 1024 (pdp_bound_config.bucket_threads)")
    ap.add_argument("--small-ids", type=float, default=0.0,
                    help="C3 variant: this fraction of the privacy ids holds 1-3 rows each (light users)")
    ap.add_argument("--merge", type=int, default=0, help="PDP_MERGE_* (0 auto, 1 atomic, 2 ranges)")
    ap.add_argument("--seed", type=int, default=20261017,
                    help="sampling seed base: step i uses seed + i, so a run is reproducible (c2 / c3)")
    ap.add_argument("--strategy", choices=("truncated_geometric", "gaussian", "laplace"),
                    default="truncated_geometric",
                    help="c4 / c5: AggregateParams.partition_selection_strategy (SURVEY §8(d) C4 names "
                         "TRUNCATED_GEOMETRIC and GAUSSIAN_THRESHOLDING)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks join a gloo group and rank 0 prints the "
                         "n_gpus it sees (tests/test_bench_launcher.py)")
    ap.add_argument("--share-of", type=int, default=0,
                    help="c3 at N = 1: one rank's share of an N-GPU run -- rows / N, privacy ids / N, and "
                         "selection + noise over the rank's P / N partitions after the (omitted) "
                         "reduce-scatter, as every rank of the N-GPU run does (VERDICT r04 #4)")
    ap.add_argument("--no-api", dest="api", action="store_false",
                    help="skip the public-API timing (DPEngine.aggregate on ColumnarBackend)")
    return ap.parse_args()


def maybe_spawn(args):
    """--gpus N > 1 without a torch.distributed environment: run N ranks of
    this script under torch.distributed.run as a CHILD process (no exec, no
    GPU touched in this process) and exit with its status."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.call(cmd, env=env))


def build_plan(l0, linf):
    """Noise / selection parameters exactly as DPEngine + NaiveBudgetAccountant
    derive them for this AggregateParams (3 mechanisms of weight 1: MEAN's
    count and normalized-sum Laplace mechanisms + the GENERIC selection)."""
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import dp_computations as dpc
    from pipelinedp_amd import executor as X
    eps_each = EPS / 3
    mid = dpc.compute_middle(MIN_VALUE, MAX_VALUE)
    count_noise = dpc.laplace_noise_params(eps_each, l0 * linf)
    nsum_noise = dpc.laplace_noise_params(eps_each, l0 * (MAX_VALUE - MIN_VALUE) / 2 * linf)
    bounding = X.BoundingSpec(l0=l0, linf=linf, value_kind=N.VALUE_F64, flags=N.ACC_NSUM,
                              min_value=MIN_VALUE, max_value=MAX_VALUE, middle=mid)
    selection = X.SelectionSpec(strategy=N.SELECT_TRUNCATED_GEOMETRIC,
                                keep_prob=dpc.truncated_geometric_keep_table(eps_each, DELTA, l0))
    ops = [X.MetricOpSpec(kind=N.OP_MEAN, out_col=(0, 1, 2), noise=(count_noise, nsum_noise), middle=mid)]
    return bounding, selection, ops


def cpu_baselines(workload, sample_rows):
    """Rank 0, N = 1, after the GPU work in a child process.  `port`: the
    row-wise restatement of LocalBackend DPEngine.aggregate (the reference's
    single-threaded CPU path, oracle/local_backend_port.py) on a bounded
    sample of the workload; `strong`: the vectorised NumPy oracle on every
    CPU this process may use (os.cpu_count() bounded by the affinity mask and
    the cgroup quota, oracle/strong_baseline.py); `c1`: the
    port at BASELINE config 1 itself (1e6 movie_view rows, COUNT + SUM,
    BASELINE.md §3.1)."""
    from oracle import local_backend_port as port
    from oracle import strong_baseline as strong
    w = C3 if workload == "c3" else C2
    U = max(1, sample_rows // 100)
    if workload == "c3":
        pid, pk, val = strong.c3_shard(sample_rows, U, w["partitions"], w["zipf"], 1)
    else:
        rng = np.random.default_rng(1)
        pid = rng.integers(0, U, sample_rows)
        pk = rng.integers(0, w["partitions"], sample_rows)
        val = np.clip(rng.normal(5.0, 3.0, sample_rows), MIN_VALUE, MAX_VALUE)
    rows = list(zip(pid.tolist(), pk.tolist(), val.tolist()))
    t0 = time.perf_counter()
    out = port.aggregate_count_sum_mean(rows, l0=w["l0"], linf=w["linf"], min_value=MIN_VALUE,
                                        max_value=MAX_VALUE, eps=EPS, delta=DELTA)
    dt = time.perf_counter() - t0
    model = strong.cpu_model()
    base = {"value": sample_rows / dt, "unit": "rows/s", "cores": 1, "kind": "port", "cpu_model": model,
            "sample": f"{sample_rows} rows shaped like {workload.upper()} (U={U}, P={w['partitions']}, "
                      f"L0={w['l0']}, Linf={w['linf']}); oracle/local_backend_port.py, a row-wise "
                      f"restatement of the reference's single-threaded LocalBackend path (dict group-bys, "
                      f"np.random.choice, np.clip per pair; no namedtuples or DPEngine generators, so it "
                      f"runs ~2x the reference's own measured rate, BASELINE.md §2); {dt:.1f} s, "
                      f"{len(out)} partitions kept; the full workload is a linear extrapolation"}
    workers, cpu_note = strong.usable_cpus()
    per = 2_000_000
    rate, sdt, kept = strong.run(workers, per, per // 100, w["partitions"], w.get("zipf", 0.0) or 1.0001,
                                 w["l0"], w["linf"], EPS, DELTA)
    strong_res = {"value": rate, "unit": "rows/s", "cores": workers, "kind": "port", "cpu_model": model,
                  "sample": f"{workers} x {per} rows (privacy-id shards, Zipf pk), vectorised NumPy oracle "
                            f"(oracle/columnar.py) one process per shard + merge/select/noise; "
                            f"{sdt:.2f} s, {kept} partitions kept; {cpu_note}"}
    c1_rows = port.movie_view_rows(1_000_000, seed=0)
    t0 = time.perf_counter()
    c1_out = port.aggregate_count_sum(c1_rows, l0=2, linf=1, min_value=1.0, max_value=5.0, eps=EPS, delta=DELTA)
    c1_dt = time.perf_counter() - t0
    c1 = {"value": len(c1_rows) / c1_dt, "unit": "rows/s", "cores": 1, "kind": "port", "cpu_model": model,
          "sample": f"BASELINE config 1 itself: 1e6 synthetic movie_view rows (user_id over 1e5, movie_id "
                    f"min(Zipf(1.3), 17770), rating 1-5), COUNT+SUM, L0=2, Linf=1, clip [1, 5], Laplace, "
                    f"truncated-geometric selection; oracle/local_backend_port.py aggregate_count_sum on one "
                    f"core, {c1_dt:.1f} s, {len(c1_out)} partitions kept"}
    return base, strong_res, c1


def gen_c3(n, U, P, rank, world, device, seed, small_ids=0.0):
    """This rank's shard: its U privacy ids as local codes k in [0, U) --
    the dataset-wide id of code k on rank r is owned_identities(...)[k], so
    ranks hold disjoint, hash-owned ids -- and Zipf(1.1) pk."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed + rank)
    small = int(U * small_ids)
    if small == 0:
        pid = torch.randint(0, U, (n,), generator=g, device=device, dtype=torch.int64)
    else:
        # --small-ids F: the last F*U codes hold 1-3 rows each (light users,
        # ids short of l0 partitions), the rest of the rows go
        # uniformly to the other ids, in random row order
        reps = torch.randint(1, 4, (small,), generator=g, device=device, dtype=torch.int64)
        tail = torch.repeat_interleave(torch.arange(U - small, U, device=device, dtype=torch.int64), reps)
        head = torch.randint(0, U - small, (n - tail.numel(),), generator=g, device=device, dtype=torch.int64)
        pid = torch.cat([head, tail])
        del head, tail, reps
        pid = pid[torch.randperm(n, generator=g, device=device)]
    w = torch.arange(1, P + 1, device=device, dtype=torch.float64).pow_(-C3["zipf"])
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    pk = torch.empty(n, device=device, dtype=torch.int64)
    for c0 in range(0, n, 1 << 27):  # bounded temporaries
        c1 = min(n, c0 + (1 << 27))
        u = torch.rand(c1 - c0, generator=g, device=device, dtype=torch.float64)
        pk[c0:c1] = torch.searchsorted(cdf, u).clamp_(max=P - 1)
        del u
    value = torch.rand(n, generator=g, device=device, dtype=torch.float64) * MAX_VALUE
    del w, cdf
    return pid, pk, value


def gen_c2(n, U, P, rank, device, seed):
    """Local privacy-id codes as in gen_c3 (dataset-wide ids: owned_identities)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed + rank)
    pid = torch.randint(0, U, (n,), generator=g, device=device, dtype=torch.int64)
    pk = torch.randint(0, P, (n,), generator=g, device=device, dtype=torch.int64)
    value = (torch.randn(n, generator=g, device=device, dtype=torch.float64) * 3.0 + 5.0).clamp_(
        MIN_VALUE, MAX_VALUE)
    return pid, pk, value


def gen_c4(n, U, P, rank, device, seed):
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed + rank)
    pid = torch.randint(0, U, (n,), generator=g, device=device, dtype=torch.int64)
    pk = torch.randint(0, P, (n,), generator=g, device=device, dtype=torch.int64)
    value = torch.rand(n, generator=g, device=device, dtype=torch.float64) * MAX_VALUE
    return pid, pk, value


def gen_c5(n, U, P, rank, device, seed):
    """SURVEY §8(d) C5 shard: rows per privacy id discrete Pareto(1.5)
    (floor(x_m * u^(-1/1.5)), capped at 1e6, rescaled so they sum to n, the
    remainder spread one row each over random ids), rows shuffled; pk Zipf(1.1)
    folded into P; values lognormal(1, 1) clipped to [0, 20]."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed + rank)
    u = torch.rand(U, generator=g, device=device, dtype=torch.float64).clamp_(min=1e-300)
    cnt = u.pow_(-1.0 / C5["pareto"]).floor_().clamp_(max=C5["max_rows_per_id"])
    cnt = (cnt * (n / float(cnt.sum()))).floor_().to(torch.int64).clamp_(min=0)
    short = n - int(cnt.sum())
    if short > 0:
        cnt.index_add_(0, torch.randint(0, U, (short,), generator=g, device=device),
                       torch.ones(short, dtype=torch.int64, device=device))
    pid = torch.repeat_interleave(torch.arange(U, device=device), cnt)
    del u, cnt
    pid = pid[torch.randperm(n, generator=g, device=device)]
    w = torch.arange(1, P + 1, device=device, dtype=torch.float64).pow_(-C5["zipf"])
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    pk = torch.empty(n, device=device, dtype=torch.int64)
    for c0 in range(0, n, 1 << 27):  # bounded temporaries
        c1 = min(n, c0 + (1 << 27))
        x = torch.rand(c1 - c0, generator=g, device=device, dtype=torch.float64)
        pk[c0:c1] = torch.searchsorted(cdf, x).clamp_(max=P - 1)
        del x
    del w, cdf
    value = torch.randn(n, generator=g, device=device, dtype=torch.float64).add_(1.0).exp_().clamp_(
        0.0, C5["max_value"])
    return pid, pk, value


def owned_identities(U, world, rank, device):
    """Dataset-wide privacy-id identities of rank r's local codes k in [0, U):
    the k-th non-negative integer that parallel.owner_of assigns to r, so the
    ranks' ids are disjoint and hash-owned (as parallel.shard_by_privacy_id
    or the "shuffle" mode leave them)."""
    import torch
    from pipelinedp_amd import parallel
    n = int(U * world * 1.05) + 4096
    while True:
        c = torch.arange(n, device=device, dtype=torch.int64)
        mine = c[parallel.owner_of(c, world) == rank]
        if mine.numel() >= U:
            return mine[:U].clone()
        n *= 2


def verify_sharding(ids, world, rank, U):
    """The library's default privacy_id_sharding="verify"
    (parallel.verify_privacy_id_sharding) on this rank's per-row dataset-wide
    identities, run once before the timed region: one owner check per row and
    a flag all-reduce (the id exchange only if some rank holds an id it does
    not own).  Returns {ms, path} (None at N = 1, nothing to verify)."""
    import torch
    from pipelinedp_amd import parallel
    if world == 1:
        return None
    import torch.distributed as dist
    ident = owned_identities(U, world, rank, ids.device)[ids]
    times = []
    for _ in range(2):  # the first call also loads the library's code object
        torch.cuda.synchronize()
        dist.barrier()  # time the check, not the ranks' arrival skew
        t0 = time.perf_counter()
        path = parallel.verify_privacy_id_sharding(ident)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
    del ident
    return {"ms": times[1], "first_call_ms": times[0], "path": path, "rows": int(ids.numel())}


def tuning_of(args):
    """The bench's data-movement knobs (identical results) as ColumnarBackend tuning."""
    t = dict(key_format=args.key_format, sieve=args.sieve, sieve_band=args.sieve_band,
             sieve_threads=args.sieve_threads, bucket_threads=args.bucket_threads, merge=args.merge)
    return {k: v for k, v in t.items() if v}


def run_api_workload(args, workload, world, rank, device):
    """c4 / c5: one step = DPEngine.aggregate (the public API) over this
    rank's device-resident rows on ColumnarBackend, compute_budgets(), and
    the collected result; the accumulator exchange runs over RCCL at N > 1."""
    import torch
    import torch.distributed as dist
    import pipelinedp_amd as pdp
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import columnar_backend as CB
    from pipelinedp_amd import executor as X
    w = C4 if workload == "c4" else C5
    n, U, P = args.rows or w["rows"], args.privacy_ids or w["privacy_ids"], w["partitions"]
    gen = gen_c4 if workload == "c4" else gen_c5
    pid, pk, value = gen(n, U, P, rank, device, 4000 if workload == "c4" else 5000)
    # local privacy-id codes k in [0, U), dataset-wide ids owned_identities
    # (as in gen_c3): a rank's table is dense in its own ids, so its bounding plan
    # is the one-GPU plan (global codes in [0, U * world) would give 8x the
    # buckets at N = 8, past the bucketed plan's limit: the global-sketch path)
    torch.cuda.synchronize()
    # the default privacy_id_sharding="verify" on the dataset-wide ids, once,
    # before timing (the steps below pass "trusted": the check does not
    # change between steps)
    verify_ms = verify_sharding(pid, world, rank, U)
    table = pdp.ColumnTable({"pid": pid, "pk": pk, "v": value}, n_privacy_ids=U, n_partitions=P)
    strategy = {"truncated_geometric": pdp.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC,
                "gaussian": pdp.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING,
                "laplace": pdp.PartitionSelectionStrategy.LAPLACE_THRESHOLDING}[args.strategy]
    if workload == "c4":
        params = pdp.AggregateParams(metrics=[pdp.Metrics.VARIANCE, pdp.Metrics.PRIVACY_ID_COUNT],
                                     partition_selection_strategy=strategy,
                                     noise_kind=pdp.NoiseKind.GAUSSIAN, max_partitions_contributed=w["l0"],
                                     max_contributions_per_partition=w["linf"], min_value=MIN_VALUE,
                                     max_value=MAX_VALUE)
    else:
        params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.MEAN],
                                     partition_selection_strategy=strategy,
                                     noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=w["l0"],
                                     max_contributions_per_partition=w["linf"], min_value=MIN_VALUE,
                                     max_value=C5["max_value"])
    ext = pdp.DataExtractors(privacy_id_extractor=pdp.ColumnExtractor("pid"),
                             partition_extractor=pdp.ColumnExtractor("pk"),
                             value_extractor=pdp.ColumnExtractor("v"))
    ws = X.BoundWorkspace()
    tune = tuning_of(args)

    counter = [0]

    def step():
        # seeded per step (bench.py --seed): the line is reproducible
        counter[0] += 1
        acc = pdp.NaiveBudgetAccountant(total_epsilon=EPS, total_delta=DELTA)
        backend = CB.ColumnarBackend(privacy_id_sharding="trusted", workspace=ws, tuning=tune,
                                     seed=args.seed + counter[0])
        sink = pdp.DPEngine(acc, backend).aggregate(table, params, ext)
        acc.compute_budgets()
        return len(sink.collect()), backend

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kept = 0
    for _ in range(args.steps):
        kept, backend = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    N.profiler_enable(True)
    for _ in range(args.steps):
        step()
    kernels = N.profiler_report()
    N.profiler_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    info = backend.last_plan_info
    # kept pairs / rows and the plan's stats for the byte accounting: one more
    # bounding pass with the spec the API built (untimed)
    spec = backend.last_bounding
    acc = X.new_accumulators(P, spec, device)
    X.bound_and_reduce(pid, pk, value, n_privacy_ids=U, n_partitions=P, bounding=spec, seed=1, acc=acc,
                       workspace=ws, **tune)
    kept_pairs = int(acc["privacy_id_count"].sum().item())
    kept_rows = int(acc["count"].sum().item())
    n_fields = sum(acc[k] is not None for k in ("sum", "normalized_sum", "normalized_sum_sq"))
    stats = ws.stats()
    plan = X.bound_plan(n, U, P, spec, **tune)
    del pid, pk, value, table, ws, acc
    kernel_ms = {k: v[0] / v[1] for k, v in kernels.items()}
    launches = {k: v[1] / args.steps for k, v in kernels.items()}
    ms_per_step = elapsed / args.steps * 1e3
    traffic, traffic_src, traffic_refused = load_pmc(PMC_SUMMARY[workload], workload, n, world, stats)
    alg = kernel_alg_bytes(plan, n, kept_pairs, kept_rows, n_fields, stats, P)
    table = {}
    for k, ms in kernel_ms.items():
        e = {"ms": ms, "launches_per_step": launches[k]}
        if k in alg:
            e["alg_bytes"] = alg[k]
            e["achieved_gbs"] = alg[k] / (ms * 1e-3) / 1e9
            e["frac"] = e["achieved_gbs"] / HBM_PEAK_GBS
        if not pmc_entry(e, k, traffic, ms):
            traffic.pop(k, None)  # out of traffic_per_step too
        table[k] = e
    dom = max(kernel_ms, key=lambda k: kernel_ms[k] * launches[k])
    # compulsory bytes: the three input columns once, and per
    # kept partition its key, accumulators and output metrics
    k_out = 2 if workload == "c4" else 3
    path_bytes = 24.0 * n + kept * (8 + 8 * (2 + n_fields) + 8 * k_out)
    path_gbs = path_bytes / (ms_per_step * 1e-3) / 1e9
    strat = args.strategy.replace("_", " ") + ("" if args.strategy == "truncated_geometric" else " thresholding")
    desc = (f"C4: DPEngine.aggregate VARIANCE+PRIVACY_ID_COUNT, Gaussian, private partitions ({strat}), "
            f"L0=4, Linf=2, uniform keys" if workload == "c4" else
            f"C5: DPEngine.aggregate COUNT+SUM+MEAN, Laplace, private partitions ({strat}), L0=4, Linf=2, rows per "
            "privacy id Pareto(1.5) capped at 1e6, Zipf(1.1) partition keys, lognormal values in [0, 20]")
    return {
        "value": n * world * args.steps / elapsed,
        "ms_per_step": ms_per_step,
        "config": {"workload": f"{desc}, {n:.3g} rows and {U:.3g} privacy ids per GPU, {P:.3g} partitions",
                   "rows_per_gpu": n, "privacy_ids_per_gpu": U, "partitions": P,
                   "parallelism": f"rows sharded by privacy_id over {world} GPU(s)",
                   "timed": "public API per step: DPEngine.aggregate + compute_budgets() + collect()"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": table[dom].get("achieved_gbs"),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": table[dom].get("frac"),
                     "traffic": traffic.get(dom), "traffic_source": traffic_src, "traffic_refused": traffic_refused,
                     "bytes_per_launch": alg.get(dom), "avg_ms": kernel_ms[dom]},
        "path_roofline": {"achieved": path_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": path_gbs / HBM_PEAK_GBS, "bytes_per_step": path_bytes,
                          "traffic_per_step": sum(traffic.values()) if traffic else None},
        "kernels": table, "kept_pairs": kept_pairs, "kept_rows": kept_rows,
        "bound_plan": None if info is None else {
            "algorithm": info.algorithm, "bucket_bits": info.bucket_bits, "n_buckets": info.n_buckets,
            "lds_bytes": info.lds_bytes, "merge": info.merge, "sieve": info.sieve / 65536.0,
            "band": info.band / 65536.0, "tuning": tune, "stats": stats,
            "bucket_threads": info.bucket_threads,
            "key_format": {1: "wide", 2: "compact", 3: "packed", 4: "packed_wide", 5: "packed64"}.get(info.key_format,
                                                                                     info.key_format)},
        "seed": args.seed,
        "partitions_kept": kept,
        "privacy_id_verify_ms": verify_ms,
    }


HIST = dict(rows=100_000_000, privacy_ids=1_000_000, partitions=100_000)


def run_hist_workload(args, world, rank, device):
    """compute_dataset_histograms' device pass (SURVEY §8(f) rank 4,
    computing_histograms.py:456-513) on C2's shape: 1e8 rows per GPU, 1e6
    privacy ids, 1e5 partitions, fp64 values N(5, 3) clipped to [0, 10],
    inputs resident in HBM.  One step = one pdp_dataset_histograms call (all
    seven histograms, bins on the device; multi-rank: the exchange and merge
    included)."""
    import torch
    import torch.distributed as dist
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import executor as X
    n = args.rows or HIST["rows"]
    U, P = HIST["privacy_ids"], HIST["partitions"]
    g = torch.Generator(device=device)
    g.manual_seed(3000 + rank)
    pid = torch.randint(0, U, (n,), generator=g, device=device, dtype=torch.int64)
    pk = torch.randint(0, P, (n,), generator=g, device=device, dtype=torch.int64)
    val = (torch.randn(n, generator=g, device=device, dtype=torch.float64) * 3.0 + 5.0).clamp_(MIN_VALUE, MAX_VALUE)
    ws = X.BoundWorkspace()

    def step():
        X.dataset_histograms(pid, pk, val, n_privacy_ids=U, n_partitions=P, workspace=ws)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    N.profiler_enable(True)
    for _ in range(args.steps):
        step()
    kernels = N.profiler_report()
    N.profiler_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    pairs = int(torch.unique(pid * P + pk).numel())  # distinct (privacy id, partition) pairs, untimed
    del pid, pk, val, ws
    kernel_ms = {k: v[0] / v[1] for k, v in kernels.items()}
    launches = {k: v[1] / args.steps for k, v in kernels.items()}
    # algorithmic bytes per launch: rows read / records moved once
    alg = {"k_hb_count": 16.0 * n, "k_hb_l1": (24.0 + 16.0) * n, "k_hb_bcount": 8.0 * n,
           "k_hb_l2": 32.0 * n, "k_hb_pairs": 16.0 * n,
           # the per-bucket pair pass: 16-byte records in, a 16-byte (partition,
           # rows, sum) record out per distinct pair; the range pass and the
           # float histogram's two passes (counts + sums, maxima) read those
           # once each; per-id / per-partition stats
           "k_hb_pid_pairs": 16.0 * n + 16.0 * pairs, "k_hb_prange": 16.0 * pairs,
           "k_h_float": 16.0 * pairs, "k_h_float_max": 16.0 * pairs, "k_h_ids": 16.0 * (U + P)}
    traffic, traffic_src, traffic_refused = load_pmc(PMC_SUMMARY["hist"], "hist", n, world)
    table = {}
    for k, ms in kernel_ms.items():
        e = {"ms": ms, "launches_per_step": launches[k]}
        if k in alg:
            e["alg_bytes"] = alg[k]
            e["achieved_gbs"] = alg[k] / (ms * 1e-3) / 1e9
            e["frac"] = e["achieved_gbs"] / HBM_PEAK_GBS
        if not pmc_entry(e, k, traffic, ms):
            traffic.pop(k, None)  # out of traffic_per_step too
        table[k] = e
    dom = max(kernel_ms, key=lambda k: kernel_ms[k] * launches[k])
    ms_per_step = elapsed / args.steps * 1e3
    path_bytes = 24.0 * n
    path_gbs = path_bytes / (ms_per_step * 1e-3) / 1e9
    return {
        "value": n * world * args.steps / elapsed,
        "ms_per_step": ms_per_step,
        "config": {"workload": f"dataset histograms (compute_dataset_histograms, all seven) over {n:.3g} rows "
                               f"per GPU, {U:.3g} privacy ids, {P:.3g} partitions, fp64 values",
                   "rows_per_gpu": n, "privacy_ids": U, "partitions": P,
                   "parallelism": f"rows sharded by privacy_id over {world} GPU(s)"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": table[dom].get("achieved_gbs"),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": table[dom].get("frac"),
                     "traffic": traffic.get(dom), "traffic_source": traffic_src, "traffic_refused": traffic_refused,
                     "bytes_per_launch": alg.get(dom), "avg_ms": kernel_ms[dom]},
        "path_roofline": {"achieved": path_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": path_gbs / HBM_PEAK_GBS, "bytes_per_step": path_bytes},
        "kernels": table, "bound_plan": None, "partitions_kept": None, "api": None, "pairs": pairs,
    }


def hist_cpu_baseline(sample_rows):
    """The NumPy oracle of compute_dataset_histograms (oracle/histograms.py,
    vectorised, one process) on a sample of the hist workload."""
    from oracle import histograms as OH
    from oracle import strong_baseline as strong
    rng = np.random.default_rng(3)
    n = sample_rows
    pid = rng.integers(0, max(1, HIST["privacy_ids"] * n // HIST["rows"]), n)
    pk = rng.integers(0, HIST["partitions"], n)
    val = np.clip(rng.normal(5.0, 3.0, n), MIN_VALUE, MAX_VALUE)
    t0 = time.perf_counter()
    OH.dataset_histograms(pid, pk, val)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "rows/s", "cores": 1, "kind": "port", "cpu_model": strong.cpu_model(),
            "sample": f"{n} rows shaped like the hist workload; oracle/histograms.py (vectorised NumPy "
                      f"restatement of computing_histograms.py) on one core, {dt:.1f} s"}


def kernel_alg_bytes(plan, n, kept_pairs, kept_rows, n_fields, stats, P=0):
    """Algorithmic bytes of each kernel of one step: every
    input it must read once plus every output it must write once.  `stats`
    (BoundWorkspace.stats): rows through the partition passes (the sieve's
    candidates) and the sieve's fix-up rows."""
    from pipelinedp_amd import _native as N
    rec1 = {N.KEYS_COMPACT: 8, N.KEYS_WIDE: 12}.get(plan.key_format, 8)        # level-1 record
    rec2 = {N.KEYS_WIDE: 12, N.KEYS_PACKED_WIDE: 12}.get(plan.key_format, 8)   # level-2 key + row
    key2 = 8 if plan.key_format == N.KEYS_PACKED64 else rec2 - 4                # what B1 streams
    pair_rec = 8 + 8 * n_fields
    cand = stats["rows_partitioned"]
    fix = stats["fixup_rows"]
    out = {}
    # level 1 reads the two key columns once and writes one record per row
    # that goes on (the tile-local form needs no histogram pass over ids)
    band = stats.get("band_rows", 0)
    # (with the side band, level 1 also writes one (id, row) entry per band row)
    out["k_sieve_l1" if plan.sieve else "k_scatter_l1"] = 16.0 * n + rec1 * cand + 8.0 * band
    out["k_scatter_l2"] = (rec1 + rec2) * cand
    # B1 streams the level-2 keys; kept rows' indices and values are
    # gathered; one record per kept pair out
    out["k_bucket_bound"] = key2 * cand + 12.0 * kept_rows + pair_rec * kept_pairs
    if plan.sieve:
        fix2 = stats.get("fixup2_rows", 0)
        if getattr(plan, "band", 0):
            # the band lists in (when some id is unresolved), the ids still
            # unresolved after them re-read from the privacy-id column
            out["k_band_scan"] = 8.0 * band if stats.get("unresolved_ids", 1) else 0.0
            out["k_sieve_rescan"] = (8.0 * n + 8.0 * fix2) if stats.get("unresolved2_ids", 1) else 0.0
            out["k_bucket_fix2"] = key2 * fix2
        else:
            # privacy ids in, (id, row) per fix-up row out; with no unresolved
            # privacy id the rescan exits before reading anything
            out["k_sieve_rescan"] = (8.0 * n + 8.0 * fix) if stats.get("unresolved_ids", 1) else 0.0
        out["k_fix_scatter"] = (8.0 + 8.0 + rec2) * (fix + fix2)  # list in, partition gathered, record out
        out["k_bucket_fix"] = key2 * fix
    out["k_range_reduce"] = 2.0 * pair_rec * kept_pairs
    # two-level merge (P > 2^21): the coarse records' keys counted per fine
    # range, the records moved once into fine-range order, then read once
    # and summed into the accumulators (written once)
    acc_bytes = 8.0 * (2 + n_fields) * P
    out["k_split_count"] = 8.0 * kept_pairs
    out["k_split_scatter"] = 2.0 * pair_rec * kept_pairs
    out["k_fine_reduce"] = pair_rec * kept_pairs + acc_bytes
    out["k_select"] = acc_bytes  # selection reads every partition's accumulators
    return out


def api_timing(args, workload, pid, pk, value, U, P, ws):
    """The same aggregate through the public API: DPEngine.aggregate over a
    device-resident ColumnTable on ColumnarBackend, + compute_budgets() + the
    materialised result (graph recognition, parameter/budget plumbing, key
    checks, output columns included), timed like the steps."""
    import torch
    import pipelinedp_amd as pdp
    from pipelinedp_amd import columnar_backend as CB
    w = C3 if workload == "c3" else C2
    table = pdp.ColumnTable({"pid": pid, "pk": pk, "v": value}, n_privacy_ids=U, n_partitions=P)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.MEAN],
                                 noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=w["l0"],
                                 max_contributions_per_partition=w["linf"], min_value=MIN_VALUE,
                                 max_value=MAX_VALUE)
    ext = pdp.DataExtractors(privacy_id_extractor=pdp.ColumnExtractor("pid"),
                             partition_extractor=pdp.ColumnExtractor("pk"),
                             value_extractor=pdp.ColumnExtractor("v"))

    def api_step():
        acc = pdp.NaiveBudgetAccountant(total_epsilon=EPS, total_delta=DELTA)
        sink = pdp.DPEngine(acc, CB.ColumnarBackend(workspace=ws)).aggregate(table, params, ext)
        acc.compute_budgets()
        return len(sink.collect())

    for _ in range(max(1, args.warmup)):
        api_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kept = 0
    for _ in range(args.steps):
        kept = api_step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    return {"ms_per_call": ms, "rows_per_s": len(pk) / (ms * 1e-3), "partitions_out": kept,
            "what": "pipelinedp_amd.DPEngine.aggregate(ColumnTable of device tensors, COUNT+SUM+MEAN) on "
                    "ColumnarBackend + compute_budgets() + collect() (AggregateResult columns on the host)"}


def run_workload(args, workload, world, rank, device, pmc_file):
    import torch
    import torch.distributed as dist
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import executor as X
    from pipelinedp_amd import parallel
    share = args.share_of if (workload == "c3" and world == 1 and args.share_of > 1) else 1
    if workload == "c3":
        total = (args.rows or C3["rows"]) // share
        n = total // world
        U = (args.privacy_ids or C3["privacy_ids"]) // share // world
        P = C3["partitions"]
        bounding, selection, ops = build_plan(C3["l0"], C3["linf"])
        pid, pk, value = gen_c3(n, U, P, rank, world, device, 2000, args.small_ids)
    else:
        n = args.rows or C2["rows"]
        U = max(1, (C2["privacy_ids"] * n) // C2["rows"])
        P = C2["partitions"]
        bounding, selection, ops = build_plan(C2["l0"], C2["linf"])
        pid, pk, value = gen_c2(n, U, P, rank, device, 1000)
    torch.cuda.synchronize()
    # rank r holds the dataset-wide ids owned_identities(U, world, r): checked
    # once with the library's default verify (it raises on an id held by two
    # ranks); the kernels take the local codes
    verify_ms = verify_sharding(pid, world, rank, U)

    P_pad, _ = parallel.partition_slices(P, world)
    ws = X.BoundWorkspace()
    tune = tuning_of(args)
    plan = X.bound_plan(n, U, P_pad, bounding, **tune)
    acc = X.new_accumulators(P_pad, bounding, device)
    seed_base = args.seed

    def step(i):
        X.zero_accumulators(acc)  # one fill: the fields share a block
        X.bound_and_reduce(pid, pk, value, n_privacy_ids=U, n_partitions=P_pad, bounding=bounding,
                           seed=seed_base + i, row_offset=rank * n, acc=acc, workspace=ws,
                           check_keys=False, **tune)
        # RCCL reduce-scatter (identity at N=1); counts are at most the global
        # row count, so the int32 wire format needs no device read
        mine, first = parallel.exchange_accumulators(acc, int_bound=n * world)
        if share > 1:  # one rank's share: its slice of the partitions (rank 0's)
            mine = {k: (None if t is None else t[:P_pad // share]) for k, t in mine.items()}
        _, _, n_kept = X.select_and_noise(mine, selection=selection, ops=ops, n_cols=3,
                                          seed_select=seed_base ^ (i * 7919 + 1),
                                          seed_noise=seed_base ^ (i * 104729 + 2),
                                          partition_offset=first, sync_count=False)
        return n_kept  # a device count: no host round trip inside a step

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kept = 0
    for i in range(args.steps):
        kept = step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kept = int(kept)
    # key-error check of the data once (outside the timed region)
    X.bound_and_reduce(pid, pk, value, n_privacy_ids=U, n_partitions=P_pad, bounding=bounding, seed=1,
                       row_offset=rank * n, acc=acc, workspace=ws, check_keys=True, **tune)
    # per-kernel times from a second, untimed pass of the same steps: the HIP
    # events the profiler records around every launch (on its launch stream)
    # would otherwise sit inside the timed region
    N.profiler_enable(True)
    for i in range(args.steps):
        step(args.warmup + args.steps + i)
    kernels = N.profiler_report()
    N.profiler_enable(False)
    kept_pairs = int(acc["privacy_id_count"].sum().item())  # last step, this rank
    kept_rows = int(acc["count"].sum().item())
    stats = ws.stats()
    # run-to-run spread: up to 10 more steps, each timed on its own (synced),
    # outside the timed region (their seeds differ, as the timed steps' do)
    samples = []
    for i in range(min(args.steps, 10)):
        torch.cuda.synchronize()
        ts = time.perf_counter()
        step(args.warmup + 2 * args.steps + i)
        torch.cuda.synchronize()
        samples.append((time.perf_counter() - ts) * 1e3)
    # the plan the timed steps ran: the auto plan, unless the library's plan
    # feedback (executor.py) turned the sieve off for these columns
    feedback = X.plan_feedback_state(pid, pk, n_privacy_ids=U, n_partitions=P_pad, bounding=bounding,
                                     row_offset=rank * n)
    if feedback and feedback["unsieved"] and not args.sieve:
        plan = X.bound_plan(n, U, P_pad, bounding, **dict(tune, sieve=-1))
    api = api_timing(args, workload, pid, pk, value, U, P, ws) if (world == 1 and args.api) else None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    del pid, pk, value, acc, ws

    kernel_ms = {k: v[0] / v[1] for k, v in kernels.items()}  # average ms per launch
    launches = {k: v[1] / args.steps for k, v in kernels.items()}
    ms_per_step = elapsed / args.steps * 1e3
    total_rows = n * world * args.steps
    # a variant's counters are not the base workload's: --small-ids names its own
    traffic, traffic_src, traffic_refused = load_pmc(
        pmc_file, f"{workload}-small{args.small_ids:g}" if args.small_ids else workload, n, world, stats)
    alg = kernel_alg_bytes(plan, n, kept_pairs, kept_rows, 2, stats)
    table = {}
    for k, ms in kernel_ms.items():
        e = {"ms": ms, "launches_per_step": launches[k]}
        if k in alg:
            e["alg_bytes"] = alg[k]
            e["achieved_gbs"] = alg[k] / (ms * 1e-3) / 1e9
            e["frac"] = e["achieved_gbs"] / HBM_PEAK_GBS
        if not pmc_entry(e, k, traffic, ms):
            traffic.pop(k, None)  # out of traffic_per_step too
        table[k] = e
    dom = max(kernel_ms, key=lambda k: kernel_ms[k] * launches[k])
    path_bytes = 24.0 * n + kept * (8 + 8 * 3 + 8 * 3)  # SURVEY §8(d) compulsory bytes
    path_gbs = path_bytes / (ms_per_step * 1e-3) / 1e9
    w = C3 if workload == "c3" else C2
    return {
        "value": total_rows / elapsed,
        "ms_per_step": ms_per_step,
        "workload_name": workload,
        "config": {
            "workload": (f"{workload.upper()}: DPEngine.aggregate COUNT+SUM+MEAN, Laplace, private partitions "
                         f"(truncated geometric), L0={w['l0']}, Linf={w['linf']}, "
                         + (f"{n * world:.3g} rows in total, Zipf({C3['zipf']}) partition keys"
                            if workload == "c3" else f"{n:.3g} rows per GPU, uniform keys")
                         + (f", {args.small_ids:g} of the privacy ids with 1-3 rows"
                            if workload == "c3" and args.small_ids else "")),
            "rows_per_gpu": n, "privacy_ids_per_gpu": U, "partitions": P,
            "parallelism": (f"rows sharded by privacy_id over {world} GPU(s)" if share == 1 else
                            f"ONE RANK'S SHARE of a {share}-GPU run on one GPU: rows and privacy ids / {share}, "
                            f"selection + noise over P / {share} partitions, the reduce-scatter not included"),
        },
        "roofline": {  # dominant kernel, its OWN algorithmic bytes
            "bound": "hbm", "kernel": dom,
            "achieved": table[dom].get("achieved_gbs"), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": table[dom].get("frac"), "traffic": traffic.get(dom), "traffic_source": traffic_src,
            "traffic_refused": traffic_refused, "bytes_per_launch": alg.get(dom), "avg_ms": kernel_ms[dom],
        },
        "path_roofline": {  # the headline fraction: 24 B/row compulsory over the whole step
            "achieved": path_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": path_gbs / HBM_PEAK_GBS,
            "bytes_per_step": path_bytes,
            "traffic_per_step": sum(traffic.values()) if traffic else None,
        },
        "kernels": table,
        "bound_plan": {"algorithm": plan.algorithm, "bucket_bits": plan.bucket_bits,
                       "n_buckets": plan.n_buckets, "lds_bytes": plan.lds_bytes,
                       "key_format": {1: "wide", 2: "compact", 3: "packed", 4: "packed_wide", 5: "packed64"}.get(
                           plan.key_format, plan.key_format),
                       "sieve": plan.sieve / 65536.0, "band": plan.band / 65536.0,
                       "sieve_threads": plan.sieve_threads, "bucket_threads": plan.bucket_threads,
                       "stats": stats, "plan_feedback": feedback,
                       "placement": list(X._placement_log)},
        "seed": args.seed,
        "partitions_kept": kept, "kept_pairs": kept_pairs, "kept_rows": kept_rows,
        "api": api, "privacy_id_verify_ms": verify_ms,
        "step_ms_spread": ({"n": len(samples), "min": min(samples), "median": float(np.median(samples)),
                            "max": max(samples), "what": "steps timed one by one after the timed region"}
                           if samples else None),
    }


def main():
    args = parse()
    maybe_spawn(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo")
            dist.barrier()
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "requested": args.gpus}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.cpu_baseline_only:  # the child started below: CPU baselines as one JSON line, no GPU
        cpu = (cpu_baselines(args.workload, args.cpu_sample_rows) if args.workload in ("c3", "c2")
               else (hist_cpu_baseline(4 * args.cpu_sample_rows), None, None))
        print(json.dumps(cpu), flush=True)
        return
    import torch
    import torch.distributed as dist
    # PDP_BENCH_BACKEND=gloo rehearses the multi-rank path with every rank on
    # the visible GPUs round-robin (e.g. two ranks on a one-GPU box); the
    # measured configuration is RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("PDP_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local_rank = local_rank % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local_rank)

    if args.workload in ("c4", "c5"):
        r = run_api_workload(args, args.workload, world, rank, device)
        r.setdefault("api", None)
    elif args.workload == "hist":
        r = run_hist_workload(args, world, rank, device)
    else:
        r = run_workload(args, args.workload, world, rank, device, PMC_SUMMARY[args.workload])
    result = {
        "metric": "input rows/sec aggregated (whole node) + achieved HBM GB/s vs peak",
        "value": r["value"],
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong" if args.workload == "c3" else "weak",
        "workload_name": args.workload,
        "vs_baseline": None,
        "dtype": "f64",
        "data": {"c3": "synthetic (uniform pid, Zipf(1.1) pk, U(0,10) values), generated on device",
                 "c2": "synthetic (uniform pid/pk, N(5,3) clipped values), generated on device",
                 "c4": "synthetic (uniform pid/pk, U(0,10) values), generated on device",
                 "c5": "synthetic (Pareto(1.5) rows per pid, Zipf(1.1) pk, lognormal(1,1) values clipped to "
                       "[0,20]), generated on device",
                 "hist": "synthetic (uniform pid/pk, N(5,3) clipped values), generated on device",
                 }[args.workload],
        "config": r["config"],
        "roofline": r["roofline"],
        "path_roofline": r["path_roofline"],
        "kernels": r["kernels"],
        "bound_plan": r["bound_plan"],
        "seed": r.get("seed"),
        "partitions_kept": r["partitions_kept"],
        "kept_pairs": r.get("kept_pairs"), "kept_rows": r.get("kept_rows"),
        "privacy_id_verify": r.get("privacy_id_verify_ms"),
        "step_ms_spread": r.get("step_ms_spread"),
        "api": r["api"],
        "cpu_baseline": None,
        "cpu_baseline_strong": None,
        "cpu_baseline_c1": None,
    }
    if world == 1 and args.workload == "c3" and not args.no_secondary and not args.rows and not args.share_of:
        torch.cuda.empty_cache()
        s = run_workload(args, "c2", 1, 0, device, PMC_SUMMARY["c2"])
        result["secondary"] = {k: s[k] for k in ("value", "ms_per_step", "config", "roofline",
                                                 "path_roofline", "kernels", "bound_plan", "api")}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload in ("c3", "c2", "hist"):
        # after the GPU measurements, in a child process (no GPU state there):
        # its ~30 s of host work can neither precede nor overlap the timed steps
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--workload",
                              args.workload, "--cpu-sample-rows", str(args.cpu_sample_rows)],
                             capture_output=True, text=True, check=True)
        cpu = json.loads([l for l in out.stdout.splitlines() if l.startswith("[")][-1])
    if cpu:
        result["cpu_baseline"], result["cpu_baseline_strong"] = cpu[0], cpu[1]
        result["cpu_baseline_c1"] = cpu[2] if len(cpu) > 2 else None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
