#!/usr/bin/env python3
"""Benchmark of the DPEngine.aggregate hot path on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1], SURVEY §8(d) "C2"): per GPU N = 1e8 rows,
P = 1e5 partitions (pk uniform), U = 1e6 privacy ids (pid uniform, ~100 rows
each), value fp64 ~ N(5, 3) clipped to [0, 10]; COUNT + SUM + MEAN, Laplace,
max_partitions_contributed = 8, max_contributions_per_partition = 2,
min/max value 0/10, eps = 1, delta = 1e-6, private partitions (truncated
geometric).  Weak scaling: every rank holds its own 1e8 rows of its own 1e6
privacy ids (rows sharded by privacy id), partitions are global; the one
cross-GPU step is an RCCL reduce-scatter of the per-partition accumulators,
after which each rank selects and noises its slice of partitions.

A step = one full aggregate over the resident batch: contribution bounding
(L0 + Linf sampling), per-partition reduction, [reduce-scatter], partition
selection, compaction and noisy metrics, ending with the kept-partition count
on the host.  Inputs are resident in HBM before timing starts.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1: launched by torch.distributed.run, one rank per GPU)
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

# HBM bytes per launch from rocprofv3 PMC passes over this same bench command
# (tools/gpu_pmc.sh -> tools/pmc_summary.py: 2 x FETCH_SIZE for the gfx950
# wide-load under-count + WRITE_SIZE, MI355X_MICROARCH.md "HBM").  Valid for the
# default C2 shape only; None otherwise.
PMC_SUMMARY = os.path.join(HERE, "profiles", "r01", "v18_pmc.json")


def pmc_traffic(n_rows):
    if n_rows != ROWS_PER_GPU or not os.path.exists(PMC_SUMMARY):
        return {}
    with open(PMC_SUMMARY) as f:
        kernels = json.load(f)["kernels"]
    return {k: v["hbm_bytes"] for k, v in kernels.items() if "hbm_bytes" in v}

# workload constants (C2)
ROWS_PER_GPU = 100_000_000
PRIVACY_IDS_PER_GPU = 1_000_000
PARTITIONS = 100_000
L0, LINF = 8, 2
MIN_VALUE, MAX_VALUE = 0.0, 10.0
EPS, DELTA = 1.0, 1e-6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=ROWS_PER_GPU, help="rows per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-rows", type=int, default=2_000_000)
    ap.add_argument("--key-format", type=int, default=0, help="PDP_KEYS_* (0 auto, 1 wide, 2 compact)")
    ap.add_argument("--workload", choices=("c2", "c3"), default="c2",
                    help="c2 (default, BASELINE configs[1]); c3: configs[2], 1e9 rows in total, "
                         "Zipf(1.1) partition keys over 1e6 partitions, 1e7 privacy ids, L0=2, "
                         "Linf=1, values U(0, 10), strong scaling over the GPUs")
    return ap.parse_args()


# C3: N = 1e9 in total, pk Zipf(a=1.1) over P = 1e6, U = 1e7
C3_ROWS, C3_PRIVACY_IDS, C3_PARTITIONS, C3_L0, C3_LINF, C3_ZIPF = 1_000_000_000, 10_000_000, 1_000_000, 2, 1, 1.1


def build_plan(l0=L0, linf=LINF):
    """Noise / selection parameters exactly as DPEngine + NaiveBudgetAccountant
    derive them for this AggregateParams (3 mechanisms of weight 1: MEAN's
    count and normalized-sum Laplace mechanisms + the GENERIC selection)."""
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import dp_computations as dpc
    from pipelinedp_amd import executor as X
    eps_each = EPS / 3
    mid = dpc.compute_middle(MIN_VALUE, MAX_VALUE)
    b_count = dpc.laplace_diversity(eps_each, l0 * linf)
    b_nsum = dpc.laplace_diversity(eps_each, l0 * (MAX_VALUE - MIN_VALUE) / 2 * linf)
    bounding = X.BoundingSpec(l0=l0, linf=linf, value_kind=N.VALUE_F64, flags=N.ACC_NSUM,
                              min_value=MIN_VALUE, max_value=MAX_VALUE, middle=mid)
    selection = X.SelectionSpec(strategy=N.SELECT_TRUNCATED_GEOMETRIC,
                                keep_prob=dpc.truncated_geometric_keep_table(eps_each, DELTA, l0))
    ops = [X.MetricOpSpec(kind=N.OP_MEAN, noise_kind=N.NOISE_LAPLACE, out_col=(0, 1, 2),
                          scale=(b_count, b_nsum), middle=mid)]
    return bounding, selection, ops


def cpu_baseline(sample_rows):
    """Row-wise restatement of LocalBackend DPEngine.aggregate (the reference's
    single-threaded CPU path) on a bounded sample of the same workload."""
    from oracle import local_backend_port as port
    rng = np.random.default_rng(1)
    U = max(1, sample_rows // 100)
    pid = rng.integers(0, U, sample_rows)
    pk = rng.integers(0, PARTITIONS, sample_rows)
    val = np.clip(rng.normal(5.0, 3.0, sample_rows), MIN_VALUE, MAX_VALUE)
    rows = list(zip(pid.tolist(), pk.tolist(), val.tolist()))
    t0 = time.perf_counter()
    out = port.aggregate_count_sum_mean(rows, l0=L0, linf=LINF, min_value=MIN_VALUE,
                                        max_value=MAX_VALUE, eps=EPS, delta=DELTA)
    dt = time.perf_counter() - t0
    return {"value": sample_rows / dt, "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": f"{sample_rows} rows of the same workload (U={U}, P={PARTITIONS}), "
                      f"oracle/local_backend_port.py row-wise LocalBackend restatement, "
                      f"{dt:.1f} s, {len(out)} partitions kept"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import executor as X
    from pipelinedp_amd import parallel

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    device = torch.device("cuda", local_rank)

    c3 = args.workload == "c3"
    g = torch.Generator(device=device)
    g.manual_seed(1000 + rank)
    if c3:  # strong scaling: 1e9 rows and 1e7 privacy ids in total, sharded by privacy id
        n = C3_ROWS // world
        U = C3_PRIVACY_IDS // world
        P = C3_PARTITIONS
        bounding, selection, ops = build_plan(C3_L0, C3_LINF)
        pid = torch.randint(0, U, (n,), generator=g, device=device, dtype=torch.int64)
        w = torch.arange(1, P + 1, device=device, dtype=torch.float64).pow_(-C3_ZIPF)
        cdf = torch.cumsum(w, 0)
        cdf /= cdf[-1].clone()
        pk = torch.empty(n, device=device, dtype=torch.int64)
        for c0 in range(0, n, 1 << 27):  # bounded temporaries
            c1 = min(n, c0 + (1 << 27))
            u = torch.rand(c1 - c0, generator=g, device=device, dtype=torch.float64)
            pk[c0:c1] = torch.searchsorted(cdf, u).clamp_(max=P - 1)
        value = torch.rand(n, generator=g, device=device, dtype=torch.float64) * MAX_VALUE
        del w, cdf
    else:
        n = args.rows
        U = max(1, (PRIVACY_IDS_PER_GPU * n) // ROWS_PER_GPU)
        P = PARTITIONS
        bounding, selection, ops = build_plan()
        pid = torch.randint(0, U, (n,), generator=g, device=device, dtype=torch.int64)
        pk = torch.randint(0, P, (n,), generator=g, device=device, dtype=torch.int64)
        value = (torch.randn(n, generator=g, device=device, dtype=torch.float64) * 3.0 + 5.0).clamp_(
            MIN_VALUE, MAX_VALUE)
    torch.cuda.synchronize()

    P_pad, _ = parallel.partition_slices(P, world)
    ws = X.BoundWorkspace()
    plan = X.bound_plan(n, U, P_pad, bounding, key_format=args.key_format)
    acc = X.new_accumulators(P_pad, bounding, device)
    seed_base = parallel.broadcast_seeds((int.from_bytes(os.urandom(8), "little"),))[0]

    def step(i):
        for t in acc.values():
            if t is not None:
                t.zero_()
        X.bound_and_reduce(pid, pk, value, n_privacy_ids=U, n_partitions=P_pad, bounding=bounding,
                           seed=seed_base + i, row_offset=rank * n, acc=acc, workspace=ws,
                           check_keys=False, key_format=args.key_format)
        mine, first = parallel.exchange_accumulators(acc)  # RCCL reduce-scatter; identity at N=1
        _, _, n_kept = X.select_and_noise(mine, selection=selection, ops=ops, n_cols=3,
                                          seed_select=seed_base ^ (i * 7919 + 1),
                                          seed_noise=seed_base ^ (i * 104729 + 2),
                                          partition_offset=first)
        return n_kept

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
    # per-kernel times from a second, untimed pass of the same steps: the HIP
    # events the profiler records around every launch (on its launch stream)
    # would otherwise sit inside the timed region
    N.profiler_enable(True)
    for i in range(args.steps):
        step(args.warmup + args.steps + i)
    kernels = N.profiler_report()
    N.profiler_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kernel_ms = {k: v[0] / v[1] for k, v in kernels.items()}  # average ms per launch
    launches_per_step = {k: v[1] / args.steps for k, v in kernels.items()}
    dom = max(kernel_ms, key=lambda k: kernel_ms[k] * launches_per_step[k])
    # algorithmic bytes of the path: 24 B per input row (pid, pk,
    # value), attributed to the dominant kernel's launch
    alg_bytes = 24.0 * n
    achieved = alg_bytes / (kernel_ms[dom] * 1e-3) / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    total_rows = n * world * args.steps
    value_rows_s = total_rows / elapsed
    path_bytes = 24.0 * n + kept * (8 + 8 * 3 + 8 * 3)
    traffic = pmc_traffic(n)
    result = {
        "metric": "input rows/sec aggregated (whole node) + achieved HBM GB/s vs peak",
        "value": value_rows_s,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if c3 else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (uniform pid, Zipf(1.1) pk, U(0,10) values), generated on device" if c3 else
                 "synthetic (uniform pid/pk, N(5,3) clipped values), generated on device"),
        "config": {
            "workload": ("C3: DPEngine.aggregate COUNT+SUM+MEAN, Laplace, private partitions "
                         "(truncated geometric), L0=2, Linf=1, 1e9 rows in total" if c3 else
                         "C2: DPEngine.aggregate COUNT+SUM+MEAN, Laplace, private partitions "
                         "(truncated geometric), L0=8, Linf=2"),
            "rows_per_gpu": n, "privacy_ids_per_gpu": U, "partitions": P,
            "parallelism": f"rows sharded by privacy_id over {world} GPU(s)",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic.get(dom),
            "traffic_source": os.path.relpath(PMC_SUMMARY, HERE) if dom in traffic else None,
            "bytes_per_launch": alg_bytes,
            "avg_ms": kernel_ms[dom],
        },
        "path_roofline": {
            "achieved": path_bytes / (ms_per_step * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": path_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "bytes_per_step": path_bytes,
            "traffic_per_step": sum(traffic.values()) if traffic else None,
        },
        "kernel_ms": kernel_ms,
        "bound_plan": {"algorithm": plan.algorithm, "bucket_bits": plan.bucket_bits,
                       "n_buckets": plan.n_buckets, "lds_bytes": plan.lds_bytes,
                       "key_format": {1: "wide", 2: "compact"}.get(plan.key_format, plan.key_format)},
        "partitions_kept": kept,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not c3:
        result["cpu_baseline"] = cpu_baseline(args.cpu_sample_rows)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
