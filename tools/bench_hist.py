"""Throughput of compute_dataset_histograms' device pass (csrc/pdp_hist.hip,
SURVEY §8(f) rank 4) on C2's shape: 1e8 rows, 1e6 privacy ids, 1e5
partitions, fp64 values, inputs resident in HBM.  One step = one
pdp_dataset_histograms call (all seven histograms, bins left on the device).

Prints one JSON line: rows/s, per-kernel HIP-event times, the roofline of the
dominant kernel (algorithmic bytes: 24 B/row of pid + pk + value for k_h_rows,
the 32-byte pair-table slots for the table scans)
and a CPU baseline: the NumPy oracle (oracle/histograms.py, vectorised, one
process) on a 4e6-row sample of the same workload.

Usage: python tools/bench_hist.py [--steps K] [--warmup W] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ROWS, PIDS, PARTS = 100_000_000, 1_000_000, 100_000
PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=ROWS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import executor as X

    d = torch.device("cuda", 0)
    g = torch.Generator(device=d).manual_seed(1)
    n = args.rows
    pid = torch.randint(0, PIDS, (n,), device=d, generator=g)
    pk = torch.randint(0, PARTS, (n,), device=d, generator=g)
    val = (torch.randn(n, device=d, generator=g, dtype=torch.float64) * 3 + 5).clamp_(0, 10)
    ws = X.BoundWorkspace()
    for _ in range(args.warmup):
        X.dataset_histograms(pid, pk, val, n_privacy_ids=PIDS, n_partitions=PARTS, workspace=ws)
    torch.cuda.synchronize()
    N.profiler_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        X.dataset_histograms(pid, pk, val, n_privacy_ids=PIDS, n_partitions=PARTS, workspace=ws)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    kernels = N.profiler_report()
    N.profiler_enable(False)
    kernel_ms = {k: v[0] / v[1] for k, v in kernels.items()}
    dom = max(kernel_ms, key=kernel_ms.get)
    # algorithmic bytes per launch: k_h_rows streams pid + pk + value (24 B/row);
    # k_h_pairs / k_h_float scan the pair table (1.5 slots of 32 B per row)
    cap = max(1024, ((n + n // 2) + 255) // 256 * 256)
    per_kernel_bytes = {"k_h_rows": 24.0 * n, "k_h_pairs": 32.0 * cap, "k_h_float": 32.0 * cap}
    dom_bytes = per_kernel_bytes.get(dom)
    # PMC-measured HBM bytes per launch (tools/gpu_hist_pmc.sh: 2 x FETCH_SIZE + WRITE_SIZE)
    pmc_path = os.path.join(ROOT, "profiles", "r01", "h6_pmc.json")
    traffic = None
    if os.path.exists(pmc_path) and n == ROWS:
        with open(pmc_path) as f:
            traffic = json.load(f)["kernels"].get(dom, {}).get("hbm_bytes")
    out = {
        "metric": "dataset histogram input rows/sec (compute_dataset_histograms device pass)",
        "value": n / dt, "unit": "rows/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt * 1e3, "higher_is_better": True, "dtype": "f64", "data": "synthetic, generated on device",
        "config": {"workload": "C2 shape: uniform pid/pk, N(5,3) clipped values", "rows": n,
                   "privacy_ids": PIDS, "partitions": PARTS},
        "kernel_ms": kernel_ms,
        "roofline": {"bound": "hbm", "kernel": dom,
                     "achieved": dom_bytes / (kernel_ms[dom] * 1e-3) / 1e9 if dom_bytes else None,
                     "peak": PEAK_GBS, "unit": "GB/s",
                     "frac": dom_bytes / (kernel_ms[dom] * 1e-3) / 1e9 / PEAK_GBS if dom_bytes else None,
                     "bytes_per_launch": dom_bytes, "traffic": traffic,
                     "traffic_source": "profiles/r01/h6_pmc.json" if traffic else None},
        "path_roofline": {"achieved": 24.0 * n / dt / 1e9, "peak": PEAK_GBS, "unit": "GB/s",
                          "frac": 24.0 * n / dt / 1e9 / PEAK_GBS},
    }
    if not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        from oracle import histograms as OH
        m = 4_000_000
        rng = np.random.default_rng(1)
        p, k = rng.integers(0, PIDS // 25, m), rng.integers(0, PARTS, m)
        v = np.clip(rng.normal(5, 3, m), 0, 10)
        t0 = time.perf_counter()
        OH.dataset_histograms(p, k, v)
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": m / cdt, "unit": "rows/s", "cores": 1, "kind": "port",
                               "sample": f"{m} rows (U={PIDS // 25}, P={PARTS}), oracle/histograms.py "
                                         f"(vectorised NumPy restatement), {cdt:.1f} s"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
