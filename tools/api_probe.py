#!/usr/bin/env python3
"""Where the public API's per-call time goes beyond the timed kernel path
(VERDICT r05 #5): DPEngine.aggregate over a device ColumnTable on
ColumnarBackend, C2- or C3-shaped (bench.py's generators), with host
timestamps at the stage boundaries and a cProfile of 10 calls.
Usage: python tools/api_probe.py [c2|c3]"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    import pipelinedp_amd as pdp
    from pipelinedp_amd import columnar_backend as CB
    from pipelinedp_amd import executor as X
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    device = torch.device("cuda", 0)
    if wl == "c3":
        w = bench.C3
        n, U, P = w["rows"], w["privacy_ids"], w["partitions"]
        pid, pk, value = bench.gen_c3(n, U, P, 0, 1, device, 2000)
    else:
        w = bench.C2
        n, U, P = w["rows"], w["privacy_ids"], w["partitions"]
        pid, pk, value = bench.gen_c2(n, U, P, 0, device, 1000)
    torch.cuda.synchronize()
    ws = X.BoundWorkspace()
    table = pdp.ColumnTable({"pid": pid, "pk": pk, "v": value}, n_privacy_ids=U, n_partitions=P)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.MEAN],
                                 noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=w["l0"],
                                 max_contributions_per_partition=w["linf"], min_value=bench.MIN_VALUE,
                                 max_value=bench.MAX_VALUE)
    ext = pdp.DataExtractors(privacy_id_extractor=pdp.ColumnExtractor("pid"),
                             partition_extractor=pdp.ColumnExtractor("pk"),
                             value_extractor=pdp.ColumnExtractor("v"))
    marks = []
    orig_b, orig_s = X.bound_and_reduce, X.select_and_noise

    def bound(*a, **k):
        marks.append(("bound_in", time.perf_counter()))
        r = orig_b(*a, **k)
        marks.append(("bound_out", time.perf_counter()))
        return r

    def select(*a, **k):
        marks.append(("select_in", time.perf_counter()))
        r = orig_s(*a, **k)
        marks.append(("select_out", time.perf_counter()))
        return r

    X.bound_and_reduce, X.select_and_noise = bound, select

    def step():
        marks.append(("start", time.perf_counter()))
        acc = pdp.NaiveBudgetAccountant(total_epsilon=bench.EPS, total_delta=bench.DELTA)
        sink = pdp.DPEngine(acc, CB.ColumnarBackend(workspace=ws)).aggregate(table, params, ext)
        acc.compute_budgets()
        marks.append(("budgets", time.perf_counter()))
        k = len(sink.collect())
        marks.append(("end", time.perf_counter()))
        return k

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    marks.clear()
    steps = 20
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"{wl}: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms per API call")
    # mean gap between consecutive marks, per (from, to) label pair
    gaps = {}
    for (a, ta), (b, tb) in zip(marks, marks[1:]):
        if a == "end":
            continue
        gaps.setdefault(f"{a}->{b}", []).append((tb - ta) * 1e3)
    for k, v in gaps.items():
        print(f"  {k:24s} {sum(v) / len(v):.3f} ms")
    X.bound_and_reduce, X.select_and_noise = orig_b, orig_s
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        step()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
