#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh) into per-kernel HBM bytes.

HBM bytes per launch = 2 x FETCH_SIZE (gfx950 counts half of a wide coalesced
read, MI355X_MICROARCH.md "HBM") + WRITE_SIZE; both counters are in KiB.
Usage: python tools/pmc_summary.py <pmc dir> <out.json> [workload tag] [bench log]

With a bench log (the profiled command's own output), the summary also keeps
that run's bound_plan.stats (unresolved ids, fix-up and band rows): bench.py
joins a data-dependent kernel's bytes only when its own run has the same
work statistics (DATA_DEPENDENT there).  Per kernel it keeps the smallest and
largest launch as well, since a kernel whose work differs step to step (the
rescan: an empty launch or the whole privacy-id column) has no single figure.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tree_id import source_tree_id  # noqa: E402


def short_name(full):
    m = re.search(r"(k_[a-z0-9_]+)", full)
    if not m:
        return full[:60]
    # the histogram's bin-maximum pass is k_h_float<true> (the profiler's name)
    if m.group(1) == "k_h_float" and ("k_h_float<true>" in full or "k_h_floatILb1E" in full):
        return "k_h_float_max"
    # the tile-local partition kernels report under the pass names the
    # library's profiler (and bench.py) use
    return {"k_scatter_l1_local": "k_scatter_l1", "k_scatter_l2_local": "k_scatter_l2",
            "k_split_scatter_staged": "k_split_scatter"}.get(m.group(1), m.group(1))


def main():
    src, out = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else ""
    bench_log = sys.argv[4] if len(sys.argv) > 4 else ""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    launch_kib = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> per launch
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "pdp::" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        label, prev, fixes = {}, None, 0
        for r in rows:
            did = r.get("Dispatch_Id")
            if did not in label:
                name = short_name(r["Kernel_Name"])
                # the sieve's fix-up launches of the bucket kernel follow
                # k_fix_buckets (k_fix_scatter before round 5): the first after
                # a main launch is the library profiler's k_bucket_fix, the
                # second its k_bucket_fix2
                if name == "k_bucket_bound" and prev in ("k_fix_buckets", "k_fix_scatter"):
                    fixes += 1
                    name = "k_bucket_fix" if fixes == 1 else "k_bucket_fix2"
                elif name == "k_bucket_bound":
                    fixes = 0
                label[did] = name
                prev = name
            vals[label[did]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                launch_kib[label[did]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, d in vals.items():
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        e = {"counters_avg_per_launch": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["fetch_bytes"] = 2.0 * avg["FETCH_SIZE"] * 1024.0
            e["write_bytes"] = avg["WRITE_SIZE"] * 1024.0
            e["hbm_bytes"] = e["fetch_bytes"] + e["write_bytes"]
            # FETCH_SIZE and WRITE_SIZE come from separate passes (processes),
            # so a launch's extremes are taken per counter
            f_all, w_all = launch_kib[k]["FETCH_SIZE"], launch_kib[k]["WRITE_SIZE"]
            if f_all and w_all:
                e["launch_hbm_bytes_min"] = (2.0 * min(f_all) + min(w_all)) * 1024.0
                e["launch_hbm_bytes_max"] = (2.0 * max(f_all) + max(w_all)) * 1024.0
        kernels[k] = e
    stats = None
    if bench_log and os.path.exists(bench_log):
        lines = [l for l in open(bench_log) if l.startswith("{")]
        if lines:
            stats = (json.loads(lines[-1]).get("bound_plan") or {}).get("stats")
    json.dump({"workload": tag, "tree": source_tree_id(), "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes)",
               "stats": stats, "kernels": kernels}, open(out, "w"), indent=1, sort_keys=True)
    for k, e in sorted(kernels.items()):
        if "hbm_bytes" in e:
            print(f"{k:24s} fetch {e['fetch_bytes'] / 1e9:7.3f} GB  write {e['write_bytes'] / 1e9:7.3f} GB")


if __name__ == "__main__":
    main()
