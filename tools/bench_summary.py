#!/usr/bin/env python3
"""One-screen summary of bench.py JSON lines (usage: bench_summary.py LOG [LOG ...])."""
import json
import sys


def show(tag, r):
    print(f"{tag}: {r['ms_per_step']:.3f} ms/step  {r['value']:.4g} rows/s  path frac "
          f"{r['path_roofline']['frac']:.3f}  dominant {r['roofline']['kernel']} frac "
          f"{(r['roofline']['frac'] or 0):.3f}  plan {r.get('bound_plan')}")
    ks = r.get("kernels", {})
    print("   " + "  ".join(f"{k}={v['ms']:.3f}" for k, v in ks.items() if v["ms"] * v["launches_per_step"] > 0.02))


for path in sys.argv[1:]:
    line = [l for l in open(path) if l.startswith("{")][-1]
    r = json.loads(line)
    show(path, r)
    if r.get("secondary"):
        show("secondary", r["secondary"])
    for k in ("cpu_baseline", "cpu_baseline_strong", "cpu_baseline_c1"):
        if r.get(k):
            print(f"{k}: {r[k]['value']:.4g} rows/s on {r[k]['cores']} core(s)  ({r[k]['sample'][-90:]})")
