"""Level 1's placement effect (DESIGN.md §3 "Level 1's placement"): does the
level-1 time of one C3 workspace change when the same allocation is used
from a shifted start?  One allocation of the workspace plus SLACK bytes;
k_sieve_l1 timed (library profiler, level 1 alone via PDP_PROBE_LEVEL1) with
the workspace starting at each offset, two rounds so a stable per-offset
time shows as equal rounds.
Usage: python tools/ws_offset_probe.py [--steps K] [--allocs A]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OFFSETS_KB = [0, 4, 64, 256, 1024, 2048, 4096, 6144, 8192, 16384, 32768, 65536, 98304, 131072, 196608]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--allocs", type=int, default=2)
    a = ap.parse_args()
    import torch
    import bench
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import executor as X
    dev = torch.device("cuda:0")
    n, U, P = bench.C3["rows"], bench.C3["privacy_ids"], bench.C3["partitions"]
    pid, pk, val = bench.gen_c3(n, U, P, 0, 1, dev, 20261017)
    torch.cuda.synchronize()
    spec = X.BoundingSpec(l0=2, linf=1, value_kind=N.VALUE_F64, flags=N.ACC_SUM | N.ACC_NSUM, min_value=0.0,
                          max_value=bench.MAX_VALUE, middle=bench.MAX_VALUE / 2)
    cfg = X.bound_config(n, U, P, spec, 77)
    cfg.flags |= N.PROBE_LEVEL1
    nbytes = ctypes.c_uint64(0)
    lib = N.lib()
    N.check(lib.pdp_bound_workspace_bytes(ctypes.byref(cfg), ctypes.byref(nbytes)), "workspace")
    slack = (OFFSETS_KB[-1] + 4) * 1024
    bufs = [torch.empty(nbytes.value + slack, dtype=torch.uint8, device=dev) for _ in range(a.allocs)]

    def time_l1(buf, off):
        ws = buf[off:off + nbytes.value]

        def run():
            N.check(lib.pdp_bound_contributions(ctypes.byref(cfg), X._ptr(pid), X._ptr(pk), X._ptr(val), None,
                                                X._ptr(ws), ws.numel(), X._stream(None)), "bound")
        run()
        torch.cuda.synchronize()
        N.profiler_enable(True)
        for _ in range(a.steps):
            run()
        rep = N.profiler_report()
        N.profiler_enable(False)
        return round(rep["k_sieve_l1"][0] / rep["k_sieve_l1"][1], 4)

    for i, buf in enumerate(bufs):
        for kb in OFFSETS_KB:
            t = [time_l1(buf, kb * 1024) for _ in range(2)]
            print(json.dumps({"alloc": i, "offset_kb": kb, "l1_ms": t}), flush=True)


if __name__ == "__main__":
    main()
