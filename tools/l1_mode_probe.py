"""Level 1's per-process slow mode (DESIGN.md §3, C3 rounds 4-6): in ONE
process, k_sieve_l1 timed (library profiler, level 1 alone via the test
hook) over three workspaces allocated side by side and over a copy of the
key columns, alternating.  A per-allocation effect shows as workspaces of
different speed in one process; a per-process one as equal times.
Usage: python tools/l1_mode_probe.py [--steps K]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PIPELINEDP_AMD_TEST_HOOKS"] = "1"
os.environ["PIPELINEDP_AMD_STOP_AFTER_L1"] = "1"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
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
    nbytes = ctypes.c_uint64(0)
    lib = N.lib()
    N.check(lib.pdp_bound_workspace_bytes(ctypes.byref(cfg), ctypes.byref(nbytes)), "workspace")
    wss = [torch.empty(nbytes.value, dtype=torch.uint8, device=dev) for _ in range(3)]
    cols = {"orig": (pid, pk)}

    def time_l1(ws, p, k):
        def run():
            N.check(lib.pdp_bound_contributions(ctypes.byref(cfg), X._ptr(p), X._ptr(k), X._ptr(val), None,
                                                X._ptr(ws), ws.numel(), X._stream(None)), "bound")
        run()
        torch.cuda.synchronize()
        N.profiler_enable(True)
        for _ in range(a.steps):
            run()
        rep = N.profiler_report()
        N.profiler_enable(False)
        return round(rep["k_sieve_l1"][0] / rep["k_sieve_l1"][1], 4)

    out = []
    for rnd in range(2):
        for i, ws in enumerate(wss):
            out.append({"round": rnd, "ws": i, "cols": "orig", "l1_ms": time_l1(ws, pid, pk)})
            print(json.dumps(out[-1]), flush=True)
        if rnd == 0:  # a second copy of the key columns
            cols["copy"] = (pid.clone(), pk.clone())
            torch.cuda.synchronize()
        out.append({"round": rnd, "ws": 0, "cols": "copy", "l1_ms": time_l1(wss[0], *cols["copy"])})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
