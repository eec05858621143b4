"""Level 1's placement effect (DESIGN.md §3 "Level 1's placement"): the
level-1 time of the C3 workspace by how it was allocated -- PyTorch's
caching allocator, hipMalloc, hipExtMallocWithFlags(hipDeviceMallocContiguous)
-- in one process, two rounds each.
Usage: python tools/ws_alloc_probe.py [--steps K] [--each A]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--each", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=0,
                    help="instead: ROUNDS rounds of EACH torch workspaces; all but the fastest freed "
                         "(and the cache emptied) between rounds -- do new allocations get new speeds?")
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
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]

    def time_l1(ptr):
        def run():
            N.check(lib.pdp_bound_contributions(ctypes.byref(cfg), X._ptr(pid), X._ptr(pk), X._ptr(val), None,
                                                ptr, nbytes.value, X._stream(None)), "bound")
        run()
        torch.cuda.synchronize()
        N.profiler_enable(True)
        for _ in range(a.steps):
            run()
        rep = N.profiler_report()
        N.profiler_enable(False)
        return round(rep["k_sieve_l1"][0] / rep["k_sieve_l1"][1], 4)

    if a.rounds:
        best = None
        for rnd in range(a.rounds):
            cands = [] if best is None else [best]
            while len(cands) < a.each:
                cands.append(torch.empty(nbytes.value, dtype=torch.uint8, device=dev))
            ts = [time_l1(ctypes.c_void_p(t.data_ptr())) for t in cands]
            print(json.dumps({"round": rnd, "l1_ms": ts}), flush=True)
            best = cands[min(range(len(ts)), key=ts.__getitem__)]
            del cands
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        return
    held = []
    for kind in ("torch", "hipMalloc", "contiguous"):
        for i in range(a.each):
            p = ctypes.c_void_p()
            if kind == "torch":
                t = torch.empty(nbytes.value, dtype=torch.uint8, device=dev)
                held.append(t)
                p = ctypes.c_void_p(t.data_ptr())
                rc = 0
            elif kind == "hipMalloc":
                rc = hip.hipMalloc(ctypes.byref(p), nbytes.value)
            else:
                rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes.value, HIP_DEVICE_MALLOC_CONTIGUOUS)
            if rc != 0:
                print(json.dumps({"kind": kind, "i": i, "error": rc}), flush=True)
                continue
            ts = [time_l1(p) for _ in range(2)]
            print(json.dumps({"kind": kind, "i": i, "l1_ms": ts}), flush=True)
            if kind != "torch":
                held.append(p)
    torch.cuda.synchronize()
    for p in held:
        if isinstance(p, ctypes.c_void_p):
            hip.hipFree(p)


if __name__ == "__main__":
    main()
