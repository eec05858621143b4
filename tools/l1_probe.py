"""Level 1 alone (test hook PIPELINEDP_AMD_STOP_AFTER_L1): C3's k_sieve_l1 timed by
the library profiler, for A/B builds (the round-5 PDP_L1_ABL ablations gave wrong results by design:
nothing downstream runs).  Library from PIPELINEDP_AMD_LIB.  Prints one JSON line.
Usage: python tools/l1_probe.py [--rows N] [--steps K] [--tag T]"""
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
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import torch
    import bench
    from pipelinedp_amd import _native as N
    from pipelinedp_amd import executor as X
    dev = torch.device("cuda:0")
    U, P = bench.C3["privacy_ids"], bench.C3["partitions"]
    pid, pk, val = bench.gen_c3(a.rows, U, P, 0, 1, dev, 20261017)
    spec = X.BoundingSpec(l0=2, linf=1, value_kind=N.VALUE_F64, flags=N.ACC_SUM | N.ACC_NSUM, min_value=0.0,
                          max_value=bench.MAX_VALUE, middle=bench.MAX_VALUE / 2)
    cfg = X.bound_config(a.rows, U, P, spec, 77)
    nbytes = ctypes.c_uint64(0)
    lib = N.lib()
    N.check(lib.pdp_bound_workspace_bytes(ctypes.byref(cfg), ctypes.byref(nbytes)), "workspace")
    ws = torch.empty(nbytes.value, dtype=torch.uint8, device=dev)

    def run():
        N.check(lib.pdp_bound_contributions(ctypes.byref(cfg), X._ptr(pid), X._ptr(pk), X._ptr(val), None,
                                            X._ptr(ws), ws.numel(), X._stream(None)), "bound")
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    N.profiler_enable(True)
    for _ in range(a.steps):
        run()
    rep = N.profiler_report()
    N.profiler_enable(False)
    ms = {k: v[0] / v[1] for k, v in rep.items()}
    print(json.dumps({"tag": a.tag, "lib": os.path.basename(os.environ.get("PIPELINEDP_AMD_LIB", "")),
                      "k_sieve_l1_ms": round(ms.get("k_sieve_l1", -1), 4), "kernels": {k: round(v, 4) for k, v in ms.items()}}))


if __name__ == "__main__":
    main()
