"""k_sieve_l1 at C3 against the relative placement of the two key columns:
pid and pk as views of ONE allocation, pk starting `gap` bytes after pid's
end, all in one process (so per-process placement cannot differ).
Usage: python tools/layout_probe.py  (prints one line per gap and repeat)"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import bench  # noqa: E402
from pipelinedp_amd import _native as N  # noqa: E402
from pipelinedp_amd import executor as X  # noqa: E402

dev = torch.device("cuda:0")
n, U, P = bench.C3["rows"], bench.C3["privacy_ids"], bench.C3["partitions"]
pid0, pk0, val = bench.gen_c3(n, U, P, 0, 1, dev, 2000)
bounding, _, _ = bench.build_plan(bench.C3["l0"], bench.C3["linf"])
ws = X.BoundWorkspace()
acc = X.new_accumulators(P, bounding, dev)
for rep in range(2):
    for gap in (0, 4096, 65536, 1 << 20, (1 << 21) + 8192, 3 << 20):
        buf = torch.empty(2 * n + gap // 8, dtype=torch.int64, device=dev)
        pid, pk = buf[:n], buf[n + gap // 8:]
        pid.copy_(pid0)
        pk.copy_(pk0)
        for i in range(3):
            X.bound_and_reduce(pid, pk, val, n_privacy_ids=U, n_partitions=P, bounding=bounding, seed=7 + i,
                               acc=acc, workspace=ws, check_keys=False)
        torch.cuda.synchronize()
        N.profiler_enable(True)
        for i in range(5):
            X.bound_and_reduce(pid, pk, val, n_privacy_ids=U, n_partitions=P, bounding=bounding, seed=17 + i,
                               acc=acc, workspace=ws, check_keys=False)
        torch.cuda.synchronize()
        k = N.profiler_report()
        N.profiler_enable(False)
        t = k["k_sieve_l1"]
        print(f"rep {rep} gap {gap:>8d} B  pid at +{pid.data_ptr() % (1 << 21):>7d} mod 2MiB  k_sieve_l1 {t[0] / t[1]:.3f} ms",
              flush=True)
        del buf, pid, pk
        torch.cuda.empty_cache()
