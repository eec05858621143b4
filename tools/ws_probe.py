"""k_sieve_l1 at C3 in ONE process against fresh allocations: a new bounding
workspace (and, second, new copies of the key columns) each round, the
caching allocator emptied in between -- does the per-process level-1 mode
follow the workspace's or the columns' placement?"""
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
pid, pk, val = bench.gen_c3(n, U, P, 0, 1, dev, 2000)
bounding, _, _ = bench.build_plan(bench.C3["l0"], bench.C3["linf"])
acc = X.new_accumulators(P, bounding, dev)


def l1_ms(pid, pk, ws):
    for i in range(3):
        X.bound_and_reduce(pid, pk, val, n_privacy_ids=U, n_partitions=P, bounding=bounding, seed=7 + i, acc=acc,
                           workspace=ws, check_keys=False)
    torch.cuda.synchronize()
    N.profiler_enable(True)
    for i in range(5):
        X.bound_and_reduce(pid, pk, val, n_privacy_ids=U, n_partitions=P, bounding=bounding, seed=17 + i, acc=acc,
                           workspace=ws, check_keys=False)
    torch.cuda.synchronize()
    k = N.profiler_report()
    N.profiler_enable(False)
    return k["k_sieve_l1"][0] / k["k_sieve_l1"][1]


class AlignedWorkspace(X.BoundWorkspace):
    """the workspace as a view starting on a 1 GiB virtual-address boundary"""

    def get(self, nbytes, device):
        if self.buf is None or self.buf.numel() < nbytes:
            self.raw = torch.empty(int(nbytes) + (1 << 30), dtype=torch.uint8, device=device)
            off = (-self.raw.data_ptr()) % (1 << 30)
            self.buf = self.raw[off:off + int(nbytes)]
        return self.buf


print(f"pid at {pid.data_ptr() % (1 << 30):#x} mod 1 GiB, pk at {pk.data_ptr() % (1 << 30):#x}", flush=True)
for r in range(4):
    ws = X.BoundWorkspace() if r < 2 else AlignedWorkspace()
    t = l1_ms(pid, pk, ws)
    print(f"fresh workspace {r} ({type(ws).__name__}) at {ws.buf.data_ptr() % (1 << 30):#x} mod 1 GiB "
          f"({ws.buf.data_ptr() % (1 << 21):#x} mod 2 MiB): k_sieve_l1 {t:.3f} ms", flush=True)
    del ws
    torch.cuda.empty_cache()
ws = X.BoundWorkspace()
for r in range(3):
    pid2, pk2 = pid.clone(), pk.clone()
    print(f"fresh columns {r}: k_sieve_l1 {l1_ms(pid2, pk2, ws):.3f} ms", flush=True)
    del pid2, pk2
    torch.cuda.empty_cache()
