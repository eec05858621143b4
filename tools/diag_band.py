"""Diagnostic for the sieve's side band: the first sieve test case at every
threshold, band on and off, against the oracle; prints which combinations
differ, by how much, and the workspace stats (GPU)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import columnar as O  # noqa: E402
from tests import test_gpu_sieve as T  # noqa: E402
from tests.test_gpu_kernels import _gen  # noqa: E402


def main():
    import torch
    from pipelinedp_amd import executor as X
    dev = torch.device("cuda", 0)
    case = T.CASES[0]
    spec = T._spec(case)
    U, P = case[7], 3001
    n = 2_000_000 + 12_345
    pid, pk, val = _gen(77 + spec.l0, n, U, P, spec.value_kind, skew=True)
    seed = 0xA5A5_0000_1111 + spec.l0
    want = T._want(pid, pk, val, U, P, spec, seed)
    for sieve in T.SIEVES:
        for band in (0, -1):
            ws = X.BoundWorkspace()
            got = T._run(dev, pid, pk, val, U, P, spec, seed, sieve, band=band, workspace=ws)
            d = got["privacy_id_count"].astype(np.int64) - want["privacy_id_count"].astype(np.int64)
            c = got["count"].astype(np.int64) - want["count"].astype(np.int64)
            print(f"sieve={sieve} band={band} pid_count_diff: n={np.count_nonzero(d)} sum={d.sum()} "
                  f"count_diff: n={np.count_nonzero(c)} sum={c.sum()} stats={ws.stats()}", flush=True)


if __name__ == "__main__":
    main()
