"""GPU: pdp_owner_mismatches (the privacy_id_sharding="verify" fast path)
counts exactly the ids whose owner_of rank differs, for aligned and
unaligned columns, negative and extreme ids, and every world size."""
import numpy as np
import pytest

from pipelinedp_amd import parallel

pytestmark = pytest.mark.gpu


def _count(ids_t, world, rank):
    import ctypes
    import torch
    from pipelinedp_amd import _native as N
    out = torch.empty(1, dtype=torch.int32, device=ids_t.device)
    N.check(N.lib().pdp_owner_mismatches(ctypes.c_void_p(ids_t.data_ptr()), ids_t.numel(), world, rank,
                                         ctypes.c_void_p(out.data_ptr()), None), "pdp_owner_mismatches")
    torch.cuda.synchronize()
    return int(out.item())


def test_owner_mismatches_match_owner_of(device):
    import torch
    rng = np.random.default_rng(4)
    ids = np.concatenate([rng.integers(-2**63, 2**63 - 1, 300_001, dtype=np.int64), np.arange(-64, 64),
                          np.array([2**63 - 1, -2**63], dtype=np.int64)])
    t = torch.as_tensor(ids, device=device)
    for world in (1, 2, 5, 8):
        own = parallel.owner_of_np(ids, world)
        for rank in range(world):
            assert _count(t, world, rank) == int((own != rank).sum())
            assert _count(t[1:], world, rank) == int((own[1:] != rank).sum())  # 8-byte aligned start
    owned = t[torch.as_tensor(parallel.owner_of_np(ids, 4) == 3, device=device)]
    assert _count(owned, 4, 3) == 0 and parallel.ids_hash_owned(owned, 4, 3)
    assert _count(t[:0], 4, 0) == 0
