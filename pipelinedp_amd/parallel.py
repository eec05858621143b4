"""Multi-GPU execution: rows sharded by privacy id, one accumulator exchange.

All contribution bounding is a function of one privacy id's rows
(contribution_bounders.py:62-111), so each rank bounds and reduces its own
shard with no communication.  The only exchange is the per-partition merge
(LocalBackend.combine_accumulators_per_key, pipeline_backend.py:555-565):
the dense per-partition accumulator arrays are summed across ranks with one
reduce-scatter (RCCL over xGMI on MI355X; gloo in the CPU tests), after which
rank r owns partitions [r * slice, (r + 1) * slice) and runs selection and
noise on them locally (noise counters are global partition indices, so the
result does not depend on the number of ranks).
"""
from typing import Dict, Optional, Tuple


def world_info(group=None) -> Tuple[int, int]:
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def partition_slices(n_partitions: int, world: int) -> Tuple[int, int]:
    """(padded partition count, partitions per rank)."""
    padded = ((n_partitions + world - 1) // world) * world
    return padded, padded // world


def exchange_accumulators(acc: Dict[str, Optional["torch.Tensor"]], group=None, narrow_ints: bool = True,
                          int_bound: Optional[int] = None):
    """Sums the dense accumulators of all ranks and returns (this rank's
    slice of every accumulator, global index of the slice's first partition).
    Accumulator tensors must have the padded length partition_slices(...)[0].
    narrow_ints: int64 fields (counts, privacy-id counts, int sums) travel as
    int32 when no sum can overflow (exact either way; half the bytes of those
    fields over xGMI).  int_bound: a host-known bound on every int64 entry's
    sum over the ranks (counts and privacy-id counts are at most the global
    row count) -- then the choice needs no device read; without it the global
    maximum is read back (one MAX all-reduce and a device-to-host copy)."""
    import torch
    import torch.distributed as dist
    world, rank = world_info(group)
    if world == 1:
        return acc, 0
    sizes = {t.shape[0] for t in acc.values() if t is not None}
    if len(sizes) != 1:
        raise ValueError("accumulators must have equal lengths")
    padded = sizes.pop()
    if padded % world:
        raise ValueError(f"accumulator length {padded} is not a multiple of world size {world}")
    slice_len = padded // world
    backend = dist.get_backend(group)
    # one collective per dtype: the fields of a dtype are interleaved rank-major
    # ([rank][field][slice]) so that rank r's chunk of the sum is its slices of
    # every field
    out = {name: None for name in acc}
    by_dtype = {}
    for name, t in acc.items():
        if t is not None:
            by_dtype.setdefault(t.dtype, []).append(name)
    for dtype, names in by_dtype.items():
        stacked = torch.stack([acc[n].reshape(world, slice_len) for n in names], dim=1).contiguous()
        wire = stacked
        if dtype == torch.int64 and narrow_ints and int_bound is not None:
            if 0 <= int_bound < 2 ** 31:
                wire = stacked.to(torch.int32)
        elif dtype == torch.int64 and narrow_ints:
            # counts and privacy-id counts travel as int32 when no sum over
            # ranks can reach 2^31: every rank's entries lie in [0, m] with m
            # the global maximum (one all-reduce of 8 bytes), so every sum of
            # `world` of them is <= world * m (sums of fp accumulators stay fp64)
            lo_hi = torch.stack([(-stacked).max(), stacked.max()]) if stacked.numel() else \
                torch.zeros(2, dtype=torch.int64, device=stacked.device)
            lo_hi = lo_hi.to(_coll_device(group))
            dist.all_reduce(lo_hi, op=dist.ReduceOp.MAX, group=group)
            if int(lo_hi[0]) <= 0 and world * int(lo_hi[1]) < 2 ** 31:
                wire = stacked.to(torch.int32)
        if backend == "nccl":
            part = torch.empty((len(names), slice_len), dtype=wire.dtype, device=stacked.device)
            dist.reduce_scatter_tensor(part.view(-1), wire.view(-1), op=dist.ReduceOp.SUM, group=group)
        else:  # gloo (CPU tests): all-reduce then keep the owned chunk
            dist.all_reduce(wire, op=dist.ReduceOp.SUM, group=group)
            part = wire[rank].clone()
        part = part.to(dtype)
        for i, n in enumerate(names):
            out[n] = part[i]
    return out, rank * slice_len


def shard_by_privacy_id(privacy_ids, world: int, rank: int):
    """Boolean mask of the rows rank `rank` owns (privacy id hashed mod world),
    for callers that shard their own input before building a ColumnTable."""
    import numpy as np
    pid = np.asarray(privacy_ids)
    if pid.dtype.kind not in "iu":  # other keys: their identities (key_identities), as the library hashes them
        pid = key_identities(pid)
    # owner_of: data sharded by this helper passes the "verify" fast path
    return owner_of_np(pid, world) == rank


def _coll_device(group=None):
    """Device of the tensors a collective takes: the GPU under nccl (RCCL),
    the CPU under gloo."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _all_gather_sizes(n: int, group=None):
    import torch
    import torch.distributed as dist
    world, _ = world_info(group)
    dev = _coll_device(group)
    mine = torch.tensor([int(n)], dtype=torch.int64, device=dev)
    out = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(out, mine, group=group)
    return [int(t.item()) for t in out]


def _all_gather_var(arr, group=None):
    """All-gather of a variable-length 1-D int64 / uint8 numpy array as one
    padded tensor collective: every rank gets the list of all ranks' arrays
    (rank order)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world, _ = world_info(group)
    dev = _coll_device(group)
    sizes = _all_gather_sizes(len(arr), group)
    width = max(max(sizes), 1)
    buf = torch.zeros(width, dtype=torch.from_numpy(np.zeros(0, dtype=arr.dtype)).dtype, device=dev)
    if len(arr):
        buf[:len(arr)] = torch.from_numpy(np.ascontiguousarray(arr)).to(dev)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    return [o[:m].cpu().numpy() for o, m in zip(out, sizes)]


def row_offset(n_rows: int, group=None) -> int:
    """Global index of this rank's first row (ranks' shards concatenated in
    rank order); row sampling priorities are keyed by it."""
    return row_offset_and_total(n_rows, group)[0]


def row_offset_and_total(n_rows: int, group=None) -> Tuple[int, int]:
    """(row_offset, rows over all ranks) from one all-gather of the sizes."""
    world, rank = world_info(group)
    if world == 1:
        return 0, int(n_rows)
    sizes = _all_gather_sizes(n_rows, group)
    return int(sum(sizes[:rank])), int(sum(sizes))


def _key_kind(decode) -> str:
    import numpy as np
    if decode is None:
        return "ids"
    arr = np.asarray(decode, dtype=object)
    if all(isinstance(k, (int, np.integer)) and not isinstance(k, bool) for k in arr):
        return "int"
    if all(isinstance(k, str) for k in arr):
        return "str"
    return "object"


def global_partition_keys(enc, group=None):
    """Makes a rank-local partition-key encoding (columnar.EncodedKeys) global:
    every rank gets the same dense code for the same key, so the per-partition
    accumulators of all ranks line up for the exchange.  Dense integer keys
    keep the identity encoding (range = max over ranks); other keys get one
    dictionary in rank-then-first-appearance order.  Integer and string keys
    travel as tensors (int64 keys; UTF-8 bytes + lengths), so 1e7-key
    dictionaries need no pickling; other key types fall back to
    all_gather_object."""
    world, rank = world_info(group)
    if world == 1:
        return enc
    import numpy as np
    import torch
    import torch.distributed as dist
    from pipelinedp_amd.columnar import EncodedKeys
    kind = _key_kind(enc.decode)
    code = {"ids": 0, "int": 1, "str": 2, "object": 3}[kind]
    dev = _coll_device(group)
    mine = torch.tensor([code, int(enc.n)], dtype=torch.int64, device=dev)
    infos = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(infos, mine, group=group)
    kinds = [int(t[0].item()) for t in infos]
    ns = [int(t[1].item()) for t in infos]
    if all(k == 0 for k in kinds):
        return EncodedKeys(enc.codes, max(ns), None)
    if max(kinds) <= 1:  # identity ranges and integer dictionaries: int64 tensors
        local = np.arange(enc.n, dtype=np.int64) if kind == "ids" else np.asarray(enc.decode, dtype=np.int64)
        parts = _all_gather_var(local, group)
        allk = np.concatenate(parts) if parts else np.zeros(0, np.int64)
        uniq, first = np.unique(allk, return_index=True)
        order = np.argsort(first, kind="stable")      # rank-then-first-appearance
        decode = uniq[order]
        rank_of = np.empty(len(uniq), dtype=np.int64)
        rank_of[order] = np.arange(len(uniq))
        remap = rank_of[np.searchsorted(uniq, local)] if len(local) else np.zeros(0, np.int64)
        dec_obj = decode
    elif all(k == 2 for k in kinds):  # string dictionaries: UTF-8 bytes + byte lengths
        local_keys = list(enc.decode)
        enc_keys = [k.encode("utf-8") for k in local_keys]
        lens = np.fromiter((len(b) for b in enc_keys), dtype=np.int64, count=len(enc_keys))
        all_lens = _all_gather_var(lens, group)
        all_blobs = _all_gather_var(np.frombuffer(b"".join(enc_keys), dtype=np.uint8), group)
        mapping, dec = {}, []
        for ln, bl in zip(all_lens, all_blobs):
            raw, pos = bl.tobytes(), 0
            for m in ln.tolist():
                k = raw[pos:pos + m].decode("utf-8")
                pos += m
                if k not in mapping:
                    mapping[k] = len(dec)
                    dec.append(k)
        remap = np.fromiter((mapping[k] for k in local_keys), dtype=np.int64, count=len(local_keys))
        dec_obj = np.asarray(dec, dtype=object)
        decode = dec_obj
    else:
        return _global_keys_objects(enc, group)
    codes = enc.codes
    if type(codes).__module__.startswith("torch"):
        codes = torch.as_tensor(remap, device=codes.device)[codes]
    else:
        codes = remap[np.asarray(codes)] if len(remap) else np.asarray(codes, dtype=np.int64)
    return EncodedKeys(codes, max(len(decode), 1), np.asarray(dec_obj, dtype=object), None)


def _global_keys_objects(enc, group=None):
    """global_partition_keys for key types without a tensor form (tuples,
    mixed types): the dictionaries travel through all_gather_object."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from pipelinedp_amd.columnar import EncodedKeys
    world, _ = world_info(group)
    mine = ("ids", int(enc.n)) if enc.decode is None else ("dict", list(enc.decode))
    objs = [None] * world
    dist.all_gather_object(objs, mine, group=group)
    mapping, decode = {}, []
    for kind, payload in objs:
        keys = range(payload) if kind == "ids" else payload
        for k in keys:
            if k not in mapping:
                mapping[k] = len(decode)
                decode.append(k)
    local = range(enc.n) if enc.decode is None else enc.decode
    remap = np.fromiter((mapping[k] for k in local), dtype=np.int64, count=len(local))
    codes = enc.codes
    if type(codes).__module__.startswith("torch"):
        codes = torch.as_tensor(remap, device=codes.device)[codes]
    else:
        codes = remap[np.asarray(codes)] if len(remap) else np.asarray(codes, dtype=np.int64)
    return EncodedKeys(codes, len(decode), np.asarray(decode, dtype=object), mapping)


def broadcast_seeds(seeds, group=None):
    """Rank 0's seeds on every rank (selection and noise are keyed by global
    partition index, so all ranks must draw from the same streams): one
    uint64 tensor broadcast."""
    world, _ = world_info(group)
    if world == 1:
        return tuple(seeds)
    import torch
    import torch.distributed as dist
    vals = [int(x) & 0xFFFFFFFFFFFFFFFF for x in seeds]
    t = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in vals], dtype=torch.int64,
                     device=_coll_device(group))
    dist.broadcast(t, src=0, group=group)
    return tuple(int(v) & 0xFFFFFFFFFFFFFFFF for v in t.cpu().tolist())


def all_ranks_any(flag: bool, group=None) -> bool:
    world, _ = world_info(group)
    if world == 1:
        return bool(flag)
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=_coll_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(t.item())


_SIGN = -(1 << 63)


def exchange_histogram_stats(pkstat, psum, minmax, group=None):
    """Between pdp_dataset_histograms_pairs and _finish (pipelinedp_amd.h):
    sums the per-partition packed counters and value sums over ranks, and
    takes the global minimum / maximum of the pair sums.  The min / max words
    are order-preserving uint64 images; flipping the top bit makes their
    order the signed int64 order that ReduceOp.MIN / MAX use."""
    import torch.distributed as dist
    # each word packs (distinct pids << 32 | rows) for one rank's shard; sum
    # the two halves separately so that a partition's global row count cannot
    # carry into its privacy-id count, and refuse totals the packed format of
    # pdp_dataset_histograms_finish cannot hold
    mask = 0xFFFFFFFF
    lo = pkstat & mask
    hi = (pkstat >> 32) & mask
    dist.all_reduce(lo, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.SUM, group=group)
    if bool((lo > mask).any()) or bool((hi > mask).any()):
        raise ValueError("a partition holds 2^32 or more rows or privacy ids over all ranks; "
                         "the dataset histograms count per partition in 32 bits")
    pkstat.copy_((hi << 32) | lo)
    dist.all_reduce(psum, op=dist.ReduceOp.SUM, group=group)
    signed = minmax ^ _SIGN
    lo, hi = signed[0:1].clone(), signed[1:2].clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    minmax[0:1] = lo ^ _SIGN
    minmax[1:2] = hi ^ _SIGN


def exchange_preaggregated_stats(pk_rows, pk_count, psum, minmax, group=None):
    """Between pdp_dataset_histograms_preaggregated_rows and _finish: sums the
    per-partition row counts, count sums and value sums over ranks and takes
    the global minimum / maximum of the row sums (order-preserving words, as
    in exchange_histogram_stats)."""
    import torch.distributed as dist
    for t in (pk_rows, pk_count, psum):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    signed = minmax ^ _SIGN
    lo, hi = signed[0:1].clone(), signed[1:2].clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    minmax[0:1] = lo ^ _SIGN
    minmax[1:2] = hi ^ _SIGN


def exchange_preaggregated_weights(wsmall, wtab, group=None):
    """Between pdp_dataset_histograms_preaggregated_rows and _finish: makes the
    L0 / L1 weight sums global before they are rounded (a privacy
    id whose rows sit on two ranks must not be rounded per rank).  `wsmall`
    (double[2000], values below 1000) is summed over ranks and kept on rank 0
    only; every live entry of the weight table `wtab` (int64[slots, 2]: key,
    weight bits; key 0 = empty) goes to the rank that owns its key, which sums
    the entries per key; the table itself is zeroed.  Returns (keys, weights),
    the global sums of the keys this rank owns, for
    pdp_dataset_histograms_weight_bins after _finish (each key on one rank,
    so merge_histogram_bins adds every value's bin once)."""
    import torch
    import torch.distributed as dist
    world, rank = world_info(group)
    host = dist.get_backend(group) == "gloo"
    ws = wsmall.cpu() if host else wsmall
    dist.all_reduce(ws, op=dist.ReduceOp.SUM, group=group)
    if rank == 0:
        wsmall.copy_(ws)
    else:
        wsmall.zero_()
    live = wtab[:, 0] != 0
    keys = wtab[:, 0][live].clone()
    w = wtab[:, 1][live].clone().view(torch.float64)
    wtab.zero_()
    dest = _owner(keys, world)
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=world)
    rk, rw = _exchange([keys[order], w[order]], counts, group)
    uniq, inv = torch.unique(rk, return_inverse=True)
    tot = torch.zeros(uniq.numel(), dtype=torch.float64, device=rw.device)
    tot.index_add_(0, inv, rw)
    return uniq.to(wtab.device), tot.to(wtab.device)


def merge_histogram_bins(out, group=None):
    """Merges the bin arrays of pdp_dataset_histograms_finish over ranks:
    counts and sums added, maxima by maximum over the bins that hold
    elements, per-partition lowers from the rank that built them (the others
    hold zeros and no lowers), pair lowers identical on every rank."""
    import torch
    import torch.distributed as dist
    # mask with this rank's own counts, before they are summed
    fmax = torch.where(out["float_count"] > 0, out["float_max"], torch.full_like(out["float_max"], -float("inf")))
    for k in ("int_count", "int_sum", "float_count", "float_sum"):
        dist.all_reduce(out[k], op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(out["int_max"], op=dist.ReduceOp.MAX, group=group)  # counts >= 0: empty bins hold 0
    dist.all_reduce(fmax, op=dist.ReduceOp.MAX, group=group)
    out["float_max"].copy_(torch.where(torch.isfinite(fmax), fmax, torch.zeros_like(fmax)))
    part = out["float_lowers"][1:2].clone()  # only the partition-histogram rank wrote it
    dist.all_reduce(part, op=dist.ReduceOp.SUM, group=group)
    out["float_lowers"][1:2] = part
    dist.all_reduce(out["float_n_lowers"], op=dist.ReduceOp.MAX, group=group)


# ------------------------------------------------- privacy ids across ranks --
# Contribution bounding is exact only if all rows of a privacy id are on one
# rank (contribution_bounders.py:62-111 bounds per privacy id over the whole
# dataset).  ColumnarBackend either verifies that the caller sharded by
# privacy id, or shuffles the rows so that it holds.  Privacy ids are compared
# by a 64-bit identity: the id itself for integer ids, a fixed-key 64-bit hash
# of the key for other ids (the same on every rank).

def key_identities(keys) -> "np.ndarray":
    """int64 identities of a dictionary's keys (pandas' fixed-key SipHash;
    integers map to themselves)."""
    import numpy as np
    arr = np.asarray(keys, dtype=object)
    if len(arr) and all(isinstance(k, (int, np.integer)) and not isinstance(k, bool) for k in arr):
        return arr.astype(np.int64)
    from pandas.util import hash_array
    return hash_array(arr, categorize=False).view(np.int64)


def owner_of(ident, world: int):
    """Rank that owns an identity: a SplitMix64-style mix mod world (so that
    structured ids, e.g. multiples of the world size, still spread); the
    kernel twin is pdp_owner_mismatches (pipelinedp_amd.h)."""
    import torch
    z = ident.to(torch.int64)
    z = (z ^ (z >> 31)) * -7046029254386353131  # 0x9E3779B97F4A7C15 as int64
    z = z ^ (z >> 29)
    return torch.remainder(z, world)


_owner = owner_of


def owner_of_np(ident, world: int):
    """NumPy twin of owner_of (int64 wrap-around, arithmetic shifts)."""
    import numpy as np
    z = np.asarray(ident).astype(np.int64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> 31)) * np.int64(-7046029254386353131)
    z = z ^ (z >> 29)
    return np.mod(z, world)


def ids_hash_owned(ident, world: int, rank: int) -> bool:
    """True when every identity in `ident` (int64 tensor) has owner_of == rank:
    one pass of pdp_owner_mismatches on a GPU tensor, torch ops on a CPU one."""
    import torch
    if ident.numel() == 0:
        return True
    if ident.is_cuda:
        import ctypes
        from pipelinedp_amd import _native as N
        ids = ident.to(torch.int64).contiguous()
        out = torch.empty(1, dtype=torch.int32, device=ids.device)
        st = torch.cuda.current_stream(ids.device).cuda_stream
        N.check(N.lib().pdp_owner_mismatches(ctypes.c_void_p(ids.data_ptr()), ids.numel(), world, rank,
                                             ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st)),
                "pdp_owner_mismatches")
        return int(out.item()) == 0
    return bool((owner_of(ident, world) == rank).all())


def verify_privacy_id_sharding(ident, group=None) -> str:
    """ColumnarBackend privacy_id_sharding="verify": raises ValueError when a
    privacy id (int64 identity; rows or distinct keys) is on more than one
    rank.  Fast path: every rank holds only ids it owns (owner_of, one pass
    over the ids and one all-reduce of a flag) -- then no id can be on two
    ranks; otherwise the distinct ids are exchanged
    (check_privacy_ids_disjoint).  Returns "single", "owned" or "exchanged"."""
    import torch
    import torch.distributed as dist
    world, rank = world_info(group)
    if world == 1:
        return "single"
    ok = ids_hash_owned(ident, world, rank)
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=_coll_device(group))
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if int(flag.item()):
        return "owned"
    check_privacy_ids_disjoint(torch.unique(ident), group)
    return "exchanged"


def _exchange(parts_by_dest, counts, group):
    """all-to-all of one tensor already ordered by destination rank."""
    import torch
    import torch.distributed as dist
    host = dist.get_backend(group) == "gloo"  # gloo moves host tensors (CPU tests, 2-rank GPU test)
    send = counts.to(torch.int64)
    send = send.cpu() if host else send
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    in_sizes = send.tolist()
    out_sizes = recv.tolist()
    out = []
    for t in parts_by_dest:
        src = t.contiguous().cpu() if host else t.contiguous()
        o = torch.empty((sum(out_sizes),) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
        dist.all_to_all_single(o, src, output_split_sizes=out_sizes, input_split_sizes=in_sizes, group=group)
        out.append(o.to(t.device))
    return out


def check_privacy_ids_disjoint(ids, group=None):
    """Raises ValueError when a privacy id (int64 identity) is present on more
    than one rank.  `ids`: the distinct identities of this rank.  Each
    identity goes to its owner rank (one all-to-all of 8 B per distinct id);
    owners look for an identity that arrived from two ranks."""
    import torch
    import torch.distributed as dist
    world, rank = world_info(group)
    if world == 1:
        return
    ids = ids.to(torch.int64)
    dest = _owner(ids, world)
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=world)
    (recv,) = _exchange([ids[order]], counts, group)
    s = torch.sort(recv).values
    dup = bool((s[1:] == s[:-1]).any()) if s.numel() > 1 else False
    flag = torch.tensor([1 if dup else 0], dtype=torch.int64,
                        device="cpu" if dist.get_backend(group) == "gloo" else ids.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    if int(flag.item()):
        raise ValueError("a privacy id appears on more than one rank: rows must be sharded by privacy id "
                         "(contribution bounding is per privacy id over the whole dataset, "
                         "contribution_bounders.py:62-111); pass ColumnarBackend(privacy_id_sharding="
                         "'shuffle') to let the library exchange the rows")


def shuffle_by_privacy_id(ident, columns, group=None):
    """Moves every row to the rank that owns its privacy id (identity):
    returns (identities, columns) of the rows this rank now holds, in
    (source rank, source order) order — deterministic for a fixed input.
    `columns` may hold None entries (passed through as None)."""
    import torch
    world, _ = world_info(group)
    if world == 1:
        return ident, columns
    dest = _owner(ident, world)
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=world)
    live = [c for c in columns if c is not None]
    out = _exchange([ident[order]] + [c[order] for c in live], counts, group)
    it = iter(out[1:])
    return out[0], [None if c is None else next(it) for c in columns]
