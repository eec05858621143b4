"""TEST INFRASTRUCTURE — vectorised NumPy restatement of the bounded aggregation.

Restates, for one shard of dense columns (privacy_id, partition_key, value):

* SamplingCrossAndPerPartitionContributionBounder.bound_contributions
  (reference pipeline_dp/contribution_bounders.py:72-111): per (pid, pk) keep a
  uniform sample of <= linf rows, per pid keep a uniform sample of <= l0 of its
  distinct partitions; linf = 0 restates SamplingCrossPartitionContributionBounder
  (:168-201, every row of a kept pair); l0 = 0 restates LinfSampler (:204-230)
  and, with linf = 0, NoOpSampler (:233-246); max_contributions restates
  SamplingPerPrivacyIdContributionBounder (:114-156); rows_are_units restates
  DPEngine's contribution_bounds_already_enforced branch (dp_engine.py:143-150);
* CompoundCombiner.create_accumulator + merge (combiners.py:749-764) for the
  Count/Sum/Mean/Variance/PrivacyIdCount children (combiners.py:241-587);
* LocalBackend.combine_accumulators_per_key (pipeline_backend.py:555-565);
* private partition selection (dp_engine.py:315-371) and
  CompoundCombiner.compute_metrics noise (combiners.py:766-788,
  dp_computations.py:306-365, 540-575).

Uniform sampling without replacement is "keep the k smallest i.i.d. uniform
priorities".  With ``priorities="hash"`` the priorities are the exact
counter-based values the HIP kernels compute (pair keys: a MurmurHash3 fmix32
hash of (seed, pid, pk); row keys: SplitMix64 of the global row index), so the
sampled sets match the GPU bit-for-bit; with ``priorities="rng"`` they come
from a NumPy Generator (the reference's np.random.choice distribution).
Noise and selection use the same Philox4x32-10 streams and the same
granularity-snapped secure samplers as the kernels.
"""
import numpy as np

# flags / kinds (must equal include/pipelinedp_amd.h)
VALUE_NONE, VALUE_F64, VALUE_I64 = 0, 1, 2
ACC_SUM, ACC_NSUM, ACC_NSUM2, SUM_PER_PARTITION, SUM_INT = 0x1, 0x2, 0x4, 0x8, 0x10
SELECT_ALL_NONEMPTY, SELECT_TRUNCATED_GEOMETRIC, SELECT_LAPLACE, SELECT_GAUSSIAN, SELECT_PUBLIC = range(5)
OP_COUNT, OP_SUM, OP_PRIVACY_ID_COUNT, OP_MEAN, OP_VARIANCE, OP_THRESHOLDED_PID = 1, 2, 3, 4, 5, 6
NOISE_LAPLACE, NOISE_GAUSSIAN = 0, 1

_U64 = np.uint64
EMPTY = _U64(0xFFFFFFFFFFFFFFFF)


def mix64(z):
    """SplitMix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> _U64(30))) * _U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U64(27))) * _U64(0x94D049BB133111EB)
    return z ^ (z >> _U64(31))


def pk_bits(n_partitions):
    b = 1
    while b < 63 and (1 << b) < n_partitions:
        b += 1
    return b


def fmix32(h):
    """MurmurHash3 32-bit finaliser on uint32 arrays (wrapping arithmetic)."""
    h = np.asarray(h, dtype=np.uint32)
    with np.errstate(over="ignore"):
        h = h ^ (h >> np.uint32(16))
        h = h * np.uint32(0x85EBCA6B)
        h = h ^ (h >> np.uint32(13))
        h = h * np.uint32(0xC2B2AE35)
        return h ^ (h >> np.uint32(16))


def pair_hash(seed, pid, pk):
    """32 random bits per (pid, pk) pair (kernels: pdp_internal.h pair_hash)."""
    pid = np.asarray(pid).astype(np.uint64)
    pk = np.asarray(pk).astype(np.uint64)
    s0, s1 = np.uint32(int(seed) & 0xFFFFFFFF), np.uint32((int(seed) >> 32) & 0xFFFFFFFF)
    lo = (pid & _U64(0xFFFFFFFF)).astype(np.uint32)
    hi = (pid >> _U64(32)).astype(np.uint32)
    pk32 = (pk & _U64(0xFFFFFFFF)).astype(np.uint32)
    with np.errstate(over="ignore"):
        rot = (hi << np.uint32(16)) | (hi >> np.uint32(16))
        h = (lo ^ rot ^ s0) * np.uint32(0x9E3779B1)
        return fmix32(h ^ (pk32 * np.uint32(0xC2B2AE3D) + s1))


def pair_priority(seed, pid, pk, rand_shift):
    """Sampling key of (pid, pk): the pair hash in bits [32, 64), cleared below
    rand_shift, then pk (the kernels may also place the bucket-local pid in
    between; that does not change the order among one pid's pairs)."""
    h = pair_hash(seed, pid, pk).astype(np.uint64) << _U64(32)
    low = _U64((1 << rand_shift) - 1)
    x = (h & ~low) | np.asarray(pk).astype(np.uint64)
    bad = (x | low) == EMPTY
    return np.where(bad, x & ~_U64(1 << rand_shift), x)


def derive_row_seed(seed):
    return int(mix64(np.array([_U64(seed) ^ _U64(0x5851F42D4C957F2D)]))[0])


def row_priority(row_seed, global_row, local_row):
    g = np.asarray(global_row).astype(np.uint64)
    with np.errstate(over="ignore"):
        h = mix64(_U64(row_seed) ^ (g * _U64(0xD6E8FEB86659FD93)))
    return (h & _U64(0xFFFFFFFF00000000)) | np.asarray(local_row).astype(np.uint64)


# ------------------------------------------------------------------ philox --
def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint32) for c in (c0, c1, c2, c3))
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    m0, m1 = _U64(0xD2511F53), _U64(0xCD9E8D57)
    for _ in range(10):
        p0 = c0.astype(np.uint64) * m0
        p1 = c2.astype(np.uint64) * m1
        hi0, lo0 = (p0 >> _U64(32)).astype(np.uint32), p0.astype(np.uint32)
        hi1, lo1 = (p1 >> _U64(32)).astype(np.uint32), p1.astype(np.uint32)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint32(k0), lo1, hi0 ^ c3 ^ np.uint32(k1), lo0)
        k0 = (k0 + 0x9E3779B9) & 0xFFFFFFFF
        k1 = (k1 + 0xBB67AE85) & 0xFFFFFFFF
    return c0, c1, c2, c3


def u01(hi, lo):
    x = ((hi.astype(np.uint64) << _U64(32)) | lo.astype(np.uint64)) >> _U64(11)
    return (x.astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


def philox_for(seed, gidx, slot):
    gidx = np.asarray(gidx, dtype=np.int64).astype(np.uint64)
    c0 = (gidx & _U64(0xFFFFFFFF)).astype(np.uint32)
    c1 = (gidx >> _U64(32)).astype(np.uint32)
    c2 = np.full(c0.shape, slot & 0xFFFFFFFF, dtype=np.uint32)
    c3 = np.full(c0.shape, 0x50445021, dtype=np.uint32)
    return philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)


# ------------------------------------------------------------ secure noise --
# Restates the kernels' secure samplers (pdp_internal.h secure_*), which
# restate the granularity-snapped samplers of Google's differential-privacy
# library behind PyDP (python-dp ~=1.1.5rc4, not installed here):
# out = round_to_multiple(x, g) + g * k, k two-sided geometric (Laplace) or a
# centred binomial (Gaussian).  Philox blocks are consumed in the kernels'
# order, so GPU and oracle agree bit for bit (up to a last-ulp difference of
# expm1 / exp flipping one Bernoulli, probability ~1e-16 per draw).
INT64_MAX = np.int64(0x7FFFFFFFFFFFFFFF)


def noise_block(seed, gidx, slot, k):
    gidx = np.asarray(gidx, dtype=np.int64).astype(np.uint64)
    c0 = (gidx & _U64(0xFFFFFFFF)).astype(np.uint32)
    c1 = (gidx >> _U64(32)).astype(np.uint32)
    c2 = np.full(c0.shape, slot & 0xFFFFFFFF, dtype=np.uint32)
    c3 = (np.uint32(0x4E000000) + np.asarray(k, dtype=np.uint32)).astype(np.uint32)
    return philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)


def round_to_multiple(x, base):
    x = np.asarray(x, dtype=np.float64)
    if base == 0.0:
        return x
    r = np.fmod(x, base)
    return np.where(np.abs(r) > base / 2, x - r + np.copysign(base, r), x - r)


def secure_geometric(lam, seed, gidx, slot, k):
    """Bisection geometric sampler (pdp_internal.h secure_geometric); k: the
    per-element next Philox block index (updated in place)."""
    n = len(gidx)
    lo = np.zeros(n, dtype=np.int64)
    hi = np.full(n, INT64_MAX, dtype=np.int64)
    half = np.zeros(n, dtype=bool)
    bz = np.zeros(n, dtype=np.uint32)
    bw = np.zeros(n, dtype=np.uint32)
    idx = np.arange(n)
    while len(idx):
        l, h = lo[idx], hi[idx]
        mid = l + ((h - l) >> 1)
        with np.errstate(over="ignore"):
            q = np.expm1(lam * (l - mid).astype(np.float64)) / np.expm1(lam * (l - h).astype(np.float64))
        det = q >= 1.0
        hi[idx[det]] = mid[det]
        r = idx[~det]
        if len(r):
            qr, mr = q[~det], mid[~det]
            fresh = r[~half[r]]
            u = np.empty(len(r))
            if len(fresh):
                b = noise_block(seed, gidx[fresh], slot, k[fresh])
                k[fresh] += 1
                bz[fresh], bw[fresh] = b[2], b[3]
                u[~half[r]] = u01(b[0], b[1])
            old = half[r]
            if old.any():
                u[old] = u01(bz[r[old]], bw[r[old]])
            half[r] = ~half[r]
            low = u <= qr
            hi[r[low]] = mr[low]
            lo[r[~low]] = mr[~low]
        idx = idx[lo[idx] + 1 < hi[idx]]
    return hi - 1


def secure_laplace(np_, seed, gidx, slot):
    gidx = np.asarray(gidx, dtype=np.int64)
    out = np.empty(len(gidx))
    k = np.zeros(len(gidx), dtype=np.uint32)
    pend = np.arange(len(gidx))
    while len(pend):
        a = noise_block(seed, gidx[pend], slot, k[pend])
        k[pend] += 1
        positive = (a[0] >> np.uint32(31)) != 0
        kk = k[pend]
        s = secure_geometric(np_["lambda"], seed, gidx[pend], slot, kk)
        k[pend] = kk
        redo = (s == 0) & ~positive
        sf = s.astype(np.float64)
        v = np.where(positive, sf, -sf) * np_["granularity"]
        out[pend[~redo]] = v[~redo]
        pend = pend[redo]
    return out


def _clz32(v):
    v = np.asarray(v, dtype=np.uint32)
    e = np.frexp(v.astype(np.float64))[1]
    return np.where(v == 0, 32, 32 - e).astype(np.int64)


def secure_gaussian(np_, seed, gidx, slot):
    """pdp_internal.h gaussian_attempt: one Philox block per attempt -- x[31:24]
    geometric bits (leading ones, at most 8), x[23] sign, (y, z) the uniform
    offset's 64 bits, (w, x[20:0]) the acceptance uniform's 53 bits."""
    gidx = np.asarray(gidx, dtype=np.int64)
    out = np.empty(len(gidx))
    k = np.zeros(len(gidx), dtype=np.uint32)
    step = int(np_["step"])
    pend = np.arange(len(gidx))
    while len(pend):
        a = noise_block(seed, gidx[pend], slot, k[pend])
        k[pend] += 1
        ones = (~a[0] & np.uint32(0xFF000000)) | np.uint32(0x00800000)
        geom = _clz32(ones)
        two_sided = np.where(((a[0] >> np.uint32(23)) & np.uint32(1)) != 0, geom, -geom - 1)
        st = _U64(step)
        with np.errstate(over="ignore"):
            hi_part = a[1].astype(np.uint64) * st + ((a[2].astype(np.uint64) * st) >> _U64(32))
        uni = (hi_part >> _U64(32)).astype(np.int64)
        m = np.int64(step) * two_sided + uni
        u53 = (a[3].astype(np.uint64) << _U64(21)) | (a[0] & np.uint32(0x1FFFFF)).astype(np.uint64)
        accept_u = (u53.astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)
        md = m.astype(np.float64)
        inb = np.abs(md) <= np_["bound"]
        prob = np_["coef"] * np.exp(-2.0 * md * md / np_["n"]) * np_["corr"]
        ok = inb & (prob > 0.0) & (accept_u < prob * float(step) * np.ldexp(1.0, geom) / 4.0)
        out[pend[ok]] = md[ok] * np_["granularity"]
        pend = pend[~ok]
    return out


def secure_add_noise(np_, x, seed, gidx, slot):
    """mechanism.add_noise(x) for the elements x[i] with streams gidx[i]."""
    x = np.asarray(x, dtype=np.float64)
    g = float(np_["granularity"])
    if g == 0.0:
        return x.copy()
    noise = secure_gaussian(np_, seed, gidx, slot) if np_["kind"] == NOISE_GAUSSIAN else \
        secure_laplace(np_, seed, gidx, slot)
    return round_to_multiple(x, g) + noise


# ------------------------------------------------------------- bounding --
def _ranks_within(groups_sorted):
    """0-based position of each element inside its run of equal keys."""
    n = len(groups_sorted)
    if n == 0:
        return np.zeros(0, dtype=np.int64)
    start = np.ones(n, dtype=bool)
    start[1:] = groups_sorted[1:] != groups_sorted[:-1]
    gid = np.cumsum(start) - 1
    starts = np.flatnonzero(start)
    return np.arange(n, dtype=np.int64) - starts[gid]


def derive_pid_row_seed(seed):
    """Row priorities of SamplingPerPrivacyIdContributionBounder (pdp_pairs.hip)."""
    return derive_row_seed(int(seed) ^ 0x2545F4914F6CDD1D)


def bound_and_reduce(pid, pk, value, *, n_privacy_ids, n_partitions, l0, linf, value_kind,
                     flags, min_value=0.0, max_value=0.0, middle=0.0, min_sum=0.0,
                     max_sum=0.0, seed=0, row_offset=0, allowed=None, priorities="hash",
                     rng=None, rand_shift=None, max_contributions=0, rows_are_units=False,
                     row_index=None):
    """Returns dense per-partition accumulators (dict of numpy arrays, length P).

    l0 = 0: no cross-partition sampling (every pair kept).  max_contributions:
    per pid keep the rows of the max_contributions smallest row priorities
    first.  rows_are_units: every row is its own pair (pid is ignored).
    row_index: the rows' indices in the kernels' input (default 0..n-1), for
    a privacy-id subset of a larger input (oracle/parallel_oracle.py); the
    value column is then the whole input's, indexed by row_index."""
    pk = np.asarray(pk, dtype=np.int64)
    if rows_are_units:  # one privacy unit per row: the row index is the pid
        pid = np.arange(len(pk), dtype=np.int64)
        n_privacy_ids = max(1, len(pk))
    pid = np.asarray(pid, dtype=np.int64)
    n = len(pid)
    P = int(n_partitions)
    out = {
        "privacy_id_count": np.zeros(P, np.int64),
        "count": np.zeros(P, np.int64),
        "sum": np.zeros(P, np.int64 if flags & SUM_INT else np.float64),
        "normalized_sum": np.zeros(P, np.float64),
        "normalized_sum_sq": np.zeros(P, np.float64),
    }
    local = np.arange(n, dtype=np.int64) if row_index is None else np.asarray(row_index, dtype=np.int64)
    valid = (pid >= 0) & (pid < n_privacy_ids) & (pk >= 0) & (pk < P)
    if allowed is not None:
        valid &= np.asarray(allowed, dtype=bool)[np.clip(pk, 0, P - 1)]
    pid, pk, local = pid[valid], pk[valid], local[valid]
    if max_contributions:
        # per pid, the rows of the max_contributions smallest row priorities
        if priorities == "hash":
            prio = row_priority(derive_pid_row_seed(seed), row_offset + local, local)
        else:
            prio = (rng.integers(0, 1 << 32, size=len(local), dtype=np.uint64) << _U64(32)) | \
                local.astype(np.uint64)
        o = np.lexsort((prio, pid))
        keep = np.zeros(len(pid), dtype=bool)
        keep[o] = _ranks_within(pid[o]) < max_contributions
        pid, pk, local = pid[keep], pk[keep], local[keep]
    if len(pid) == 0:
        return out
    if rand_shift is None:
        rand_shift = pk_bits(P)
    # distinct pairs
    order = np.lexsort((pk, pid))
    ps, ks, ls = pid[order], pk[order], local[order]
    first = np.ones(len(ps), dtype=bool)
    first[1:] = (ps[1:] != ps[:-1]) | (ks[1:] != ks[:-1])
    row_pair = np.cumsum(first) - 1
    pair_pid, pair_pk = ps[first], ks[first]
    if priorities == "hash":
        pprio = pair_priority(seed, pair_pid, pair_pk, rand_shift)
    else:
        rand = rng.integers(0, 1 << (64 - pk_bits(P)), size=len(pair_pid), dtype=np.uint64)
        pprio = (rand << _U64(pk_bits(P))) | pair_pk.astype(np.uint64)
    # L0: rank pairs of each pid by priority
    o2 = np.lexsort((pprio, pair_pid))
    rank = np.empty(len(pair_pid), dtype=np.int64)
    rank[o2] = _ranks_within(pair_pid[o2])
    kept_pair = rank < l0 if l0 > 0 else np.ones(len(pair_pid), dtype=bool)
    # rows of kept pairs
    rk = kept_pair[row_pair]
    r_pair, r_local = row_pair[rk], ls[rk]
    if priorities == "hash":
        rprio = row_priority(derive_row_seed(seed), row_offset + r_local, r_local)
    else:
        rand = rng.integers(0, 1 << 32, size=len(r_pair), dtype=np.uint64)
        rprio = (rand << _U64(32)) | r_local.astype(np.uint64)
    o3 = np.lexsort((rprio, r_pair))
    r_pair, r_local = r_pair[o3], r_local[o3]
    if linf > 0:
        keep_row = _ranks_within(r_pair) < linf
        r_pair, r_local = r_pair[keep_row], r_local[keep_row]
    kp = np.flatnonzero(kept_pair)
    part_of_pair = pair_pk[kp]
    cnt = np.bincount(r_pair, minlength=len(pair_pid))[kp]
    np.add.at(out["privacy_id_count"], part_of_pair, 1)
    np.add.at(out["count"], part_of_pair, cnt.astype(np.int64))
    if value_kind == VALUE_NONE:
        return out
    vals = np.asarray(value)[r_local]
    fv = vals.astype(np.float64)
    cv = np.clip(fv, min_value, max_value)
    # per-pair sequential sums in ascending row-priority order (as the kernels)
    seg_start = np.flatnonzero(np.r_[True, r_pair[1:] != r_pair[:-1]])
    seg_pair = r_pair[seg_start]
    pos = np.searchsorted(kp, seg_pair)

    def seg_sum(x):
        s = np.zeros(len(kp), dtype=x.dtype)
        s[pos] = np.add.reduceat(x, seg_start) if len(x) else s[pos]
        return s

    if flags & SUM_PER_PARTITION:
        if flags & SUM_INT:
            raw = seg_sum(vals.astype(np.int64))
            psum = np.clip(raw, int(min_sum), int(max_sum))
        else:
            psum = np.clip(seg_sum(fv), min_sum, max_sum)
        np.add.at(out["sum"], part_of_pair, psum)
    elif flags & ACC_SUM:
        if flags & SUM_INT:
            psum = seg_sum(np.clip(vals.astype(np.int64), int(min_value), int(max_value)))
        else:
            psum = seg_sum(cv)
        np.add.at(out["sum"], part_of_pair, psum)
    nc = cv - middle
    if flags & ACC_NSUM:
        np.add.at(out["normalized_sum"], part_of_pair, seg_sum(nc))
    if flags & ACC_NSUM2:
        np.add.at(out["normalized_sum_sq"], part_of_pair, seg_sum(nc * nc))
    return out


# --------------------------------------------------- selection + metrics --
def select(row_count, strategy, *, max_rows_per_privacy_id=1, pre_threshold=0, keep_prob=None,
           noise=None, threshold=0.0, public_mask=None, seed=0, partition_offset=0):
    """Restates pdp_select_partitions: returns (keep bool[P], noised float[P])."""
    rc = np.asarray(row_count, dtype=np.int64)
    P = len(rc)
    noised = np.full(P, np.nan)
    if strategy == SELECT_PUBLIC:
        return np.asarray(public_mask) != 0, noised
    if strategy == SELECT_ALL_NONEMPTY:
        return rc > 0, noised
    mr = max(1, int(max_rows_per_privacy_id))
    n = (rc + mr - 1) // mr
    ok = rc > 0
    shift = 0
    if pre_threshold and pre_threshold > 0:
        ok &= n >= pre_threshold
        shift = pre_threshold - 1
        n = n - shift
    if strategy == SELECT_TRUNCATED_GEOMETRIC:
        r = philox_for(seed, partition_offset + np.arange(P), 0x53454C00)
        table = np.asarray(keep_prob, dtype=np.float64)
        t = np.minimum(np.maximum(n, 0), len(table) - 1)
        keep = ok & (u01(r[0], r[1]) < table[t])
        return keep, noised
    v = np.full(P, -np.inf)
    live = np.flatnonzero(ok)
    v[live] = secure_add_noise(noise, n[live].astype(np.float64), seed, partition_offset + live, 0x53454C00)
    keep = ok & (v > threshold)
    noised = np.where(keep, v + shift, np.nan)
    return keep, noised


def noise_metrics(ops, index, acc, sum_is_int, noised_count, seed, partition_offset=0, n_cols=None):
    """Restates pdp_noise_metrics. ops: list of dicts with the pdp_metric_op fields."""
    index = np.asarray(index, dtype=np.int64)
    g = partition_offset + index
    if n_cols is None:
        n_cols = 1 + max(c for op in ops for c in op["out_col"])
    out = np.full((n_cols, len(index)), np.nan)

    def put(col, v):
        if col >= 0:
            out[col] = v

    for o, op in enumerate(ops):
        slot = o << 4
        kind, nz, cols = op["kind"], op["noise"], op["out_col"]

        def noised(m, x, sl):
            return secure_add_noise(nz[m], np.asarray(x, dtype=np.float64), seed, g, sl)

        if kind == OP_COUNT:
            put(cols[0], noised(0, acc["count"][index], slot))
        elif kind == OP_SUM:
            put(cols[0], noised(0, acc["sum"][index].astype(np.float64), slot))
        elif kind == OP_PRIVACY_ID_COUNT:
            put(cols[0], noised(0, acc["privacy_id_count"][index], slot))
        elif kind == OP_MEAN:
            dp_count = noised(0, acc["count"][index], slot)
            denom = np.maximum(1.0, dp_count)
            dp_nsum = noised(1, acc["normalized_sum"][index], slot + 1)
            mean = op["middle"] + dp_nsum / denom
            put(cols[0], mean)
            put(cols[1], dp_count)
            put(cols[2], mean * dp_count)
        elif kind == OP_VARIANCE:
            dp_count = noised(0, acc["count"][index], slot)
            if op.get("degenerate", 0):
                dp_mean = np.full(len(index), op["min_value"])
                dp_mean_sq = np.full(len(index), op["sq_min_value"])
            else:
                denom = np.maximum(1.0, dp_count)
                dp_mean = noised(1, acc["normalized_sum"][index], slot + 1) / denom
                dp_mean_sq = noised(2, acc["normalized_sum_sq"][index], slot + 2) / denom
            dp_var = dp_mean_sq - dp_mean * dp_mean
            if not op.get("degenerate", 0):
                dp_mean = dp_mean + op["middle"]
            put(cols[0], dp_var)
            put(cols[1], dp_count)
            put(cols[2], dp_mean * dp_count)
            put(cols[3], dp_mean)
        elif kind == OP_THRESHOLDED_PID:
            put(cols[0], np.asarray(noised_count)[index])
    return out


ADD_NOISE_SLOT = 0x41444E00  # pdp_select.hip kAddNoiseSlot


def add_noise(values, noise, seed, index_offset=0):
    """DPEngine.add_dp_noise's "Add noise" map (dp_engine.py:595-599):
    mechanism.add_noise(float(value)), element i drawing from the Philox
    streams (seed, offset + i)."""
    x = np.asarray(values)
    idx = np.arange(x.shape[0], dtype=np.int64) + int(index_offset)
    return secure_add_noise(noise, x.astype(np.float64), int(seed), idx, ADD_NOISE_SLOT)
