"""Device-side execution of the aggregate hot path through the C ABI.

Everything here works on torch-ROCm device tensors (torch is only the
allocator/stream provider) and calls the HIP kernels of
``csrc/pdp_kernels.hip`` through :mod:`pipelinedp_amd._native`.  There is no
CPU fallback: every entry point raises :class:`NativeLibraryError` when the
library is missing and ``RuntimeError`` when no GPU is present.

Stage order (reference dp_engine.py:109-187):
  bound_and_reduce  -> contribution bounding + per-partition accumulators
  [all-reduce/reduce-scatter of accumulators across ranks: parallel.py]
  select_and_noise  -> partition selection, compaction, compute_metrics noise
"""
import ctypes
import dataclasses
import os
import weakref
from typing import Dict, List, Optional, Sequence

import numpy as np

from pipelinedp_amd import _native as N
from pipelinedp_amd.dp_computations import NO_NOISE, NoiseParams


@dataclasses.dataclass
class BoundingSpec:
    """Columnar form of the bounder + combiner-accumulator parameters.

    l0 > 0: SamplingCross[AndPer]PartitionContributionBounder; l0 = 0:
    LinfSampler (linf > 0) / NoOpSampler (linf = 0); max_contributions > 0:
    SamplingPerPrivacyIdContributionBounder; rows_are_units:
    contribution_bounds_already_enforced (no privacy ids)."""
    l0: int                        # 0: no cross-partition sampling
    linf: int                      # 0: keep every row of a kept pair
    value_kind: int                # N.VALUE_*
    flags: int                     # N.ACC_* | N.SUM_*
    min_value: float = 0.0
    max_value: float = 0.0
    middle: float = 0.0
    min_sum: float = 0.0
    max_sum: float = 0.0
    max_contributions: int = 0
    rows_are_units: bool = False

    @property
    def sum_is_int(self) -> bool:
        return bool(self.flags & N.SUM_INT)


@dataclasses.dataclass
class SelectionSpec:
    strategy: int                  # N.SELECT_*
    max_rows_per_privacy_id: int = 1
    pre_threshold: int = 0
    keep_prob: Optional[np.ndarray] = None
    noise: Optional[NoiseParams] = None  # thresholding strategies: the secure mechanism
    threshold: float = 0.0
    want_noised_count: bool = False

    @property
    def noise_scale(self) -> float:
        return 0.0 if self.noise is None else self.noise.scale


@dataclasses.dataclass
class MetricOpSpec:
    """One CompoundCombiner child's metric op (pdp_metric_op); `noise` holds
    its mechanisms' secure samplers (COUNT/SUM/PID: 1, MEAN: 2, VARIANCE: 3)."""
    kind: int
    out_col: Sequence[int] = (-1, -1, -1, -1)
    noise: Sequence[NoiseParams] = ()
    middle: float = 0.0
    min_value: float = 0.0
    sq_min_value: float = 0.0
    degenerate: int = 0

    @property
    def scale(self):
        return tuple(p.scale for p in self.noise)

    @property
    def noise_kind(self) -> int:
        return self.noise[0].kind if self.noise else N.NOISE_LAPLACE

    def _noise3(self):
        return list(self.noise) + [NO_NOISE] * (3 - len(self.noise))

    def to_c(self) -> N.MetricOp:
        op = N.MetricOp()
        op.kind = self.kind
        cols = list(self.out_col) + [-1] * (4 - len(self.out_col))
        for i in range(4):
            op.out_col[i] = int(cols[i])
        for i, p in enumerate(self._noise3()):
            op.noise[i] = p.to_c()
        op.middle = float(self.middle)
        op.min_value = float(self.min_value)
        op.sq_min_value = float(self.sq_min_value)
        op.degenerate = int(self.degenerate)
        return op

    def as_dict(self) -> dict:
        cols = list(self.out_col) + [-1] * (4 - len(self.out_col))
        return dict(kind=self.kind, out_col=cols, noise=[p.as_dict() for p in self._noise3()],
                    middle=self.middle, min_value=self.min_value,
                    sq_min_value=self.sq_min_value, degenerate=self.degenerate)


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("pipelinedp_amd needs a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")
    return torch


def _ptr(t) -> Optional[int]:
    return None if t is None else int(t.data_ptr())


def _stream(stream=None) -> int:
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def _check_col(t, name, dtypes, n, device):
    torch = _torch()
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch tensor on the GPU")
    if t.dtype not in dtypes:
        raise TypeError(f"{name} has dtype {t.dtype}, expected one of {dtypes}")
    if t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if t.dim() != 1 or t.shape[0] != n:
        raise ValueError(f"{name} must be 1-D of length {n}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


class StageTimer:
    """Records HIP events (torch.cuda.Event on the launch stream) at stage
    boundaries; durations() gives ms between consecutive marks."""

    def __init__(self, stream=None):
        self.stream = stream
        self.marks = []

    def mark(self, name):
        torch = _torch()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(self.stream if self.stream is not None else torch.cuda.current_stream())
        self.marks.append((name, ev))

    def durations(self):
        out = {}
        for (name, a), (_, b) in zip(self.marks, self.marks[1:]):
            if name.startswith("end_"):
                continue
            out[name] = out.get(name, 0.0) + a.elapsed_time(b)
        return out


def _mark(timer, name):
    if timer is not None:
        timer.mark(name)


def new_accumulators(n_partitions: int, bounding: BoundingSpec, device) -> Dict[str, "torch.Tensor"]:
    torch = _torch()
    P = int(n_partitions)
    names = ["privacy_id_count", "count"]
    if bounding.flags & (N.ACC_SUM | N.SUM_PER_PARTITION):
        names.append("sum")
    if bounding.flags & N.ACC_NSUM:
        names.append("normalized_sum")
    if bounding.flags & N.ACC_NSUM2:
        names.append("normalized_sum_sq")
    # one zero fill for every field: 8-byte fields side by side, each starting
    # on a 256-byte boundary (all-zero bits are 0 as int64 and 0.0 as float64)
    stride = (P + 31) // 32 * 32
    block = torch.zeros(len(names) * stride, dtype=torch.int64, device=device)
    acc = {"privacy_id_count": None, "count": None, "sum": None, "normalized_sum": None,
           "normalized_sum_sq": None}
    for k, name in enumerate(names):
        field = block[k * stride:k * stride + P]
        is_int = name in ("privacy_id_count", "count") or (name == "sum" and bounding.sum_is_int)
        acc[name] = field if is_int else field.view(torch.float64)
    return acc


def zero_accumulators(acc):
    """Zeroes accumulators from new_accumulators in one fill (their fields
    are views of one block); any other dict field by field."""
    fields = [t for t in acc.values() if t is not None]
    bases = {id(t._base): t._base for t in fields if t._base is not None}
    if len(bases) == 1 and all(t._base is not None for t in fields):
        next(iter(bases.values())).zero_()
    else:
        for t in fields:
            t.zero_()
    return acc


def _acc_struct(acc) -> N.PartitionAccumulators:
    s = N.PartitionAccumulators()
    s.privacy_id_count = _ptr(acc["privacy_id_count"])
    s.count = _ptr(acc["count"])
    s.sum = _ptr(acc["sum"])
    s.normalized_sum = _ptr(acc["normalized_sum"])
    s.normalized_sum_sq = _ptr(acc["normalized_sum_sq"])
    return s


def bound_config(n_rows, n_privacy_ids, n_partitions, bounding: BoundingSpec, seed: int,
                 row_offset: int = 0, algorithm: int = N.ALGO_AUTO,
                 merge: int = N.MERGE_AUTO, key_format: int = N.KEYS_AUTO, sieve: int = 0,
                 sieve_band: int = 0, sieve_threads: int = 0, bucket_threads: int = 0) -> N.BoundConfig:
    c = N.BoundConfig()
    c.n_rows = int(n_rows)
    c.n_privacy_ids = int(n_privacy_ids)
    c.n_partitions = int(n_partitions)
    c.l0 = int(bounding.l0)
    c.linf = int(bounding.linf)
    c.value_kind = int(bounding.value_kind)
    c.flags = int(bounding.flags)
    c.min_value = float(bounding.min_value)
    c.max_value = float(bounding.max_value)
    c.middle = float(bounding.middle)
    c.min_sum = float(bounding.min_sum)
    c.max_sum = float(bounding.max_sum)
    c.row_offset = int(row_offset)
    c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    c.algorithm = int(algorithm)
    c.merge = int(merge)
    c.max_contributions = int(bounding.max_contributions or 0)
    c.rows_are_units = 1 if bounding.rows_are_units else 0
    c.key_format = int(key_format)
    c.sieve = int(sieve)
    c.sieve_band = int(sieve_band)
    c.sieve_threads = int(sieve_threads)
    c.bucket_threads = int(bucket_threads)
    return c


def bound_plan(n_rows, n_privacy_ids, n_partitions, bounding: BoundingSpec,
               algorithm: int = N.ALGO_AUTO, merge: int = N.MERGE_AUTO,
               key_format: int = N.KEYS_AUTO, sieve: int = 0, sieve_band: int = 0,
               sieve_threads: int = 0, bucket_threads: int = 0) -> N.BoundPlanInfo:
    """Execution plan the library resolves for this shard (no device work)."""
    cfg = bound_config(n_rows, n_privacy_ids, n_partitions, bounding, 0, 0, algorithm, merge, key_format, sieve,
                       sieve_band, sieve_threads, bucket_threads)
    return bound_plan_info(cfg)


def bound_plan_info(cfg) -> N.BoundPlanInfo:
    """pdp_bound_plan of a built pdp_bound_config."""
    info = N.BoundPlanInfo()
    N.check(N.lib().pdp_bound_plan(ctypes.byref(cfg), ctypes.byref(info)), "pdp_bound_plan")
    return info


class BoundWorkspace:
    """Reusable device workspace for pdp_bound_contributions."""

    def __init__(self):
        self.buf = None
        self.last_cfg = None
        self._err_host = None   # pinned u32: the deferred copy of the error word
        self._err_event = None  # recorded after that copy
        self._err_keys = None   # (n_privacy_ids, n_partitions) for the message

    def defer_error_check(self, ws, sobj, n_privacy_ids, n_partitions):
        torch = _torch()
        if self._err_event is not None:  # an unread check: read it first (its copy owns the block)
            self.raise_deferred()
        if self._err_host is None:
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        N.check(N.lib().pdp_bound_error_flags_async(_ptr(ws), ctypes.c_void_p(self._err_host.data_ptr()),
                                                    int(sobj.cuda_stream)), "pdp_bound_error_flags_async")
        self._err_event = torch.cuda.Event()
        self._err_event.record(sobj)
        self._err_keys = (n_privacy_ids, n_partitions)

    def raise_deferred(self):
        ev, self._err_event = self._err_event, None
        if ev is None:
            return
        ev.synchronize()
        _raise_error_flags(int(self._err_host.item()) & 0xFFFFFFFF, *self._err_keys)

    def stats(self, stream=None) -> dict:
        """pdp_bound_stats_read of the last bound_and_reduce on this workspace
        (synchronises): rows through the partition passes, the sieve's
        unresolved privacy ids and fix-up rows."""
        if self.last_cfg is None or self.buf is None:
            raise RuntimeError("no bound_and_reduce has run on this workspace")
        out = N.BoundStats()
        N.check(N.lib().pdp_bound_stats_read(ctypes.byref(self.last_cfg), _ptr(self.buf), self.buf.numel(),
                                             ctypes.byref(out), _stream(stream)), "pdp_bound_stats_read")
        return {"rows_partitioned": out.rows_partitioned, "unresolved_ids": out.unresolved_ids,
                "fixup_rows": out.fixup_rows, "sieve": out.sieve, "error_flags": out.error_flags,
                "band_rows": out.band_rows, "unresolved2_ids": out.unresolved2_ids,
                "fixup2_rows": out.fixup2_rows, "band": out.band}

    def get(self, nbytes: int, device, probe=None, stream=None):
        """The workspace (grown when too small).  probe(buf) -> None runs a
        level-1 pass into `buf`: with it, a new workspace of at least
        PLACEMENT_PROBE_MIN bytes is placed by measurement (_place)."""
        torch = _torch()
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != device:
            self.buf = None
            size = max(int(nbytes), 256)
            if probe is not None and size >= PLACEMENT_PROBE_MIN and PLACEMENT_PROBE > 1:
                self.buf = _place(size, device, probe,
                                  stream if stream is not None else torch.cuda.current_stream(device))
            else:
                self.buf = torch.empty(size, dtype=torch.uint8, device=device)
        return self.buf


# Workspace placement ("Level 1's placement").  Level 1's rate
# depends on where the driver places a large workspace: in one process, the
# same C3 level 1 ran at 3.12-3.80 ms on workspaces allocated side by side
# (the input columns unchanged; profiles/r06/ab/ab4_l1_mode_probe.txt), and
# each workspace kept its speed.  So a new workspace of at least
# PLACEMENT_PROBE_MIN bytes is chosen among up to PLACEMENT_PROBE candidates
# held at once (as free memory allows), by one timed level-1 pass each (the
# PDP_PROBE_LEVEL1 flag; the call that asked for the workspace then runs
# normally on the winner).  One-time cost per workspace (C3: ~7 x 7 ms);
# PIPELINEDP_AMD_PLACEMENT_PROBE=1 turns it off.  The choice affects speed only.
# (About one candidate in five after the first was fast in round 6's probes,
# profiles/r06/ab/ab10_*: up to 8, i.e. as many as fit -- 7 at C3 on 288 GB.)
PLACEMENT_PROBE = int(os.environ.get("PIPELINEDP_AMD_PLACEMENT_PROBE", "8"))
PLACEMENT_PROBE_MIN = 2 << 30


def _place(size, device, probe, sobj):
    torch = _torch()
    free, _ = torch.cuda.mem_get_info(device)
    k = max(1, min(PLACEMENT_PROBE, int((free - (4 << 30)) // size)))
    cands, times = [], []
    for _ in range(k):
        buf = torch.empty(size, dtype=torch.uint8, device=device)
        probe(buf)  # warm
        # the faster of two timed passes: one pass read 0.08-0.26 ms above the
        # level-1 time later measured on the chosen buffer (profiles/r06/ab/ab24_*)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(sobj)
        probe(buf)
        ev[1].record(sobj)
        probe(buf)
        ev[2].record(sobj)
        ev[2].synchronize()
        cands.append(buf)
        times.append(min(ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))
    best = min(range(k), key=lambda i: times[i])
    keep = cands[best]
    del cands
    if k > 1:
        torch.cuda.empty_cache()  # the other candidates back to the driver
    _placement_log.append({"candidates_ms": [round(t, 4) for t in times], "chosen": best, "bytes": size})
    return keep


_placement_log = []  # diagnostics (bench.py reports it)


# Plan feedback ("light users").  The threshold sieve leaves
# privacy ids with fewer than l0 distinct pairs below its threshold for a
# fix-up; an id short of l0 pairs below the side band's 2t as well needs its
# rows re-read from the whole privacy-id column, and past RESCAN_BLOOM_MAX such
# ids that re-read tests every row against an L2-resident bitmap (C3 with 30 %
# of the ids holding 1-3 rows: 16.4 ms sieved against 12.9 ms unsieved,
# DESIGN.md §3 "Light users").  Whether a table is like that shows in the
# fix-up's counters, which pdp_bound_stats_async copies to pinned host memory
# at the end of every sieved call without synchronising; the next call on the
# same resident columns reads them (once their copy has completed) and, when
# the re-read was of the slow kind, runs the auto plan without the sieve.  The
# choice changes only speed: every plan computes the same result.  Every
# FEEDBACK_REPROBE-th unsieved call tries the sieve again, so a table whose
# contents changed in place is re-measured.
RESCAN_BLOOM_MAX = 8192  # pdp_bound.hip kBloomMaxIds: above it the re-read tests a bitmap per row
FEEDBACK_REPROBE = 64
# Entries live as long as the key columns: a weak map from the partition-key
# tensor object to its entries (keyed by the privacy-id tensor's identity, the
# columns' in-place version counters and the bounding parameters), so a table
# allocated at a freed table's address starts fresh and an in-place write to
# the columns through torch re-measures.  The counters sit in slots of one
# pinned block the process never frees: a dropped entry whose copy is still
# in flight returns its slot only once the copy's event has completed
# (a freed pinned block could be handed out again under a
# pending device-to-host copy).
_feedback = {}  # id(partition-key tensor) -> (weak reference to it, {key: (pid ref, _PlanFeedback)})
_FB_SLOTS = 1024
_fb_pool = None          # pinned int32 [_FB_SLOTS, 4]
_fb_free = []            # free slot indices
_fb_draining = []        # (slot, event): slots of dropped entries whose copy may be pending


def _fb_take_slot():
    global _fb_pool
    torch = _torch()
    if _fb_pool is None:
        _fb_pool = torch.zeros((_FB_SLOTS, 4), dtype=torch.int32, pin_memory=True)
        _fb_free.extend(range(_FB_SLOTS))
    for item in [d for d in _fb_draining if d[1] is None or d[1].query()]:
        _fb_draining.remove(item)
        _fb_free.append(item[0])
    return _fb_free.pop() if _fb_free else None


def _fb_release(state):
    """weakref.finalize callback of a dropped _PlanFeedback (state: [slot, event])."""
    slot, event = state
    if slot is not None:
        _fb_draining.append((slot, event))


class _PlanFeedback:
    def __init__(self, slot):
        self.slot = slot
        self.host = _fb_pool[slot]  # uint32 counters (read & 0xFFFFFFFF)
        self.state = [slot, None]   # [slot, event recorded after the copies into `host`]
        self.band = False    # the measured plan had the side band
        self.unsieved = False
        self.calls = 0
        self.sieved_calls = 0
        weakref.finalize(self, _fb_release, self.state)

    @property
    def event(self):
        return self.state[1]

    @event.setter
    def event(self, ev):
        self.state[1] = ev

    def idle(self) -> bool:
        """No copy into `host` is pending."""
        return self.event is None or self.event.query()


def _feedback_entries(pk, create=False):
    """The entries of this tensor object (identity, not equality: tensors
    compare elementwise); dropped when the tensor is freed."""
    e = _feedback.get(id(pk))
    if e is not None and e[0]() is pk:
        return e[1]
    if not create:
        return None
    d = {}
    _feedback[id(pk)] = (weakref.ref(pk), d)
    weakref.finalize(pk, _feedback.pop, id(pk), None)
    return d


def _feedback_key(pid, pk, n, U, P, bounding, row_offset):
    return (id(pid), None if pid is None else pid._version, pk._version, n, int(U), int(P), int(bounding.l0),
            int(bounding.linf), int(bounding.flags), int(row_offset))


def _feedback_get(pid, pk, key):
    d = _feedback_entries(pk)
    e = None if d is None else d.get(key)
    if e is None:
        return None
    pid_ref, fb = e
    if (pid_ref() if pid_ref is not None else None) is not pid:  # another privacy-id tensor at that id
        return None
    return fb


def _feedback_sieve(pid, pk, key) -> int:
    """The sieve argument the auto plan takes for these columns: 0 (auto) or
    -1 (off) after a measured call whose re-read covered many ids."""
    fb = _feedback_get(pid, pk, key)
    if fb is None:
        return 0
    if fb.event is not None and fb.event.query():
        c = [v & 0xFFFFFFFF for v in fb.host.tolist()]
        slow = (c[2] if fb.band else c[0]) > RESCAN_BLOOM_MAX
        fb.unsieved = fb.unsieved or slow
        fb.event = None
    if not fb.unsieved:
        return 0
    fb.calls += 1
    if fb.calls % FEEDBACK_REPROBE == 0:
        fb.unsieved = False  # measure the sieved plan again
        fb.sieved_calls = 0  # (its counters are read: the next sieved call arms the copy)
        return 0
    return -1


def plan_feedback_state(pid, pk, *, n_privacy_ids, n_partitions, bounding, row_offset=0):
    """Tests / diagnostics: None, or {"unsieved": bool, "pending": bool}."""
    fb = _feedback_get(pid, pk, _feedback_key(pid, pk, int(pk.shape[0]), n_privacy_ids, n_partitions, bounding,
                                              row_offset))
    return None if fb is None else {"unsieved": fb.unsieved, "pending": fb.event is not None}


def bound_and_reduce(pid, pk, value, *, n_privacy_ids: int, n_partitions: int,
                     bounding: BoundingSpec, seed: int, row_offset: int = 0, allowed=None,
                     acc=None, workspace: Optional[BoundWorkspace] = None, stream=None,
                     check_keys=True, timer: Optional["StageTimer"] = None,
                     algorithm: int = N.ALGO_AUTO, merge: int = N.MERGE_AUTO,
                     key_format: int = N.KEYS_AUTO, sieve: int = 0, sieve_band: int = 0,
                     sieve_threads: int = 0, bucket_threads: int = 0):
    """Bounds contributions of one shard and ADDS its per-partition accumulators.

    pid, pk: int64 device tensors of length n (dense keys; pid may be None
    with bounding.rows_are_units); value: float64 or int64 device tensor (or
    None for COUNT/PRIVACY_ID_COUNT only).  Returns the accumulator dict.
    """
    torch = _torch()
    lib = N.lib()
    device = pk.device
    n = int(pk.shape[0])
    if pid is None and not bounding.rows_are_units:
        raise ValueError("privacy_id is required unless contribution bounds are already enforced")
    if pid is not None:
        _check_col(pid, "privacy_id", (torch.int64,), n, device)
    _check_col(pk, "partition_key", (torch.int64,), n, device)
    if bounding.value_kind == N.VALUE_F64:
        _check_col(value, "value", (torch.float64,), n, device)
    elif bounding.value_kind == N.VALUE_I64:
        _check_col(value, "value", (torch.int64,), n, device)
    else:
        value = None
    if allowed is not None:
        _check_col(allowed, "pk_allowed", (torch.uint8,), int(n_partitions), device)
    if bounding.l0 < 0 or bounding.l0 > N.MAX_L0:
        raise NotImplementedError(f"max_partitions_contributed={bounding.l0} is outside the "
                                  f"supported range [1, {N.MAX_L0}]")
    if bounding.max_contributions < 0 or bounding.max_contributions > N.MAX_CONTRIBUTIONS:
        raise NotImplementedError(f"max_contributions={bounding.max_contributions} is outside the "
                                  f"supported range [1, {N.MAX_CONTRIBUTIONS}]")
    if bounding.linf < 0 or bounding.linf > N.MAX_LINF:
        raise NotImplementedError(f"max_contributions_per_partition={bounding.linf} is outside "
                                  f"the supported range [1, {N.MAX_LINF}]")
    if check_keys == "defer" and workspace is None:  # nowhere to leave the deferred word
        check_keys = True
    feedback = (sieve == 0 and algorithm == N.ALGO_AUTO and n > 0)
    fkey = _feedback_key(pid, pk, n, n_privacy_ids, n_partitions, bounding, row_offset) if feedback else None
    if feedback:
        sieve = _feedback_sieve(pid, pk, fkey)
    cfg = bound_config(n, n_privacy_ids, n_partitions, bounding, seed, row_offset, algorithm, merge,
                       key_format, sieve, sieve_band, sieve_threads, bucket_threads)
    nbytes = ctypes.c_uint64(0)
    N.check(lib.pdp_bound_workspace_bytes(ctypes.byref(cfg), ctypes.byref(nbytes)),
            "pdp_bound_workspace_bytes")
    wsobj = workspace or BoundWorkspace()
    s_probe = stream if stream is not None else torch.cuda.current_stream(device)
    st_probe = int(s_probe.cuda_stream)

    def probe(buf):  # level 1 alone into a candidate workspace (placement)
        pc = bound_config(n, n_privacy_ids, n_partitions, bounding, seed, row_offset, algorithm, merge,
                          key_format, sieve, sieve_band, sieve_threads, bucket_threads)
        pc.flags = int(pc.flags) | N.PROBE_LEVEL1
        N.check(lib.pdp_bound_contributions(ctypes.byref(pc), _ptr(pid), _ptr(pk), _ptr(value), _ptr(allowed),
                                            _ptr(buf), buf.numel(), st_probe), "pdp_bound_contributions (probe)")
    ws = wsobj.get(nbytes.value, device, probe=probe if pid is not None else None, stream=s_probe)
    wsobj.last_cfg = cfg
    if acc is None:
        acc = new_accumulators(n_partitions, bounding, device)
    # one stream object for the launches and for every event recorded after them
    sobj = stream if stream is not None else torch.cuda.current_stream(device)
    st = int(sobj.cuda_stream)
    _mark(timer, "bound")
    N.check(lib.pdp_bound_contributions(ctypes.byref(cfg), _ptr(pid), _ptr(pk), _ptr(value),
                                        _ptr(allowed), _ptr(ws), ws.numel(), st),
            "pdp_bound_contributions")
    _mark(timer, "reduce")
    if check_keys == "defer":
        # the error word copied into pinned memory behind the launches; read by
        # raise_key_errors() once the caller synchronises anyway (the public
        # API: when the result is materialised), so no drain here
        wsobj.defer_error_check(ws, sobj, n_privacy_ids, n_partitions)
    elif check_keys:
        flags = ctypes.c_uint32(0)
        N.check(lib.pdp_bound_error_flags(_ptr(ws), ctypes.byref(flags), st), "pdp_bound_error_flags")
        _raise_error_flags(flags.value, n_privacy_ids, n_partitions)
    N.check(lib.pdp_reduce_partitions(ctypes.byref(cfg), _ptr(value), _ptr(ws), ws.numel(),
                                      ctypes.byref(_acc_struct(acc)), st),
            "pdp_reduce_partitions")
    if feedback and sieve == 0:
        info = bound_plan_info(cfg)
        if info.sieve:  # a sieved call: its fix-up counters for the next one
            fb = _feedback_get(pid, pk, fkey)
            if fb is None:
                slot = _fb_take_slot()
                if slot is not None:
                    entries = _feedback_entries(pk, create=True)
                    if len(entries) > 16:  # the same columns under many parameter sets: keep the newest
                        entries.clear()
                    fb = _PlanFeedback(slot)
                    entries[fkey] = (None if pid is None else weakref.ref(pid), fb)
            if fb is not None:
                fb.sieved_calls += 1
            # counters of the first sieved call, then of every FEEDBACK_REPROBE-th
            # (a copy per call would cost a stream slot each time for no news)
            if fb is not None and fb.event is None and (fb.sieved_calls - 1) % FEEDBACK_REPROBE == 0:
                N.check(lib.pdp_bound_stats_async(ctypes.byref(cfg), _ptr(ws), ws.numel(),
                                                  ctypes.c_void_p(fb.host.data_ptr()), st),
                        "pdp_bound_stats_async")
                fb.band = bool(info.band)
                fb.event = torch.cuda.Event()
                fb.event.record(sobj)
    _mark(timer, "end_bound")
    return acc


def _raise_error_flags(flags: int, n_privacy_ids, n_partitions):
    if flags & 1:
        raise ValueError("privacy_id / partition_key outside the dense key range "
                         f"[0, {n_privacy_ids}) x [0, {n_partitions})")
    if flags & 2:
        raise N.NativeLibraryError("the sieve's fix-up row list outgrew its workspace region "
                                   "(pdp_bound_error_flags bit 1; a library bug)")


def raise_key_errors(workspace: "BoundWorkspace"):
    """The deferred key check of the last bound_and_reduce(check_keys="defer")
    on `workspace`: waits for its error-word copy (the caller has normally
    synchronised already) and raises as check_keys=True would have."""
    workspace.raise_deferred()


_tables = {}


def _device_table(values, device):
    """The truncated-geometric keep table on `device`, copied once per
    (device, contents): a pageable host-to-device copy per call would
    synchronise the stream between bounding and selection."""
    torch = _torch()
    arr = np.ascontiguousarray(values, dtype=np.float64)
    key = (str(device), arr.tobytes())
    t = _tables.get(key)
    if t is None:
        if len(_tables) > 64:
            _tables.clear()
        t = _tables[key] = torch.from_numpy(arr.copy()).to(device)  # (the cached table is read-only)
    return t


def select_and_noise(acc, *, selection: SelectionSpec, ops: List[MetricOpSpec], n_cols: int,
                     seed_select: int, seed_noise: int, partition_offset: int = 0,
                     public_mask=None, stream=None, sync_count: bool = True,
                     timer: Optional["StageTimer"] = None):
    """Selects partitions and computes the noisy metrics of the kept ones.

    Returns (index[n_kept] int64 device, out[n_cols, P] float64 device, n_kept)
    where only the first n_kept columns of `out` are valid.  With
    sync_count=False n_kept is returned as a device int64[1] tensor.
    """
    torch = _torch()
    lib = N.lib()
    rc = acc["privacy_id_count"]
    device = rc.device
    P = int(rc.shape[0])
    st = _stream(stream)
    keep = torch.empty(P, dtype=torch.uint8, device=device)
    noised = torch.empty(P, dtype=torch.float64, device=device) if selection.want_noised_count else None
    table = None
    sc = N.SelectConfig()
    sc.n_partitions = P
    sc.partition_offset = int(partition_offset)
    sc.strategy = int(selection.strategy)
    sc.max_rows_per_privacy_id = int(selection.max_rows_per_privacy_id)
    sc.pre_threshold = int(selection.pre_threshold or 0)
    if selection.strategy == N.SELECT_TRUNCATED_GEOMETRIC:
        table = _device_table(selection.keep_prob, device)
        sc.keep_table_len = int(table.numel())
        sc.keep_prob = _ptr(table)
    sc.noise = (selection.noise or NO_NOISE).to_c()
    sc.threshold = float(selection.threshold)
    if selection.strategy == N.SELECT_PUBLIC:
        if public_mask is None:
            raise ValueError("public_mask is required for public partitions")
        _check_col(public_mask, "public_mask", (torch.uint8,), P, device)
        sc.public_mask = _ptr(public_mask)
    sc.seed = int(seed_select) & 0xFFFFFFFFFFFFFFFF
    _mark(timer, "select")
    N.check(lib.pdp_select_partitions(ctypes.byref(sc), _ptr(rc), _ptr(keep), _ptr(noised), st),
            "pdp_select_partitions")
    cbytes = ctypes.c_uint64(0)
    N.check(lib.pdp_compact_workspace_bytes(P, ctypes.byref(cbytes)), "pdp_compact_workspace_bytes")
    cws = torch.empty(int(cbytes.value), dtype=torch.uint8, device=device)
    index = torch.empty(max(P, 1), dtype=torch.int64, device=device)
    n_kept_dev = torch.empty(1, dtype=torch.int64, device=device)  # pdp_compact writes it
    N.check(lib.pdp_compact(_ptr(keep), P, _ptr(index), _ptr(n_kept_dev), _ptr(cws), cws.numel(), st),
            "pdp_compact")
    out = torch.empty((max(n_cols, 1), max(P, 1)), dtype=torch.float64, device=device)
    if len(ops) > N.MAX_OPS:
        raise NotImplementedError(f"at most {N.MAX_OPS} combiners are supported")
    c_ops = (N.MetricOp * max(len(ops), 1))(*[o.to_c() for o in ops])
    N.check(lib.pdp_noise_metrics(c_ops, len(ops), _ptr(index), P, _ptr(n_kept_dev),
                                  int(partition_offset), ctypes.byref(_acc_struct(acc)),
                                  1 if (acc["sum"] is not None and acc["sum"].dtype == torch.int64) else 0,
                                  _ptr(noised), _ptr(out), out.shape[1],
                                  int(seed_noise) & 0xFFFFFFFFFFFFFFFF, st),
            "pdp_noise_metrics")
    _mark(timer, "end_select")
    if sync_count:
        n_kept = int(n_kept_dev.item())
        return index[:n_kept], out, n_kept
    return index, out, n_kept_dev


def kept_to_host(index, out, n_kept: int, keys_only: bool = False):
    """(index[:n_kept], out[:, :n_kept]) as host NumPy arrays through ONE
    packed device copy and ONE device-to-host copy into pinned memory (the
    public API's result; two pageable copies of a strided view cost two more
    synchronisations)."""
    torch = _torch()
    n_cols = 0 if keys_only else int(out.shape[0])
    if n_kept == 0:
        return np.zeros(0, dtype=np.int64), np.zeros((n_cols, 0))
    rows = [index[:n_kept].view(torch.float64).unsqueeze(0)]
    if n_cols:
        rows.append(out[:, :n_kept])
    packed = torch.cat(rows) if len(rows) > 1 else rows[0]
    global _pinned_out
    need = packed.numel()
    if _pinned_out is None or _pinned_out.numel() < need:  # grow-only: no pinned allocation per call
        _pinned_out = torch.empty(max(need, 1 << 16), dtype=torch.float64, pin_memory=True)
    host = _pinned_out[:need].view(packed.shape)
    host.copy_(packed, non_blocking=True)
    torch.cuda.current_stream(index.device).synchronize()
    h = host.numpy()
    return h[0].view(np.int64).copy(), h[1:].copy()


_pinned_out = None  # kept_to_host's pinned staging block


def kept_to_host_guess(index, out, n_kept_dev, keys_only: bool = False, key=None):
    """kept_to_host with the kept count still on the device: the count and
    the first K kept columns leave in ONE device-to-host copy and one stream
    synchronisation (K = 1.25 x the kept count of the last call with the same
    `key`, at least 4,096); only a call keeping more than K partitions pays a
    second round trip for the rest.  Returns (index, values, n_kept)."""
    torch = _torch()
    P = int(index.shape[0])
    n_cols = 0 if keys_only else int(out.shape[0])
    K = min(P, max(4096, int(_kept_guess.get(key, 0) * 1.25) + 1))
    buf = torch.empty(1 + (n_cols + 1) * K, dtype=torch.float64, device=index.device)
    buf[0:1].copy_(n_kept_dev.view(torch.float64))
    buf[1:1 + K].copy_(index[:K].view(torch.float64))
    if n_cols:
        buf[1 + K:].view(n_cols, K).copy_(out[:, :K])
    global _pinned_out
    need = buf.numel()
    if _pinned_out is None or _pinned_out.numel() < need:
        _pinned_out = torch.empty(max(need, 1 << 16), dtype=torch.float64, pin_memory=True)
    host = _pinned_out[:need]
    host.copy_(buf, non_blocking=True)
    torch.cuda.current_stream(index.device).synchronize()
    h = host.numpy()
    n_kept = int(h[0:1].view(np.int64)[0])
    _kept_guess[key] = n_kept
    if n_kept > K:  # more kept than guessed: the exact path
        idx, vals = kept_to_host(index, out, n_kept, keys_only=keys_only)
        return idx, vals, n_kept
    idx = h[1:1 + n_kept].view(np.int64).copy()
    vals = h[1 + K:].reshape(n_cols, K)[:, :n_kept].copy() if n_cols else np.zeros((0, n_kept))
    return idx, vals, n_kept


_kept_guess = {}  # kept_to_host_guess: last kept count per caller key


def add_noise(values, *, noise: NoiseParams, seed: int, index_offset: int = 0, out=None, stream=None):
    """DPEngine.add_dp_noise's "Add noise" stage (dp_engine.py:595-599) on a
    device column: returns the float64 values through the secure mechanism
    `noise` (Laplace / Gaussian, granularity-snapped), element i drawing from
    the Philox streams (seed, index_offset + i) (`pdp_add_noise`)."""
    torch = _torch()
    lib = N.lib()
    if not values.is_cuda:
        raise ValueError("values must be a device tensor")
    if values.dtype not in (torch.int64, torch.float64):
        raise ValueError("values must be int64 or float64")
    values = values.contiguous()
    n = int(values.numel())
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=values.device)
    _check_col(out, "out", (torch.float64,), n, values.device)
    vk = N.VALUE_I64 if values.dtype == torch.int64 else N.VALUE_F64
    c_noise = noise.to_c()
    N.check(lib.pdp_add_noise(_ptr(values), vk, n, ctypes.byref(c_noise),
                              int(seed) & 0xFFFFFFFFFFFFFFFF, int(index_offset), _ptr(out), _stream(stream)),
            "pdp_add_noise")
    return out


def dataset_histograms(pid, pk, value, *, n_privacy_ids: int, n_partitions: int, stream=None,
                       workspace: Optional[BoundWorkspace] = None, group=None,
                       force_pair_table: bool = False,
                       force_pair_hash: bool = False) -> Dict[str, "torch.Tensor"]:
    """compute_dataset_histograms (computing_histograms.py:456-513) on device
    columns of dense codes (`pdp_dataset_histograms`): returns the raw device
    bin arrays (int_count/int_sum/int_max [5, LOG_BINS], float_count/
    float_sum/float_max [2, SUM_BUCKETS], float_lowers [2, SUM_BUCKETS + 1],
    float_n_lowers [2]); pipelinedp_amd.dataset_histograms turns them into
    Histogram objects.  Under torch.distributed (rows sharded by privacy id,
    dense codes global) every rank returns the merged, global bins."""
    torch = _torch()
    lib = N.lib()
    if not pk.is_cuda:
        raise ValueError("columns must be device tensors")
    device = pk.device
    n = int(pk.numel())
    _check_col(pid, "privacy_id", (torch.int64,), n, device)
    _check_col(pk, "partition", (torch.int64,), n, device)
    vk = N.VALUE_NONE
    if value is not None:
        _check_col(value, "value", (torch.int64, torch.float64), n, device)
        vk = N.VALUE_I64 if value.dtype == torch.int64 else N.VALUE_F64
    if force_pair_table:  # tests: the HBM pair-table path instead of the buckets
        vk |= N.HIST_FORCE_PAIR_TABLE
    if force_pair_hash:   # tests: pair-keyed buckets instead of privacy-id buckets
        vk |= N.HIST_FORCE_PAIR_HASH
    nbytes = ctypes.c_uint64()
    N.check(lib.pdp_dataset_histograms_workspace_bytes(n, int(n_privacy_ids), int(n_partitions),
                                                      ctypes.byref(nbytes)),
            "pdp_dataset_histograms_workspace_bytes")
    ws = (workspace or BoundWorkspace()).get(nbytes.value, device)
    out = _histogram_outputs(device)
    s = N.HistogramBins(**{k: _ptr(v) for k, v in out.items()})
    from pipelinedp_amd import parallel
    world, rank = parallel.world_info(group)
    args = (int(n_privacy_ids), int(n_partitions))
    if world == 1:
        N.check(lib.pdp_dataset_histograms(_ptr(pid), _ptr(pk), _ptr(value) if value is not None else None, vk, n,
                                           *args, ctypes.byref(s), _ptr(ws), int(ws.numel()), _stream(stream)),
                "pdp_dataset_histograms")
    else:
        # rows sharded by privacy id: pid- and pair-level statistics are
        # complete per rank; partition statistics and the pair-sum range are
        # reduced between the phases, then the bins are merged
        # each rank passes its own value kind: the kernels sum int64 and fp64
        # values alike in fp64, so the ranks' partition sums add up
        N.check(lib.pdp_dataset_histograms_pairs(_ptr(pid), _ptr(pk), _ptr(value) if value is not None else None,
                                                 vk, n, *args, ctypes.byref(s), _ptr(ws), int(ws.numel()),
                                                 _stream(stream)),
                "pdp_dataset_histograms_pairs")
        offs = [ctypes.c_uint64() for _ in range(3)]
        N.check(lib.pdp_dataset_histograms_exchange_offsets(n, *args, *[ctypes.byref(o) for o in offs]),
                "pdp_dataset_histograms_exchange_offsets")
        P = int(n_partitions)
        pkstat = ws[offs[0].value:offs[0].value + 8 * P].view(torch.int64)
        psum = ws[offs[1].value:offs[1].value + 8 * P].view(torch.float64)
        minmax = ws[offs[2].value:offs[2].value + 16].view(torch.int64)
        parallel.exchange_histogram_stats(pkstat, psum, minmax, group)
        N.check(lib.pdp_dataset_histograms_finish(vk, n, *args, 1 if rank == 0 else 0, ctypes.byref(s), _ptr(ws),
                                                  int(ws.numel()), _stream(stream)),
                "pdp_dataset_histograms_finish")
        parallel.merge_histogram_bins(out, group)
    out["workspace"] = ws
    return out


def _histogram_outputs(device):
    torch = _torch()
    i64 = dict(dtype=torch.int64, device=device)
    f64 = dict(dtype=torch.float64, device=device)
    return {
        "int_count": torch.empty((N.HIST_N_INT, N.HIST_LOG_BINS), **i64),
        "int_sum": torch.empty((N.HIST_N_INT, N.HIST_LOG_BINS), **i64),
        "int_max": torch.empty((N.HIST_N_INT, N.HIST_LOG_BINS), **i64),
        "float_count": torch.empty((N.HIST_N_FLOAT, N.HIST_SUM_BUCKETS), **i64),
        "float_sum": torch.empty((N.HIST_N_FLOAT, N.HIST_SUM_BUCKETS), **f64),
        "float_max": torch.empty((N.HIST_N_FLOAT, N.HIST_SUM_BUCKETS), **f64),
        "float_lowers": torch.empty((N.HIST_N_FLOAT, N.HIST_SUM_BUCKETS + 1), **f64),
        "float_n_lowers": torch.empty(N.HIST_N_FLOAT, dtype=torch.int32, device=device),
    }


def dataset_histograms_preaggregated(pk, count, total, n_partitions_of_pid, n_contributions_of_pid, *,
                                     n_partitions: int, stream=None,
                                     workspace: Optional[BoundWorkspace] = None,
                                     group=None) -> Dict[str, "torch.Tensor"]:
    """compute_dataset_histograms_on_preaggregated_data (computing_histograms.py:
    713-758) on device columns, one row per (privacy id, partition) pair
    (`pdp_dataset_histograms_preaggregated`): pk (dense codes), count (rows of
    the pair), total (their value sum, fp64), and the pair's privacy id's
    n_partitions / n_contributions.  Returns the raw device bin arrays of
    `dataset_histograms`.  Under torch.distributed (the rows of one privacy id
    on one rank, partition codes global) every rank returns the merged bins."""
    torch = _torch()
    lib = N.lib()
    if not pk.is_cuda:
        raise ValueError("columns must be device tensors")
    device = pk.device
    n = int(pk.numel())
    _check_col(pk, "partition", (torch.int64,), n, device)
    _check_col(count, "count", (torch.int64,), n, device)
    _check_col(total, "sum", (torch.float64,), n, device)
    _check_col(n_partitions_of_pid, "n_partitions", (torch.int64,), n, device)
    _check_col(n_contributions_of_pid, "n_contributions", (torch.int64,), n, device)
    nbytes = ctypes.c_uint64()
    N.check(lib.pdp_dataset_histograms_preaggregated_workspace_bytes(n, int(n_partitions), ctypes.byref(nbytes)),
            "pdp_dataset_histograms_preaggregated_workspace_bytes")
    ws = (workspace or BoundWorkspace()).get(nbytes.value, device)
    out = _histogram_outputs(device)
    s = N.HistogramBins(**{k: _ptr(v) for k, v in out.items()})
    cols = (_ptr(pk), _ptr(count), _ptr(total), _ptr(n_partitions_of_pid), _ptr(n_contributions_of_pid))
    from pipelinedp_amd import parallel
    world, rank = parallel.world_info(group)
    P = int(n_partitions)
    if world == 1:
        N.check(lib.pdp_dataset_histograms_preaggregated(*cols, n, P, ctypes.byref(s), _ptr(ws), int(ws.numel()),
                                                         _stream(stream)),
                "pdp_dataset_histograms_preaggregated")
    else:
        N.check(lib.pdp_dataset_histograms_preaggregated_rows(*cols, n, P, ctypes.byref(s), _ptr(ws),
                                                              int(ws.numel()), _stream(stream)),
                "pdp_dataset_histograms_preaggregated_rows")
        offs = [ctypes.c_uint64() for _ in range(4)]
        N.check(lib.pdp_dataset_histograms_preaggregated_exchange_offsets(n, P, *[ctypes.byref(o) for o in offs]),
                "pdp_dataset_histograms_preaggregated_exchange_offsets")
        pk_rows = ws[offs[0].value:offs[0].value + 8 * P].view(torch.int64)
        pk_count = ws[offs[1].value:offs[1].value + 8 * P].view(torch.int64)
        psum = ws[offs[2].value:offs[2].value + 8 * P].view(torch.float64)
        minmax = ws[offs[3].value:offs[3].value + 16].view(torch.int64)
        parallel.exchange_preaggregated_stats(pk_rows, pk_count, psum, minmax, group)
        # L0 / L1 weight sums: global before rounding (one owner rank per value)
        woff = [ctypes.c_uint64() for _ in range(3)]
        N.check(lib.pdp_dataset_histograms_preaggregated_weight_offsets(n, P, *[ctypes.byref(o) for o in woff]),
                "pdp_dataset_histograms_preaggregated_weight_offsets")
        wsmall = ws[woff[0].value:woff[0].value + 8 * 2000].view(torch.float64)
        slots = woff[2].value
        wtab = ws[woff[1].value:woff[1].value + 16 * slots].view(torch.int64).view(slots, 2)
        wkeys, wsums = parallel.exchange_preaggregated_weights(wsmall, wtab, group)
        N.check(lib.pdp_dataset_histograms_preaggregated_finish(_ptr(total), n, P, 1 if rank == 0 else 0,
                                                                ctypes.byref(s), _ptr(ws), int(ws.numel()),
                                                                _stream(stream)),
                "pdp_dataset_histograms_preaggregated_finish")
        wkeys, wsums = wkeys.contiguous(), wsums.contiguous()
        N.check(lib.pdp_dataset_histograms_weight_bins(_ptr(wkeys), _ptr(wsums), int(wkeys.numel()),
                                                       ctypes.byref(s), _stream(stream)),
                "pdp_dataset_histograms_weight_bins")
        parallel.merge_histogram_bins(out, group)
    out["workspace"] = ws
    return out

