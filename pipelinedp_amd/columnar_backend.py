"""ColumnarBackend — the MI355X drop-in for LocalBackend on DPEngine.aggregate.

DPEngine builds the aggregation as a chain of backend calls with stable
stage names (reference dp_engine.py:109-187, contribution_bounders.py:72-111).
Every call here records a lazy plan node; nothing runs until the result is
iterated (after BudgetAccountant.compute_budgets(), when eps/delta exist).
Iteration recognises the chain, resolves the input columns, and runs the
whole aggregation through the HIP kernels:

    extract -> [public filter] -> bound (L0/Linf sampling) -> reduce per
    partition -> [public padding] -> [private selection] -> noisy metrics
    -> [post-aggregation threshold drop]

The recognised chain carries everything the kernels need: the combiner
(bound method ``create_accumulator`` / ``compute_metrics``), the selection
``functools.partial`` (budget, max_partitions, max_rows_per_privacy_id,
strategy, pre_threshold) and the AggregateParams passed to ``annotate``.
Both the reference's own DPEngine (pipeline_dp) and pipelinedp_amd.DPEngine
produce this chain.

Unsupported chains raise NotImplementedError (there is no row-wise CPU
fallback); so does a missing GPU or HIP library.
"""
import collections
import functools
import os
from typing import Any, List, Optional

import numpy as np

from pipelinedp_amd import _native as N
from pipelinedp_amd import columnar as C
from pipelinedp_amd import combiners as pdc
from pipelinedp_amd import dp_computations as dpc
from pipelinedp_amd import parallel
from pipelinedp_amd import partition_selection as ps
from pipelinedp_amd import pipeline_backend

# stage names DPEngine / the bounders use (reference file:line)
ST_EXTRACT = "Extract (privacy_id, partition_key, value))"          # dp_engine.py:415
ST_KEY_BY_PREFIX = "Key by partition"                                # pipeline_functions.py:25-27
ST_FILTER_KEYS = "Filtering out partitions"                          # dp_engine.py:294-295
ST_DROP_KEY = "Drop key"                                             # dp_engine.py:296
ST_DROP_PID = "Drop privacy id"                                      # dp_engine.py:140-141
ST_COMBINE = "Reduce accumulators per partition key"                 # dp_engine.py:158-159
ST_SELECT = "Filter private partitions"                              # dp_engine.py:371
ST_METRICS = "Compute DP metrics"                                    # dp_engine.py:181-182
ST_THRESHOLD_DROP = "Drop partitions under threshold"                # dp_engine.py:547-549
ST_PUBLIC_JOIN = "Join public partitions with partitions from data"  # dp_engine.py:311-313
ST_PUBLIC_TO_COL = "Public partitions to collection"                 # dp_engine.py:305-306
ST_EMPTY_ACCS = "Build empty accumulators"                           # dp_engine.py:307-309
# DPEngine.select_partitions (dp_engine.py:235-288)
ST_SP_EXTRACT = "Extract (privacy_id, partition_key))"               # :241-244
ST_SP_COMBINE = "Combine accumulators per partition key"             # :276-277
ST_SP_KEYS = "Drop accumulators, keep only partition keys"           # :286-287
# DPEngine.add_dp_noise
ST_ADD_NOISE = "Add noise"                                           # dp_engine.py:597-599
SELECT_PARTITIONS = {"Group by privacy_id", "Sample cross-partition contributions",
                     "Drop privacy id and add accumulator"}                          # :248-273

# bounder stage sets (contribution_bounders.py)
CROSS_AND_PER = {"Rekey to ( (privacy_id, partition_key), value))",
                 "Sample per (privacy_id, partition_key)",
                 "Apply aggregate_fn after per partition bounding",
                 "Rekey to (privacy_id, (partition_key, accumulator))",
                 "Sample per privacy_id", "Rekey by privacy_id and unnest"}          # :72-111
CROSS_ONLY = {"Rekey to ((privacy_id), (partition_key, value))", "Group by privacy_id",
              "Collect values per privacy_id and partition_key", "Sample",
              "Unnest per privacy_id",
              "Apply aggregate_fn after cross-partition contribution bounding"}     # :168-201
PER_PRIVACY_ID = {"Rekey to ((privacy_id), (partition_key, value))", "Sample per privacy_id",
                  "Collect values per privacy_id and partition_key", "Unnest",
                  "Apply aggregate_fn after per privacy_id contribution bounding"}  # :122-156
LINF_ONLY = {"Rekey to ((privacy_id, partition_key), value)",
             "Sample per (privacy_id, partition_key)",
             "Apply aggregate_fn after cross-partition contribution bounding"}      # :212-230
NOOP = {"Rekey to ((privacy_id, partition_key), value)", "Group by (privacy_id, partition_key)",
        "Apply aggregate_fn"}                                                       # :236-246
ALREADY_ENFORCED = {"Remove privacy_id", "Wrap values into accumulators"}          # dp_engine.py:144-150


class _Node:
    """A lazy collection: one recorded backend call."""

    def __init__(self, backend, op, parents, stage, fn=None, arg=None, kwargs=None):
        self.backend = backend
        self.op = op
        self.parents = parents
        self.stage = stage or ""
        self.fn = fn
        self.arg = arg
        self.kwargs = kwargs or {}
        self._result = None

    def __iter__(self):
        return iter(self.collect())

    def collect(self):
        """Executes the recognised graph once and returns its result: for
        DPEngine.aggregate a columnar.AggregateResult (a sequence of
        (partition_key, MetricsTuple) with `partition_keys` / `columns` arrays), for
        select_partitions the list of keys, for add_dp_noise the pairs."""
        if self._result is None:
            self._result = self.backend._execute(self)
        return self._result

    def __bool__(self):
        return True

    def __repr__(self):
        return f"<columnar {self.op} {self.stage!r}>"


def _enum_value(e):
    return getattr(e, "value", e)


class AggregatePlan:
    """What the recognised DPEngine.aggregate chain asks for."""

    def __init__(self):
        self.source = None
        self.extract_fn = None
        self.public_keys = None          # public partitions (filter) or None
        self.public_padding = None       # public partitions (padding) or None
        self.bounder = None              # "cross_and_per" | "cross" | "linf" | "noop" |
                                         # "per_privacy_id" | "already_enforced"
        self.linf_from_graph = None      # n of "Sample per (privacy_id, partition_key)"
        self.l0_from_graph = None        # n of "Sample per privacy_id" (Cross+Per: L0;
                                         # PerPrivacyId: max_contributions)
        self.combiner = None
        self.selection = None            # functools.partial of filter_fn
        self.compute_metrics = False
        self.threshold_drop = False
        self.params = None
        self.budget = None
        self.keys_only = False           # DPEngine.select_partitions: yield partition keys


def _chain(sink):
    nodes = []
    node = sink
    while isinstance(node, _Node):
        nodes.append(node)
        node = node.parents[0] if node.parents else None
    nodes.reverse()
    return nodes, node


class NoisePlan:
    """A recognised DPEngine.add_dp_noise chain (dp_engine.py:551-607):
    source of (partition_key, value) -> map_values "Add noise" -> annotate."""

    def __init__(self, source, noise_fn, params, budget):
        self.source = source
        self.noise_fn = noise_fn
        self.params = params
        self.budget = budget


def _closure_objects(fn, depth=0):
    """Objects captured by fn's closure, recursively through captured functions."""
    out = []
    for cell in getattr(fn, "__closure__", None) or ():
        try:
            obj = cell.cell_contents
        except ValueError:
            continue
        out.append(obj)
        if callable(obj) and depth < 4:
            out.extend(_closure_objects(obj, depth + 1))
    return out


def noise_mechanism_of(noise_fn):
    """Secure sampler (dpc.NoiseParams) of the add_dp_noise lambda: the
    MechanismSpec and Sensitivities its create_mechanism() closes over
    (dp_engine.py:580-593), recomputed with the mirror's mechanisms."""
    spec = sens = None
    for obj in _closure_objects(noise_fn):
        if hasattr(obj, "mechanism_type") and hasattr(obj, "standard_deviation_is_set"):
            spec = obj
        elif all(hasattr(obj, a) for a in ("l0", "linf", "l1", "l2")):
            sens = obj
    if spec is None or sens is None:
        raise NotImplementedError("unrecognised add_dp_noise function (no MechanismSpec / Sensitivities)")
    if sens.l0 is not None and sens.linf is not None:
        local = dpc.Sensitivities(l0=sens.l0, linf=sens.linf)
    else:
        local = dpc.Sensitivities(l1=sens.l1, l2=sens.l2)
    return _additive(spec, local)


def _recognise_add_noise(nodes, source) -> NoisePlan:
    fn = params = budget = None
    for node in nodes:
        if node.op == "map_values" and node.stage == ST_ADD_NOISE:
            if fn is not None:
                raise NotImplementedError("more than one 'Add noise' stage")
            fn = node.fn
        elif node.op == "annotate":
            params = node.kwargs.get("params")
            budget = node.kwargs.get("budget")
        else:
            raise NotImplementedError(f"unrecognised stage {node.stage!r} in an add_dp_noise graph")
    return NoisePlan(source, fn, params, budget)


def recognise(sink):
    """Maps a recorded chain to an AggregatePlan (aggregate /
    select_partitions) or a NoisePlan (add_dp_noise); NotImplementedError
    otherwise."""
    nodes, source = _chain(sink)
    if any(n.op == "map_values" and n.stage == ST_ADD_NOISE for n in nodes):
        return _recognise_add_noise(nodes, source)
    if any(n.op == "map" and n.stage == ST_SP_EXTRACT for n in nodes):
        return _recognise_select_partitions(nodes, source)
    plan = AggregatePlan()
    plan.source = source
    stages = set()
    for node in nodes:
        st = node.stage
        if node.op == "map" and st == ST_EXTRACT:
            plan.extract_fn = node.fn
        elif node.op == "map" and st.startswith(ST_KEY_BY_PREFIX):
            pass
        elif node.op == "filter_by_key" and st == ST_FILTER_KEYS:
            plan.public_keys = node.arg
        elif node.op == "values" and st == ST_DROP_KEY:
            pass
        elif node.op == "map_tuple" and st == ST_DROP_PID:
            pass
        elif node.op == "flatten" and st == ST_PUBLIC_JOIN:
            plan.public_padding = _public_from_padding(node.parents[1])
        elif node.op == "combine_accumulators_per_key" and st == ST_COMBINE:
            plan.combiner = node.arg
        elif node.op == "filter" and st == ST_SELECT:
            plan.selection = node.fn
        elif node.op == "map_values" and st == ST_METRICS:
            plan.compute_metrics = True
        elif node.op == "filter" and st == ST_THRESHOLD_DROP:
            plan.threshold_drop = True
        elif node.op == "annotate":
            plan.params = node.kwargs.get("params")
            plan.budget = node.kwargs.get("budget")
        elif node.op == "sample_fixed_per_key" and st == "Sample per (privacy_id, partition_key)":
            plan.linf_from_graph = node.arg
            stages.add(st)
        elif node.op == "sample_fixed_per_key" and st == "Sample per privacy_id":
            plan.l0_from_graph = node.arg
            stages.add(st)
        else:
            stages.add(st)
    if plan.extract_fn is None:
        raise NotImplementedError("ColumnarBackend executes DPEngine.aggregate graphs only "
                                  f"(no '{ST_EXTRACT}' stage in {[n.stage for n in nodes]})")
    if stages == CROSS_AND_PER:
        plan.bounder = "cross_and_per"
    elif stages == CROSS_ONLY:
        plan.bounder = "cross"
    elif stages == PER_PRIVACY_ID:
        plan.bounder = "per_privacy_id"
    elif stages == LINF_ONLY:
        plan.bounder = "linf"
    elif stages == NOOP:
        plan.bounder = "noop"
    elif stages == ALREADY_ENFORCED:
        plan.bounder = "already_enforced"
    else:
        raise NotImplementedError(f"unrecognised stages for ColumnarBackend: {sorted(stages)}")
    if plan.combiner is None or not plan.compute_metrics:
        raise NotImplementedError("incomplete DPEngine.aggregate graph")
    if plan.params is None:
        raise NotImplementedError("DPEngine.aggregate graph without annotate(params=...)")
    return plan


def _recognise_select_partitions(nodes, source) -> AggregatePlan:
    """DPEngine.select_partitions = Cross-partition bounding (L0 only) +
    privacy-id count per partition + private selection, keys out."""
    plan = AggregatePlan()
    plan.source = source
    plan.bounder = "cross"
    plan.keys_only = True
    plan.compute_metrics = True
    stages = set()
    for node in nodes:
        st = node.stage
        if node.op == "map" and st == ST_SP_EXTRACT:
            plan.extract_fn = node.fn
        elif node.op == "combine_accumulators_per_key" and st == ST_SP_COMBINE:
            plan.combiner = node.arg
        elif node.op == "filter" and st == ST_SELECT:
            plan.selection = node.fn
        elif node.op == "keys" and st == ST_SP_KEYS:
            pass
        elif node.op == "annotate":
            plan.params = node.kwargs.get("params")
            plan.budget = node.kwargs.get("budget")
        else:
            stages.add(st)
    if stages != SELECT_PARTITIONS or plan.combiner is None or plan.selection is None:
        raise NotImplementedError(f"unrecognised select_partitions stages: {sorted(stages)}")
    if plan.params is None:
        raise NotImplementedError("select_partitions graph without annotate(params=...)")
    return plan


def _public_from_padding(branch):
    nodes, source = _chain(branch)
    for node in nodes:
        if node.op == "to_collection" and node.stage == ST_PUBLIC_TO_COL:
            return node.arg
    if nodes and nodes[0].op == "map" and nodes[0].stage == ST_EMPTY_ACCS:
        return source
    raise NotImplementedError("unrecognised public-partition padding branch")


# ------------------------------------------------------------ combiners --
class MetricsProgram:
    """Kernel metric ops + output field order for a CompoundCombiner."""

    def __init__(self):
        self.ops = []            # executor.MetricOpSpec
        self.fields = []         # output names, MetricsTuple order
        self.flags = 0
        self.min_value = self.max_value = self.middle = 0.0
        self.min_sum = self.max_sum = 0.0
        self.int_bounds = True
        self.needs_values = False
        self.threshold_combiner = None


def _noise_kind_code(kind) -> int:
    return N.NOISE_GAUSSIAN if _enum_value(kind) == "gaussian" else N.NOISE_LAPLACE


def _additive(spec, sens) -> dpc.NoiseParams:
    """The secure sampler of create_additive_mechanism(spec, sens)."""
    return dpc.create_additive_mechanism(spec, sens).secure_params()


def build_metrics_program(compound, params) -> MetricsProgram:
    from pipelinedp_amd.executor import MetricOpSpec
    prog = MetricsProgram()
    col = {}

    def out(name):
        if name not in col:
            col[name] = len(prog.fields)
            prog.fields.append(name)
        return col[name]

    def set_bounds(lo, hi):
        prog.min_value, prog.max_value = float(lo), float(hi)
        prog.middle = dpc.compute_middle(lo, hi)
        prog.int_bounds = prog.int_bounds and _is_int(lo) and _is_int(hi)

    for c in compound._combiners:
        name = type(c).__name__
        if name == "CountCombiner":
            prog.ops.append(MetricOpSpec(kind=N.OP_COUNT, out_col=(out("count"),),
                                         noise=(_additive(c._mechanism_spec, c._sensitivities),)))
        elif name == "SumCombiner":
            nz = _additive(c._mechanism_spec, c._sensitivities)
            prog.needs_values = True
            if c._bounding_per_partition:
                prog.flags |= N.SUM_PER_PARTITION
                prog.min_sum, prog.max_sum = float(c._min_bound), float(c._max_bound)
                prog.int_bounds = prog.int_bounds and _is_int(c._min_bound) and _is_int(c._max_bound)
            else:
                prog.flags |= N.ACC_SUM
                set_bounds(c._min_bound, c._max_bound)
            prog.ops.append(MetricOpSpec(kind=N.OP_SUM, out_col=(out("sum"),), noise=(nz,)))
        elif name == "PrivacyIdCountCombiner":
            prog.ops.append(MetricOpSpec(kind=N.OP_PRIVACY_ID_COUNT, out_col=(out("privacy_id_count"),),
                                         noise=(_additive(c._mechanism_spec, c._sensitivities),)))
        elif name == "PostAggregationThresholdingCombiner":
            prog.threshold_combiner = c
            prog.ops.append(MetricOpSpec(kind=N.OP_THRESHOLDED_PID, out_col=(out("privacy_id_count"),)))
        elif name == "MeanCombiner":
            prog.needs_values = True
            prog.flags |= N.ACC_NSUM
            set_bounds(c._min_value, c._max_value)
            cn = _additive(c._count_spec, c._count_sensitivities)
            sn = _additive(c._sum_spec, c._sum_sensitivities)
            names = c._metrics_to_compute
            cols = (out("mean"), out("count") if "count" in names else -1,
                    out("sum") if "sum" in names else -1)
            prog.ops.append(MetricOpSpec(kind=N.OP_MEAN, out_col=cols, noise=(cn, sn), middle=prog.middle))
        elif name == "VarianceCombiner":
            prog.needs_values = True
            prog.flags |= N.ACC_NSUM | N.ACC_NSUM2
            p = c._params.aggregate_params
            set_bounds(p.min_value, p.max_value)
            noise_params = dpc.ScalarNoiseParams(
                c._params.eps, c._params.delta, p.min_value, p.max_value, p.min_sum_per_partition,
                p.max_sum_per_partition, p.max_partitions_contributed,
                p.max_contributions_per_partition, _to_local_noise_kind(p.noise_kind))
            noise = pdc.variance_noise_params(noise_params)
            names = c._metrics_to_compute
            cols = (out("variance"), out("count") if "count" in names else -1,
                    out("sum") if "sum" in names else -1, out("mean") if "mean" in names else -1)
            lo, hi = p.min_value, p.max_value
            prog.ops.append(MetricOpSpec(kind=N.OP_VARIANCE, out_col=cols, noise=noise, middle=prog.middle,
                                         min_value=float(lo),
                                         sq_min_value=float(dpc.compute_squares_interval(lo, hi)[0]),
                                         degenerate=int(lo == hi)))
        else:
            raise NotImplementedError(f"{name} is not supported by ColumnarBackend "
                                      "(hot path: Count/Sum/Mean/Variance/PrivacyIdCount)")
    return prog


def _to_local_noise_kind(kind):
    from pipelinedp_amd import aggregate_params as agg
    return agg.NoiseKind(_enum_value(kind))


def _is_int(x) -> bool:
    return isinstance(x, (int, np.integer)) and not isinstance(x, bool)


# -------------------------------------------------------------- backend --
def shard_rows_by_privacy_id(mode, pid_t, pk_t, val_t, pid_enc):
    """Multi-rank: verify that no privacy id spans ranks ("verify"), or
    shuffle the rows to the privacy ids' owner ranks ("shuffle"); "trusted"
    returns the rows unchanged (ColumnarBackend privacy_id_sharding).
    Identities: integer ids themselves, else a fixed-key hash of the key
    (parallel.key_identities).  Returns (pid_t, pk_t, val_t, pid_enc)."""
    import torch
    if mode == "trusted" or parallel.world_info()[0] == 1:
        return pid_t, pk_t, val_t, pid_enc
    table = None if pid_enc.decode is None else \
        torch.as_tensor(parallel.key_identities(pid_enc.decode)).to(pid_t.device)
    if mode == "verify":
        parallel.verify_privacy_id_sharding(pid_t if table is None else table)
        return pid_t, pk_t, val_t, pid_enc
    ident = pid_t if table is None else table[pid_t]
    ident, (pk_t, val_t) = parallel.shuffle_by_privacy_id(ident, [pk_t, val_t])
    uniq, inv = torch.unique(ident, return_inverse=True)  # dense local codes of the received ids
    pid_t = inv.to(torch.int64).contiguous()
    return pid_t, pk_t.contiguous(), None if val_t is None else val_t.contiguous(), \
        C.EncodedKeys(pid_t, max(int(uniq.numel()), 1), None)


def parse_tuning(text: str) -> dict:
    """"k=v,k=v" (PIPELINEDP_AMD_TUNING) -> {k: int(v)} over ColumnarBackend.TUNING_KEYS."""
    out = {}
    for item in filter(None, (t.strip() for t in text.split(","))):
        k, sep, v = item.partition("=")
        if not sep or k.strip() not in ColumnarBackend.TUNING_KEYS:
            raise ValueError(f"PIPELINEDP_AMD_TUNING: bad item {item!r} (keys: "
                             f"{', '.join(ColumnarBackend.TUNING_KEYS)})")
        out[k.strip()] = int(v)
    return out


class ColumnarBackend(pipeline_backend.PipelineBackend):
    """Columnar, lazily executed PipelineBackend running on one MI355X GPU
    (or one GPU per rank with torch.distributed; see parallel.py).

    Args:
      device: torch device (default cuda:current).
      seed: fixes the sampling / selection / noise streams (testing only —
        a DP release must use fresh randomness, the default).
      privacy_id_sharding: under torch.distributed, how the rows of one
        privacy id are kept on one rank (contribution bounding is per privacy
        id over the whole dataset, contribution_bounders.py:62-111):
        "verify" (default) checks that no privacy id is on two ranks and
        raises ValueError otherwise; "shuffle" moves every row to the rank
        that owns its privacy id (one all-to-all of the rows); "trusted"
        skips the check (the caller guarantees it).
      workspace: an executor.BoundWorkspace to reuse (the bounding kernels'
        device workspace; by default each backend keeps its own across runs).
      tuning: data-movement knobs of the bounding kernels, all of which keep
        the results identical (pdp_bound_config: algorithm, merge,
        key_format, sieve, sieve_band, sieve_threads, bucket_threads); default {} = the
        library's plan.  The environment variable PIPELINEDP_AMD_TUNING
        ("sieve=16384,merge=1") supplies defaults for it.
    """

    TUNING_KEYS = ("algorithm", "merge", "key_format", "sieve", "sieve_band", "sieve_threads", "bucket_threads")

    def __init__(self, device=None, seed: Optional[int] = None, privacy_id_sharding: str = "verify",
                 workspace=None, tuning: Optional[dict] = None):
        if privacy_id_sharding not in ("verify", "shuffle", "trusted"):
            raise ValueError(f"privacy_id_sharding must be 'verify', 'shuffle' or 'trusted', "
                             f"got {privacy_id_sharding!r}")
        self._device = device
        self._seed = seed
        self._pid_sharding = privacy_id_sharding
        self._workspace = workspace
        self._tuning = parse_tuning(os.environ.get("PIPELINEDP_AMD_TUNING", ""))
        for k, v in (tuning or {}).items():
            if k not in self.TUNING_KEYS:
                raise ValueError(f"unknown tuning key {k!r} (one of {', '.join(self.TUNING_KEYS)})")
            self._tuning[k] = int(v)
        self.last_plan_info = None
        self.last_bounding = None  # BoundingSpec of the last bounding pass (bench accounting)

    # ---------------------------------------------------- recorded ops --
    def _node(self, op, col, stage, **kw):
        return _Node(self, op, (col,), stage, **kw)

    def map(self, col, fn, stage_name: str = None):
        return self._node("map", col, stage_name, fn=fn)

    def map_with_side_inputs(self, col, fn, side_input_cols, stage_name: str = None):
        return self._node("map_with_side_inputs", col, stage_name, fn=fn, arg=side_input_cols)

    def flat_map(self, col, fn, stage_name: str = None):
        return self._node("flat_map", col, stage_name, fn=fn)

    def map_tuple(self, col, fn, stage_name: str = None):
        return self._node("map_tuple", col, stage_name, fn=fn)

    def map_values(self, col, fn, stage_name: str = None):
        return self._node("map_values", col, stage_name, fn=fn)

    def group_by_key(self, col, stage_name: str = None):
        return self._node("group_by_key", col, stage_name)

    def filter(self, col, fn, stage_name: str = None):
        return self._node("filter", col, stage_name, fn=fn)

    def filter_by_key(self, col, keys_to_keep, stage_name: str = None):
        return self._node("filter_by_key", col, stage_name, arg=keys_to_keep)

    def keys(self, col, stage_name: str = None):
        return self._node("keys", col, stage_name)

    def values(self, col, stage_name: str = None):
        return self._node("values", col, stage_name)

    def sample_fixed_per_key(self, col, n: int, stage_name: str = None):
        return self._node("sample_fixed_per_key", col, stage_name, arg=n)

    def count_per_element(self, col, stage_name: str = None):
        return self._node("count_per_element", col, stage_name)

    def sum_per_key(self, col, stage_name: str = None):
        return self._node("sum_per_key", col, stage_name)

    def combine_accumulators_per_key(self, col, combiner, stage_name: str = None):
        return self._node("combine_accumulators_per_key", col, stage_name, arg=combiner)

    def reduce_per_key(self, col, fn, stage_name: str = None):
        return self._node("reduce_per_key", col, stage_name, fn=fn)

    def flatten(self, cols, stage_name: str = None):
        cols = tuple(cols)
        return _Node(self, "flatten", cols, stage_name)

    def distinct(self, col, stage_name: str = None):
        return self._node("distinct", col, stage_name)

    def to_list(self, col, stage_name: str = None):
        return self._node("to_list", col, stage_name)

    def to_collection(self, collection_or_iterable, col, stage_name: str = None):
        return _Node(self, "to_collection", (), stage_name, arg=collection_or_iterable)

    def to_multi_transformable_collection(self, col):
        return col

    def annotate(self, col, stage_name: str = None, **kwargs):
        return _Node(self, "annotate", (col,), stage_name, kwargs=kwargs)

    # ------------------------------------------------------- execution --
    def _torch_device(self):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("ColumnarBackend needs a ROCm GPU; there is no CPU fallback")
        return torch.device(self._device) if self._device is not None else \
            torch.device("cuda", torch.cuda.current_device())

    def _seeds(self):
        if self._seed is None:
            raw = os.urandom(24)
            return tuple(int.from_bytes(raw[i:i + 8], "little") for i in (0, 8, 16))
        s = int(self._seed)
        return tuple((s * 0x9E3779B97F4A7C15 + k * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF
                     for k in (1, 2, 3))

    def _execute(self, sink) -> List:
        plan = recognise(sink)
        if isinstance(plan, NoisePlan):
            return AddNoiseRun(self, plan).run()
        return AggregateRun(self, plan).run()

    def accumulators(self, col):
        """Testing aid: executes the bounding + reduction of an aggregate
        graph and returns {partition_key: reference-style pre-noise
        accumulator (row_count, (child accumulators...))}."""
        plan = recognise(col)
        return AggregateRun(self, plan).raw_accumulators()


class AggregateRun:
    """One execution of a recognised aggregate plan on the GPU."""

    def __init__(self, backend: ColumnarBackend, plan: AggregatePlan):
        self.backend = backend
        self.plan = plan
        self.params = plan.params
        self.prog = build_metrics_program(plan.combiner, plan.params)

    # ---------------------------------------------------------- ingest --
    def _columns(self):
        import torch
        device = self.backend._torch_device()
        src = self.plan.source
        specs = C.probe_columns(self.plan.extract_fn, src) if isinstance(src, C.ColumnTable) else None
        if specs is not None:
            pid_raw = src.column(specs[0].name) if specs[0] is not None else None
            pk_raw = src.column(specs[1].name)
            v = specs[2]
            val_raw = src.column(v.name) if isinstance(v, C.ColumnRef) else None
            n_pid, n_pk = src.n_privacy_ids, src.n_partitions
            pk_decode = src.partition_keys
        else:
            rows = [self.plan.extract_fn(r) for r in src]
            pid_raw = [r[0] for r in rows]
            pk_raw = [r[1] for r in rows]
            val_raw = [r[2] for r in rows] if self.prog.needs_values else None
            n_pid = n_pk = None
            pk_decode = None
        units = self.plan.bounder == "already_enforced"  # no privacy ids on this path
        if pid_raw is None and not units:
            raise ValueError("privacy_id_extractor is required unless contribution_bounds_already_enforced")
        pid_enc = None if units else C.encode_keys(_host_or_device(pid_raw), n_pid)
        pk_enc = C.encode_keys(_host_or_device(pk_raw), n_pk)
        if pk_decode is not None and pk_enc.decode is None:
            pk_enc.decode = np.asarray(pk_decode, dtype=object)
        public = self.plan.public_padding if self.plan.public_padding is not None else self.plan.public_keys
        public_codes = None
        if public is not None:
            pk_enc, public_codes = C.extend_with_keys(pk_enc, public)
        if parallel.world_info()[0] > 1:  # one partition dictionary for all ranks
            pk_enc = parallel.global_partition_keys(pk_enc)
            if public is not None and pk_enc.decode is not None:
                enc_map = pk_enc.encode if pk_enc.encode is not None else \
                    {k: i for i, k in enumerate(pk_enc.decode)}
                public_codes = np.asarray([enc_map[k] for k in public], dtype=np.int64)
        pid_t = None if pid_enc is None else \
            _h2d(pid_enc.codes, device, torch.int64)
        pk_t = _h2d(pk_enc.codes, device, torch.int64)
        val_t = None
        value_kind = N.VALUE_NONE
        if self.prog.needs_values:
            if val_raw is None:
                raise ValueError("the value extractor must return a value column for SUM/MEAN/VARIANCE")
            val_t = _value_tensor(val_raw, device)
            if parallel.all_ranks_any(val_t.dtype != torch.int64):  # one value kind on every rank
                val_t = val_t.to(torch.float64)
            value_kind = N.VALUE_I64 if val_t.dtype == torch.int64 else N.VALUE_F64
        if pid_t is not None and parallel.world_info()[0] > 1 and self.backend._pid_sharding != "trusted":
            pid_t, pk_t, val_t, pid_enc = self._shard_privacy_ids(pid_t, pk_t, val_t, pid_enc)
        return pid_t, pk_t, val_t, value_kind, pid_enc, pk_enc, public_codes

    def _shard_privacy_ids(self, pid_t, pk_t, val_t, pid_enc):
        return shard_rows_by_privacy_id(self.backend._pid_sharding, pid_t, pk_t, val_t, pid_enc)

    def _bounding_spec(self, value_kind):
        from pipelinedp_amd.executor import BoundingSpec
        p = self.params
        flags = self.prog.flags
        if (flags & (N.ACC_SUM | N.SUM_PER_PARTITION)) and value_kind == N.VALUE_I64 and self.prog.int_bounds:
            flags |= N.SUM_INT
        bounder = self.plan.bounder
        l0 = linf = max_contributions = 0
        if bounder in ("cross_and_per", "cross"):  # contribution_bounders.py:62-111, 159-201
            l0 = int(p.max_partitions_contributed)
            if self.plan.l0_from_graph is not None and self.plan.l0_from_graph != l0:
                raise ValueError("inconsistent max_partitions_contributed in the graph")
        if bounder in ("cross_and_per", "linf"):   # :72-111, :204-230
            linf = int(p.max_contributions_per_partition)
            if self.plan.linf_from_graph is not None and self.plan.linf_from_graph != linf:
                raise ValueError("inconsistent max_contributions_per_partition in the graph")
        if bounder == "per_privacy_id":             # :114-156
            max_contributions = int(self.plan.l0_from_graph or p.max_contributions)
        return BoundingSpec(l0=l0, linf=linf, value_kind=value_kind, flags=flags,
                            min_value=self.prog.min_value, max_value=self.prog.max_value,
                            middle=self.prog.middle, min_sum=self.prog.min_sum, max_sum=self.prog.max_sum,
                            max_contributions=max_contributions,
                            rows_are_units=bounder == "already_enforced")

    def _bound(self):
        from pipelinedp_amd import executor as X
        import torch
        pid_t, pk_t, val_t, vk, pid_enc, pk_enc, public_codes = self._columns()
        spec = self._bounding_spec(vk)
        world, _ = parallel.world_info()
        P, _ = parallel.partition_slices(pk_enc.n, world)  # padded to a multiple of the ranks
        row_offset, self._total_rows = parallel.row_offset_and_total(pk_t.numel())
        allowed = None
        if public_codes is not None:
            mask = np.zeros(P, dtype=np.uint8)
            mask[public_codes] = 1
            allowed = torch.as_tensor(mask).to(pk_t.device)
        seed_bound, _, _ = self._seeds
        n_pid = 1 if pid_enc is None else pid_enc.n
        if pk_t.numel() == 0:
            acc = X.new_accumulators(P, spec, pk_t.device)
        else:
            if self.backend._workspace is None:
                self.backend._workspace = X.BoundWorkspace()
            tune = self.backend._tuning
            acc = X.bound_and_reduce(pid_t, pk_t, val_t, n_privacy_ids=n_pid, n_partitions=P,
                                     bounding=spec, seed=seed_bound, allowed=allowed, row_offset=row_offset,
                                     workspace=self.backend._workspace, check_keys="defer", **tune)
            self.backend.last_plan_info = X.bound_plan(pk_t.numel(), n_pid, P, spec, **tune)
            self.backend.last_bounding = spec
        return acc, spec, pk_enc, allowed

    def _selection(self):
        from pipelinedp_amd.executor import SelectionSpec
        tc = self.prog.threshold_combiner
        if tc is not None:
            mech = tc.create_mechanism() if type(tc).__module__.startswith("pipelinedp_amd") else None
            spec = tc._mechanism_spec
            strategy = ps.create_partition_selection_strategy(
                _local_strategy(spec.mechanism_type.to_partition_selection_strategy()), spec.eps,
                spec.delta, tc._sensitivities.l0, tc._pre_threshold)
            return strategy.device_spec(1)
        if self.plan.public_keys is not None or self.plan.public_padding is not None:
            return SelectionSpec(strategy=N.SELECT_PUBLIC)
        if self.plan.selection is None:
            return SelectionSpec(strategy=N.SELECT_ALL_NONEMPTY)
        part = self.plan.selection
        if not isinstance(part, functools.partial) or len(part.args) != 5:
            raise NotImplementedError("unrecognised private partition selection function")
        budget, max_partitions, max_rows, strategy, pre_threshold = part.args
        strat = ps.create_partition_selection_strategy(_local_strategy(strategy), budget.eps, budget.delta,
                                                       max_partitions, pre_threshold)
        return strat.device_spec(int(max_rows))

    def run(self) -> List:
        """Single GPU: every partition.  Under torch.distributed (one rank per
        GPU, each holding its own rows; privacy ids must not span ranks): the
        partitions this rank owns after the accumulator exchange — the union
        over ranks is the result."""
        import torch
        from pipelinedp_amd import executor as X
        acc, spec, pk_enc, allowed = self._bound()
        # int64 fields: counts and privacy-id counts are at most the global
        # row count; an int SUM has no such bound (its maximum is read back)
        int_bound = None if spec.sum_is_int else self._total_rows
        acc, first = parallel.exchange_accumulators(acc, int_bound=int_bound)  # identity on one rank
        sel = self._selection()
        public = self.plan.public_keys is not None or self.plan.public_padding is not None
        public_mask = None
        if public:
            n_mine = acc["privacy_id_count"].shape[0]
            public_mask = allowed[first:first + n_mine].contiguous()
        _, seed_select, seed_noise = self._seeds
        index, out, n_kept_dev = X.select_and_noise(acc, selection=sel, ops=self.prog.ops,
                                                    n_cols=len(self.prog.fields), seed_select=seed_select,
                                                    seed_noise=seed_noise, public_mask=public_mask,
                                                    partition_offset=first, sync_count=False)
        # the kept count and the kept columns in one round trip (one stream sync)
        idx, vals, n_kept = X.kept_to_host_guess(index, out, n_kept_dev, keys_only=self.plan.keys_only,
                                                 key=(int(index.shape[0]), len(self.prog.fields),
                                                      self.plan.keys_only))
        self._raise_key_errors()  # the deferred key check (its copy has landed: the stream was synchronised)
        if self.plan.keys_only:  # select_partitions: "Drop accumulators, keep only partition keys"
            return pk_enc.keys_of(first + idx).tolist()
        nf = len(self.prog.fields)
        if not n_kept:
            vals = np.zeros((nf, 0))
        keep = np.ones(len(idx), dtype=bool)
        if self.prog.threshold_combiner is not None:  # dp_engine.py:544-549: drop thresholded None (NaN)
            keep = ~np.isnan(vals[self.prog.fields.index("privacy_id_count")])
        nt = pdc._get_or_create_named_tuple("MetricsTuple", tuple(self.prog.fields))
        cols = {f: np.ascontiguousarray(vals[c][keep]) for c, f in enumerate(self.prog.fields)}
        return C.AggregateResult(pk_enc.keys_of(first + idx[keep]), cols, nt)

    def raw_accumulators(self):
        acc, spec, pk_enc, allowed = self._bound()
        host = {k: (None if v is None else v.cpu().numpy()) for k, v in acc.items()}
        self._raise_key_errors()
        public = allowed.cpu().numpy().astype(bool) if allowed is not None else None
        out = {}
        for p in range(pk_enc.n):
            rc = int(host["privacy_id_count"][p])
            if public is None and rc == 0:
                continue
            if public is not None and not public[p]:
                continue
            children = []
            for c in self.plan.combiner._combiners:
                name = type(c).__name__
                if name == "CountCombiner":
                    children.append(int(host["count"][p]))
                elif name == "SumCombiner":
                    s = host["sum"][p]
                    children.append(int(s) if host["sum"].dtype == np.int64 else float(s))
                elif name in ("PrivacyIdCountCombiner", "PostAggregationThresholdingCombiner"):
                    children.append(rc)
                elif name == "MeanCombiner":
                    children.append((int(host["count"][p]), float(host["normalized_sum"][p])))
                elif name == "VarianceCombiner":
                    children.append((int(host["count"][p]), float(host["normalized_sum"][p]),
                                     float(host["normalized_sum_sq"][p])))
            row_count = rc + (1 if public is not None else 0)  # empty public accumulator
            out[pk_enc.key_of(p)] = (row_count, tuple(children))
        return out

    def _raise_key_errors(self):
        from pipelinedp_amd import executor as X
        if self.backend._workspace is not None:
            X.raise_key_errors(self.backend._workspace)

    @property
    def _seeds(self):
        if not hasattr(self, "_seed_cache"):
            self._seed_cache = parallel.broadcast_seeds(self.backend._seeds())
        return self._seed_cache


class AddNoiseRun:
    """DPEngine.add_dp_noise on the GPU: the value column + noise in one
    kernel (`pdp_add_noise`), keys passed through in input order.  A
    two-column ColumnTable (keys, values) is used as columns directly (device
    tensors stay on the device); any other source is read as (key, value)
    tuples.  Under torch.distributed each rank noises its own rows with global
    row indices as Philox counters."""

    def __init__(self, backend: ColumnarBackend, plan: NoisePlan):
        self.backend = backend
        self.plan = plan

    def run(self) -> List:
        import torch
        from pipelinedp_amd import executor as X
        noise = noise_mechanism_of(self.plan.noise_fn)
        device = self.backend._torch_device()
        src = self.plan.source
        if isinstance(src, C.ColumnTable) and len(src.names) == 2:
            keys = src.column(src.names[0])
            vals = src.column(src.names[1])
        else:
            pairs = list(src)
            keys = [k for k, _ in pairs]
            vals = [v for _, v in pairs]
        val_t = _value_tensor(vals, device)
        offset = parallel.row_offset(int(val_t.numel()))
        _, _, seed_noise = parallel.broadcast_seeds(self.backend._seeds())
        out = X.add_noise(val_t, noise=noise, seed=seed_noise, index_offset=offset)
        noised = out.cpu().numpy().tolist()
        if C._is_torch(keys):
            keys = keys.cpu().numpy()
        elif isinstance(keys, C.DictColumn):
            keys = keys.dictionary[keys.codes]
        return list(zip(np.asarray(keys).tolist() if isinstance(keys, np.ndarray) else keys, noised))


def _local_strategy(strategy):
    from pipelinedp_amd import aggregate_params as agg
    return agg.PartitionSelectionStrategy(_enum_value(strategy))


def _h2d(col, device, dtype):
    """Host column (possibly a read-only Arrow buffer view) -> contiguous
    device tensor; device tensors are converted in place on the device."""
    import torch
    if C._is_torch(col):
        return col.to(device=device, dtype=dtype).contiguous()
    arr = np.asarray(col)
    if not arr.flags.writeable:  # only read; torch warns on non-writable arrays
        arr = arr.copy()
    return torch.from_numpy(arr).to(device=device, dtype=dtype).contiguous()


def _host_or_device(col):
    if C._is_torch(col) or isinstance(col, C.DictColumn):
        return col
    return np.asarray(col) if not isinstance(col, np.ndarray) else col


def _value_tensor(col, device):
    import torch
    if C._is_torch(col):
        t = col.to(device)
        if t.dtype in (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool):
            return t.to(torch.int64).contiguous()
        return t.to(torch.float64).contiguous()
    arr = np.asarray(col)
    if arr.dtype.kind in "iub":
        return torch.as_tensor(arr.astype(np.int64)).to(device)
    if arr.dtype.kind == "f":
        return torch.as_tensor(arr.astype(np.float64)).to(device)
    vals = [float(v) for v in col]
    if all(float(v).is_integer() and isinstance(v, (int, np.integer)) for v in col):
        return torch.as_tensor(np.asarray(col, dtype=np.int64)).to(device)
    return torch.as_tensor(np.asarray(vals, dtype=np.float64)).to(device)
