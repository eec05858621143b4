"""Dataset histograms on the GPU (mirror of pipeline_dp/dataset_histograms/
computing_histograms.py).

`compute_dataset_histograms(col, data_extractors, backend)` keeps the
reference's signature and result (a one-element collection holding a
DatasetHistograms, :456-513).  The reference computes the seven histograms
with per-element Python group-bys; here the columns are dictionary-encoded
once (pipelinedp_amd.columnar) and one HIP pass (`pdp_dataset_histograms`,
csrc/pdp_hist.hip) produces every bin.  There is no CPU fallback: without a
GPU or the HIP library this raises.
"""
import ctypes
from typing import Dict, List

import numpy as np

from pipelinedp_amd import columnar as C
from pipelinedp_amd import _native as N
from pipelinedp_amd.dataset_histograms import histograms as hist

NUMBER_OF_BUCKETS_SUM_HISTOGRAM = N.HIST_SUM_BUCKETS  # computing_histograms.py:25

# order of the integer histograms in pdp_dataset_histograms.int_* (pipelinedp_amd.h)
_INT_TYPES = (hist.HistogramType.L0_CONTRIBUTIONS, hist.HistogramType.L1_CONTRIBUTIONS,
              hist.HistogramType.LINF_CONTRIBUTIONS, hist.HistogramType.COUNT_PER_PARTITION,
              hist.HistogramType.COUNT_PRIVACY_ID_PER_PARTITION)
_FLOAT_TYPES = (hist.HistogramType.LINF_SUM_CONTRIBUTIONS, hist.HistogramType.SUM_PER_PARTITION)


def log_bin_bounds(index: int):
    """(lower, upper) of dense integer-bin `index` (the bins of
    _to_bin_lower_upper_logarithmic, computing_histograms.py:28-47)."""
    if index < 1000:
        return index, index + 1
    e = (index - 1000) // 900 + 1
    q = (index - 1000) % 900 + 100
    lower = q * 10**e
    return lower, lower + 10**e


def histograms_from_device(raw: Dict) -> hist.DatasetHistograms:
    """Device bin arrays of executor.dataset_histograms(_preaggregated) ->
    DatasetHistograms (bins sorted by lower, empty bins absent, :176-195)."""
    host = {k: v.cpu().numpy() for k, v in raw.items() if k != "workspace"}
    built = {}
    for h, name in enumerate(_INT_TYPES):
        cnt = host["int_count"][h]
        bins = []
        # present bins: a count, or (pre-aggregated L0 / L1) a value whose
        # rounded weight is 0, which the reference keeps as a count-0 bin
        for b in np.flatnonzero((cnt > 0) | (host["int_max"][h] > 0)).tolist():
            lo, up = log_bin_bounds(b)
            bins.append(hist.FrequencyBin(lower=lo, upper=up, count=int(cnt[b]), sum=int(host["int_sum"][h, b]),
                                          max=int(host["int_max"][h, b])))
        built[name] = hist.Histogram(name, bins)
    for f, name in enumerate(_FLOAT_TYPES):
        nl = int(host["float_n_lowers"][f])
        lowers = host["float_lowers"][f]
        cnt = host["float_count"][f]
        bins = []
        for b in np.flatnonzero(cnt[:max(nl - 1, 0)]).tolist():
            bins.append(hist.FrequencyBin(lower=lowers[b], upper=lowers[b + 1], count=int(cnt[b]),
                                          sum=float(host["float_sum"][f, b]), max=float(host["float_max"][f, b])))
        built[name] = hist.Histogram(name, bins)
    T = hist.HistogramType
    return hist.DatasetHistograms(built[T.L0_CONTRIBUTIONS], built[T.L1_CONTRIBUTIONS],
                                  built[T.LINF_CONTRIBUTIONS], built[T.LINF_SUM_CONTRIBUTIONS],
                                  built[T.COUNT_PER_PARTITION], built[T.COUNT_PRIVACY_ID_PER_PARTITION],
                                  built[T.SUM_PER_PARTITION])


def _device(backend):
    import torch
    if hasattr(backend, "_torch_device"):
        return backend._torch_device()
    if not torch.cuda.is_available():
        raise RuntimeError("compute_dataset_histograms needs a ROCm GPU; there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def _columns(col, data_extractors):
    """(pid, pk, value) raw columns: whole ColumnTable columns when the
    extractors name columns, else one extractor call per row (:469-473)."""
    def extract(row):
        return (data_extractors.privacy_id_extractor(row), data_extractors.partition_extractor(row),
                data_extractors.value_extractor(row) if data_extractors.value_extractor else None)

    if isinstance(col, C.ColumnTable):
        specs = C.probe_columns(extract, col)
        if specs is not None and specs[0] is not None:
            v = specs[2]
            val = col.column(v.name) if isinstance(v, C.ColumnRef) else None
            if val is None and v is not None:
                val = np.full(len(col), v, dtype=np.float64)
            return (col.column(specs[0].name), col.column(specs[1].name), val,
                    col.n_privacy_ids, col.n_partitions)
    rows = [extract(r) for r in col]
    vals = [r[2] for r in rows]
    return ([r[0] for r in rows], [r[1] for r in rows],
            None if all(v is None for v in vals) else vals, None, None)


def compute_dataset_histograms(col, data_extractors, backend=None) -> List[hist.DatasetHistograms]:
    """Computes the dataset histograms (computing_histograms.py:456-513):
    contributions per privacy id (L0: distinct partitions, L1: rows), per
    (privacy id, partition) pair (Linf: rows, Linf-sum: value sum), and per
    partition (rows, distinct privacy ids, value sum).  Returns a one-element
    list holding a DatasetHistograms.  Under torch.distributed each rank
    passes its shard of rows and every rank gets the histograms of the whole
    dataset.  The rows of one privacy id must sit on one rank: as in
    DPEngine.aggregate, `backend`'s privacy_id_sharding decides whether that
    is verified (default; ValueError otherwise), established by a shuffle of
    the rows, or trusted."""
    from pipelinedp_amd import executor as X
    from pipelinedp_amd.columnar_backend import _h2d, _host_or_device, _value_tensor, shard_rows_by_privacy_id
    import torch
    device = _device(backend)
    pid_raw, pk_raw, val_raw, n_pid, n_pk = _columns(col, data_extractors)
    pid_enc = C.encode_keys(_host_or_device(pid_raw), n_pid)
    pk_enc = C.encode_keys(_host_or_device(pk_raw), n_pk)
    from pipelinedp_amd import parallel
    if parallel.world_info()[0] > 1:  # rows sharded by privacy id: one partition dictionary for all ranks
        pk_enc = parallel.global_partition_keys(pk_enc)
    pid_t = _h2d(pid_enc.codes, device, torch.int64)
    pk_t = _h2d(pk_enc.codes, device, torch.int64)
    val_t = _value_tensor(val_raw, device) if val_raw is not None else None
    if parallel.world_info()[0] > 1:
        if val_t is not None and parallel.all_ranks_any(val_t.dtype != torch.int64):
            val_t = val_t.to(torch.float64)  # one value kind on every rank
        mode = getattr(backend, "_pid_sharding", "verify")
        pid_t, pk_t, val_t, pid_enc = shard_rows_by_privacy_id(mode, pid_t, pk_t, val_t, pid_enc)
    raw = X.dataset_histograms(pid_t, pk_t, val_t, n_privacy_ids=pid_enc.n, n_partitions=pk_enc.n)
    flags = ctypes.c_uint32()
    N.check(N.lib().pdp_bound_error_flags(X._ptr(raw["workspace"]), ctypes.byref(flags), X._stream()),
            "pdp_bound_error_flags")
    if flags.value & 1:
        raise ValueError("privacy id or partition code outside the declared range")
    return [histograms_from_device(raw)]


def _preaggregated_columns(col, data_extractors):
    """(pk, count, sum, n_partitions, n_contributions) raw columns: whole
    ColumnTable columns when the extractors name columns, else one extractor
    call per row (:729-733)."""
    if isinstance(col, C.ColumnTable):
        try:
            probe = C._ProbeRow()
            pk = data_extractors.partition_extractor(probe)
            pre = tuple(data_extractors.preaggregate_extractor(probe))
        except Exception:
            pk, pre = None, ()
        refs = (pk,) + pre
        if len(refs) == 5 and all(isinstance(r, C.ColumnRef) and col.has_column(r.name) for r in refs):
            return tuple(col.column(r.name) for r in refs) + (col.n_partitions,)
    pks, cnt, tot, npart, ncontr = [], [], [], [], []
    for row in col:
        pks.append(data_extractors.partition_extractor(row))
        c, t, npp, nc = data_extractors.preaggregate_extractor(row)[:4]
        cnt.append(c)
        tot.append(t)
        npart.append(npp)
        ncontr.append(nc)
    return (pks, np.asarray(cnt, dtype=np.int64), np.asarray(tot, dtype=np.float64),
            np.asarray(npart, dtype=np.int64), np.asarray(ncontr, dtype=np.int64), None)


def compute_dataset_histograms_on_preaggregated_data(col, data_extractors,
                                                     backend=None) -> List[hist.DatasetHistograms]:
    """Computes the dataset histograms of a pre-aggregated dataset
    (computing_histograms.py:713-758): `col` holds one row per (privacy id,
    partition) pair, from which data_extractors (PreAggregateExtractors) give
    the partition key and (count, sum, n_partitions, n_contributions), as
    analysis/pre_aggregation.py:19-58 emits them.  L0 / L1 weigh each row by
    1 / n_partitions and round the weight sum per value (:520-568); the other
    five histograms are those of compute_dataset_histograms.  Returns a
    one-element list holding a DatasetHistograms.  Under torch.distributed
    each rank passes its shard (the rows of one privacy id on one rank) and
    every rank gets the histograms of the whole dataset.  count,
    n_partitions and n_contributions must be >= 1 (ValueError otherwise)."""
    from pipelinedp_amd import executor as X
    from pipelinedp_amd.columnar_backend import _h2d, _host_or_device
    import torch
    device = _device(backend)
    pk_raw, cnt, tot, npart, ncontr, n_pk = _preaggregated_columns(col, data_extractors)
    pk_enc = C.encode_keys(_host_or_device(pk_raw), n_pk)
    from pipelinedp_amd import parallel
    if parallel.world_info()[0] > 1:
        pk_enc = parallel.global_partition_keys(pk_enc)
    t = [_h2d(c, device, dt) for c, dt in ((pk_enc.codes, torch.int64), (cnt, torch.int64),
                                           (tot, torch.float64), (npart, torch.int64), (ncontr, torch.int64))]
    raw = X.dataset_histograms_preaggregated(*t, n_partitions=pk_enc.n)
    flags = ctypes.c_uint32()
    N.check(N.lib().pdp_bound_error_flags(X._ptr(raw["workspace"]), ctypes.byref(flags), X._stream()),
            "pdp_bound_error_flags")
    if flags.value & 1:
        raise ValueError("partition code outside the declared range")
    if flags.value & 2:
        raise ValueError("pre-aggregated count, n_partitions and n_contributions must be in [1, 2^62)")
    return [histograms_from_device(raw)]

