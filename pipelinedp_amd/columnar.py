"""Columnar input and ingest: ColumnTable, column probing, key encoding.

ColumnTable is the collection type the ColumnarBackend reads at HBM speed.
DataExtractors are resolved to columns by *probing*: the extraction function
DPEngine builds (dp_engine.py:402-415) is called once on a probe row whose
items/attributes are column references, so ``ColumnExtractor("user_id")``,
``lambda r: r[0]`` and ``lambda r: r.user_id`` all resolve without touching
the data.  Anything else is extracted row-wise on the host (ingest, not
compute) and then encoded.

Keys are dictionary-encoded to dense int64 ids: integer keys that are already
dense-ish are used as-is (identity dictionary); other keys go through
pandas.factorize.  The dictionary decodes output partitions back to the
user's keys.
"""
import dataclasses
from typing import Any, Mapping, Optional, Sequence

import numpy as np


class ColumnRef:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"ColumnRef({self.name!r})"


class _ProbeRow:
    """Row whose every item/attribute is a ColumnRef."""

    def __getitem__(self, key):
        return ColumnRef(key)

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return ColumnRef(name)


class _Row:
    """Row view of a ColumnTable for row-wise consumers (r[name], r[i], r.name)."""
    __slots__ = ("_t", "_i")

    def __init__(self, table, i):
        self._t, self._i = table, i

    def __getitem__(self, key):
        return self._t._item(key, self._i)

    def __getattr__(self, name):
        try:
            return self._t._item(name, self._i)
        except KeyError as e:
            raise AttributeError(name) from e

    def __iter__(self):
        return (self._t._item(k, self._i) for k in self._t.names)

    def __len__(self):
        return len(self._t.names)

    def __repr__(self):
        return "Row(" + ", ".join(f"{k}={self._t._item(k, self._i)!r}" for k in self._t.names) + ")"


class ColumnTable:
    """Named equal-length columns (numpy arrays or torch tensors, possibly
    already on the GPU).  Iterating yields row views, so a ColumnTable also
    works with row-wise backends.

    Optional metadata for device-resident integer keys:
      n_privacy_ids / n_partitions — the dense key ranges (skips a min/max pass);
      partition_keys — decoding dictionary (partition index -> user key).
    """

    def __init__(self, columns, *, n_privacy_ids: Optional[int] = None,
                 n_partitions: Optional[int] = None, partition_keys: Optional[Sequence] = None):
        if isinstance(columns, Mapping):
            self._cols = dict(columns)
        else:
            self._cols = {i: c for i, c in enumerate(columns)}
        lens = {len(c) for c in self._cols.values()}
        if len(lens) > 1:
            raise ValueError(f"columns have different lengths {sorted(lens)}")
        self._n = lens.pop() if lens else 0
        self.n_privacy_ids = n_privacy_ids
        self.n_partitions = n_partitions
        self.partition_keys = partition_keys

    @property
    def names(self):
        return list(self._cols)

    def column(self, name):
        return self._cols[name]

    def has_column(self, name) -> bool:
        return name in self._cols

    def __len__(self):
        return self._n

    def __bool__(self):
        return self._n > 0

    def _item(self, key, i):
        c = self._cols[key]
        v = c[i]
        return v.item() if hasattr(v, "item") else v

    def __iter__(self):
        return (_Row(self, i) for i in range(self._n))


def probe_columns(extract_fn, table: ColumnTable):
    """Resolves DPEngine's extraction function to (pid, pk, value) column
    specs: ColumnRef, a constant, or None; returns None when it cannot.
    select_partitions extracts (pid, pk) only (dp_engine.py:241-244): value None."""
    try:
        out = extract_fn(_ProbeRow())
    except Exception:
        return None
    if isinstance(out, tuple) and len(out) == 2:
        out = out + (None,)
    if not isinstance(out, tuple) or len(out) != 3:
        return None
    specs = []
    for i, item in enumerate(out):
        if isinstance(item, ColumnRef):
            if not table.has_column(item.name):
                return None
            specs.append(item)
        elif item is None and i == 0:
            specs.append(None)
        elif i == 2 and (item is None or isinstance(item, (int, float, np.integer, np.floating))):
            specs.append(item)  # constant value (COUNT / PRIVACY_ID_COUNT only)
        else:
            return None
    return tuple(specs)


@dataclasses.dataclass
class EncodedKeys:
    codes: Any              # int64 numpy array or torch tensor (dense ids)
    n: int                  # dense range
    decode: Optional[np.ndarray]  # None = identity
    encode: Optional[dict] = None  # key -> code (factorised keys), for public partitions

    def key_of(self, code: int):
        return int(code) if self.decode is None else self.decode[code]


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def encode_keys(values, declared_n: Optional[int] = None) -> EncodedKeys:
    """Dense int64 ids for a key column (identity when already dense)."""
    if _is_torch(values):
        import torch
        if values.dtype not in (torch.int64, torch.int32):
            raise TypeError("device-resident key columns must be int32/int64 dense ids")
        t = values.to(torch.int64)
        if declared_n is None:
            if t.numel() == 0:
                return EncodedKeys(t, 1, None)
            mn, mx = torch.aminmax(t)
            if int(mn) < 0:
                raise ValueError("device-resident key columns must be non-negative dense ids")
            declared_n = int(mx) + 1
        return EncodedKeys(t.contiguous(), max(int(declared_n), 1), None)
    arr = np.asarray(values)
    n = len(arr)
    if arr.dtype.kind in "iu" and n > 0:
        mn, mx = int(arr.min()), int(arr.max())
        if mn >= 0 and mx < max(4 * n, 1 << 16) and (declared_n is None or mx < declared_n):
            return EncodedKeys(arr.astype(np.int64, copy=False), declared_n or mx + 1, None)
    if n == 0:
        return EncodedKeys(np.zeros(0, np.int64), 1, np.zeros(0, dtype=object), {})
    import pandas as pd
    codes, uniques = pd.factorize(arr if arr.dtype != object else pd.Series(list(values), dtype=object),
                                  sort=False)
    decode = np.asarray(uniques, dtype=object)
    return EncodedKeys(np.asarray(codes, dtype=np.int64), len(decode), decode,
                       {k: i for i, k in enumerate(decode)})


def extend_with_keys(enc: EncodedKeys, keys) -> (EncodedKeys, np.ndarray):
    """Adds keys (public partitions) to a dictionary; returns the new
    dictionary and the codes of `keys`."""
    keys = list(keys)
    if enc.decode is None:
        codes = []
        for k in keys:
            if isinstance(k, (int, np.integer)) and k >= 0:
                codes.append(int(k))
            else:
                break
        else:
            n = max([enc.n] + [c + 1 for c in codes])
            return EncodedKeys(enc.codes, n, None), np.asarray(codes, dtype=np.int64)
        # non-integer public keys: switch to an explicit dictionary
        decode = list(range(enc.n))
        mapping = {i: i for i in range(enc.n)}
        enc = EncodedKeys(enc.codes, enc.n, np.asarray(decode, dtype=object), mapping)
    mapping = dict(enc.encode or {})
    decode = list(enc.decode)
    codes = []
    for k in keys:
        c = mapping.get(k)
        if c is None:
            c = len(decode)
            mapping[k] = c
            decode.append(k)
        codes.append(c)
    return EncodedKeys(enc.codes, len(decode), np.asarray(decode, dtype=object), mapping), \
        np.asarray(codes, dtype=np.int64)
