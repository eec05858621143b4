"""Columnar input and ingest: ColumnTable, column probing, key encoding.

ColumnTable is the collection type the ColumnarBackend reads at HBM speed.
DataExtractors are resolved to columns by *probing*: the extraction function
DPEngine builds (dp_engine.py:402-415) is called once on a probe row whose
items/attributes are column references, so ``ColumnExtractor("user_id")``,
``lambda r: r[0]`` and ``lambda r: r.user_id`` all resolve without touching
the data.  Anything else is extracted row-wise on the host (ingest, not
compute) and then encoded.

Keys are dictionary-encoded to dense int64 ids: integer keys that are already
dense-ish are used as-is (identity dictionary); Arrow dictionary columns
(Parquet's own dictionary pages, `ColumnTable.from_parquet`) keep their codes;
other keys (strings, tuples, sparse integers) go through Arrow's
dictionary_encode or pandas.factorize.  The dictionary decodes output
partitions back to the user's keys.
"""
import dataclasses
from collections.abc import Sequence
from typing import Any, Mapping, Optional

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

    @classmethod
    def from_arrow(cls, table, columns: Optional[Sequence[str]] = None, **meta) -> "ColumnTable":
        """ColumnTable over a pyarrow Table / RecordBatch (the columnar ingest
        SURVEY §8(f) ranks next to the path).  Numeric columns without nulls
        become NumPy views of the Arrow buffers (zero-copy for single-chunk
        columns); dictionary columns become DictColumn (codes + dictionary,
        no re-hashing); string / binary columns are dictionary-encoded by
        Arrow (C++ hash) into DictColumn.  Nulls raise, as a None key or value
        would fail in the reference's extractors and combiners."""
        import pyarrow as pa
        import pyarrow.compute as pc
        names = list(columns) if columns is not None else list(table.column_names)
        cols = {}
        for name in names:
            col = table.column(name)
            if isinstance(col, pa.ChunkedArray):
                col = col.combine_chunks() if col.num_chunks != 1 else col.chunk(0)
            if col.null_count:
                raise ValueError(f"column {name!r} has {col.null_count} nulls")
            t = col.type
            if pa.types.is_dictionary(t):
                cols[name] = DictColumn.from_arrow(col)
            elif pa.types.is_string(t) or pa.types.is_large_string(t) or pa.types.is_binary(t):
                cols[name] = DictColumn.from_arrow(pc.dictionary_encode(col))
            elif pa.types.is_integer(t) or pa.types.is_floating(t) or pa.types.is_boolean(t):
                cols[name] = col.to_numpy(zero_copy_only=False)
            else:
                cols[name] = np.asarray(col.to_pylist(), dtype=object)
        return cls(cols, **meta)

    @classmethod
    def from_parquet(cls, path, columns: Optional[Sequence[str]] = None,
                     key_columns: Sequence[str] = (), **meta) -> "ColumnTable":
        """Reads Parquet columns; `key_columns` are read as Arrow dictionary
        arrays straight from Parquet's dictionary pages (no host hashing)."""
        import pyarrow.parquet as pq
        table = pq.read_table(path, columns=list(columns) if columns is not None else None,
                              read_dictionary=list(key_columns) or None)
        return cls.from_arrow(table, columns, **meta)

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


class DictColumn:
    """A dictionary-encoded column: int64 `codes` into `dictionary` (an
    object array of the keys).  Row-wise access decodes; encode_keys uses the
    codes as the dense ids directly."""
    __slots__ = ("codes", "dictionary")

    def __init__(self, codes, dictionary):
        self.codes = np.asarray(codes, dtype=np.int64)
        self.dictionary = np.asarray(dictionary, dtype=object)

    @classmethod
    def from_arrow(cls, arr):
        return cls(arr.indices.to_numpy(zero_copy_only=False).astype(np.int64, copy=False),
                   arr.dictionary.to_pylist())

    def __len__(self):
        return len(self.codes)

    def __getitem__(self, i):
        return self.dictionary[self.codes[i]]


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

    def keys_of(self, codes: np.ndarray) -> np.ndarray:
        """Vectorised key_of (int64 codes -> int64 keys or an object array)."""
        codes = np.asarray(codes, dtype=np.int64)
        return codes.copy() if self.decode is None else np.asarray(self.decode, dtype=object)[codes]


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


class AggregateResult(Sequence):
    """The output of DPEngine.aggregate on ColumnarBackend: a sequence of
    (partition_key, MetricsTuple) — the reference's element type
    (combiners.py:786-788) — held as columns.

    Nothing is built per partition until an element is read:
    `partition_keys` (a NumPy array) and `columns` (field name -> float64
    NumPy array, the MetricsTuple field order) are the materialised result;
    indexing / iterating yields the reference's tuples on demand.  Partitions
    come in ascending partition-code order (the reference's LocalBackend
    yields first-appearance order; compare by key)."""

    def __init__(self, partition_keys: np.ndarray, columns: dict, tuple_type):
        self.partition_keys = partition_keys
        self.columns = columns
        self._fields = tuple(columns)
        self._nt = tuple_type

    @property
    def fields(self):
        return self._fields

    def __len__(self):
        return len(self.partition_keys)

    def _row(self, i):
        return (_py_key(self.partition_keys[i]), self._nt(*(float(self.columns[f][i]) for f in self._fields)))

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._row(j) for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        return self._row(i)

    def __iter__(self):
        cols = [self.columns[f].tolist() for f in self._fields]
        keys = self.partition_keys.tolist()
        nt = self._nt
        return (( k, nt(*vals)) for k, *vals in zip(keys, *cols))

    def __eq__(self, other):
        return list(self) == list(other)

    def to_arrow(self):
        """pyarrow Table (partition_key + one column per metric)."""
        import pyarrow as pa
        return pa.table({"partition_key": pa.array(self.partition_keys.tolist()),
                         **{f: pa.array(v) for f, v in self.columns.items()}})

    def __repr__(self):
        return f"AggregateResult({len(self)} partitions, fields={self._fields})"


def _py_key(k):
    return k.item() if isinstance(k, np.generic) else k


def encode_keys(values, declared_n: Optional[int] = None) -> EncodedKeys:
    """Dense int64 ids for a key column (identity when already dense)."""
    if isinstance(values, DictColumn):
        # Arrow dictionaries may hold unused or repeated entries: compact to
        # the keys that occur, first-appearance order of the dictionary
        import pandas as pd
        if len(values.dictionary) == 0:
            return EncodedKeys(np.zeros(0, np.int64), 1, np.zeros(0, dtype=object), {})
        key_codes, uniques = pd.factorize(pd.Series(list(values.dictionary), dtype=object), sort=False)
        used = np.zeros(len(uniques), dtype=bool)
        remapped = key_codes[values.codes] if len(values.codes) else np.zeros(0, np.int64)
        used[remapped] = True
        dense = np.cumsum(used) - 1
        decode = np.asarray(uniques, dtype=object)[used]
        return EncodedKeys(dense[remapped].astype(np.int64), max(len(decode), 1), decode,
                           {k: i for i, k in enumerate(decode)})
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
