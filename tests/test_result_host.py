"""AggregateResult: the columnar (pk, MetricsTuple) sequence ColumnarBackend
returns (CPU test; the reference yields (pk, MetricsTuple) tuples,
combiners.py:786-788)."""
import time

import numpy as np

from pipelinedp_amd import columnar as C
from pipelinedp_amd import combiners as pdc


def test_result_behaves_like_the_reference_list():
    nt = pdc._get_or_create_named_tuple("MetricsTuple", ("count", "sum"))
    res = C.AggregateResult(np.array([3, 7, 9]), {"count": np.array([1.5, 2.0, 3.0]),
                                                  "sum": np.array([10.0, 20.0, 30.0])}, nt)
    assert len(res) == 3
    assert list(res) == [(3, nt(1.5, 10.0)), (7, nt(2.0, 20.0)), (9, nt(3.0, 30.0))]
    assert res[1] == (7, nt(2.0, 20.0)) and res[-1][0] == 9
    assert res[0:2] == list(res)[0:2]
    assert dict(res)[9].sum == 30.0
    assert type(res[0][0]) is int and type(res[0][1].count) is float
    assert res.fields == ("count", "sum")
    t = res.to_arrow()
    assert t.column_names == ["partition_key", "count", "sum"] and t.num_rows == 3


def test_object_keys_and_empty():
    nt = pdc._get_or_create_named_tuple("MetricsTuple", ("mean",))
    res = C.AggregateResult(np.array(["a", ("b", 1)], dtype=object), {"mean": np.array([0.5, 1.5])}, nt)
    assert [k for k, _ in res] == ["a", ("b", 1)]
    empty = C.AggregateResult(np.zeros(0, np.int64), {"mean": np.zeros(0)}, nt)
    assert list(empty) == [] and len(empty) == 0


def test_ten_million_partitions_materialise_in_under_a_second():
    """verdict r1 item 8: C4-scale output (1e7 partitions) without a
    per-partition Python loop."""
    n = 10_000_000
    nt = pdc._get_or_create_named_tuple("MetricsTuple", ("variance", "count", "sum", "mean", "privacy_id_count"))
    vals = np.random.default_rng(0).random((5, n))
    enc = C.EncodedKeys(np.zeros(0, np.int64), n, None)
    t0 = time.perf_counter()
    res = C.AggregateResult(enc.keys_of(np.arange(n)), {f: vals[i] for i, f in enumerate(nt._fields)}, nt)
    assert len(res) == n and res[n - 1][0] == n - 1
    assert time.perf_counter() - t0 < 1.0
