"""Columnar ingest: Arrow / Parquet columns into
ColumnTable, dictionary-encoded keys, and their equivalence with the row
input the reference consumes.  CPU-only: encoding and graph recognition;
the GPU run of the same tables is in test_gpu_api.py."""
import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")
pq = pytest.importorskip("pyarrow.parquet")

import pipelinedp_amd as pdp
from pipelinedp_amd import columnar as C
from pipelinedp_amd import columnar_backend as CB
from tests import golden_util as G


def _string_rows():
    fx = [f for f in G.fixtures() if f["name"] == "string_keys"][0]
    return fx, [tuple(r) for r in fx["rows"]]


def test_from_arrow_types():
    t = pa.table({"pid": pa.array(["u1", "u2", "u1"]), "pk": pa.array([3, 1, 3], pa.int64()),
                  "v": pa.array([1.5, 2.0, -1.0]),
                  "tag": pa.array(["a", "b", "a"]).dictionary_encode()})
    ct = C.ColumnTable.from_arrow(t)
    assert isinstance(ct.column("pid"), C.DictColumn) and isinstance(ct.column("tag"), C.DictColumn)
    assert ct.column("pk").dtype == np.int64 and ct.column("v").dtype == np.float64
    assert [tuple(r) for r in ct] == [("u1", 3, 1.5, "a"), ("u2", 1, 2.0, "b"), ("u1", 3, -1.0, "a")]


def test_from_arrow_rejects_nulls():
    with pytest.raises(ValueError):
        C.ColumnTable.from_arrow(pa.table({"pk": pa.array([1, None, 2])}))


def test_dict_column_encoding_equals_factorize():
    """Arrow dictionary codes (with unused and chunk-repeated dictionary
    entries) compact to the same dense dictionary as factorising the keys."""
    keys = ["b", "a", "b", "c", "a"]
    arr = pa.DictionaryArray.from_arrays(pa.array([1, 0, 1, 3, 0], pa.int32()),
                                         pa.array(["a", "b", "zz", "c"]))
    enc = C.encode_keys(C.DictColumn.from_arrow(arr))
    ref = C.encode_keys(np.asarray(keys, dtype=object))
    assert enc.n == 3 and sorted(enc.decode.tolist()) == ["a", "b", "c"]
    assert [enc.key_of(c) for c in enc.codes] == keys == [ref.key_of(c) for c in ref.codes]


def test_parquet_round_trip_and_recognition(tmp_path):
    fx, rows = _string_rows()
    path = tmp_path / "rows.parquet"
    pq.write_table(pa.table({"pid": [r[0] for r in rows], "pk": [r[1] for r in rows],
                             "v": [float(r[2]) for r in rows]}), path)
    ct = C.ColumnTable.from_parquet(path, key_columns=["pid", "pk"])
    assert isinstance(ct.column("pk"), C.DictColumn)
    assert [tuple(r) for r in ct] == [(r[0], r[1], float(r[2])) for r in rows]
    # DataExtractors resolve to the columns without touching rows
    acc = pdp.NaiveBudgetAccountant(total_epsilon=1.0, total_delta=1e-6)
    engine = pdp.DPEngine(acc, CB.ColumnarBackend())
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM], noise_kind=pdp.NoiseKind.LAPLACE,
                                 max_partitions_contributed=2, max_contributions_per_partition=2,
                                 min_value=0.0, max_value=3.0)
    ext = pdp.DataExtractors(privacy_id_extractor=pdp.ColumnExtractor("pid"),
                             partition_extractor=pdp.ColumnExtractor("pk"),
                             value_extractor=pdp.ColumnExtractor("v"))
    sink = engine.aggregate(ct, params, ext)
    acc.compute_budgets()
    plan = CB.recognise(sink)
    specs = C.probe_columns(plan.extract_fn, plan.source)
    assert [s.name for s in specs] == ["pid", "pk", "v"]
    enc = C.encode_keys(ct.column("pk"))
    assert set(enc.decode.tolist()) == {r[1] for r in rows}
