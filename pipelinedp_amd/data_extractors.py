"""Data extractors (mirror of pipeline_dp/data_extractors.py:5-37) plus
ColumnExtractor, a callable that also names a column so that the columnar
backend can read whole columns instead of calling the extractor per row."""
import dataclasses
from typing import Callable


@dataclasses.dataclass
class DataExtractors:
    """Functions that, given an input row, return its privacy id, partition
    key and value."""
    privacy_id_extractor: Callable = None
    partition_extractor: Callable = None
    value_extractor: Callable = None


@dataclasses.dataclass
class PreAggregateExtractors:
    """Extractors for pre-aggregated rows (reference data_extractors.py:18-37)."""
    partition_extractor: Callable
    preaggregate_extractor: Callable


class ColumnExtractor:
    """row -> row[column] (mapping / sequence rows) or getattr(row, column)
    (object rows).  Row-wise it behaves like ``lambda row: row[column]``;
    ColumnarBackend reads the named column of a ColumnTable directly."""

    def __init__(self, column):
        self.column = column

    def __call__(self, row):
        try:
            return row[self.column]
        except (TypeError, KeyError, IndexError):
            return getattr(row, self.column)

    def __repr__(self):
        return f"ColumnExtractor({self.column!r})"
