"""PipelineBackend interface (mirror of pipeline_dp/pipeline_backend.py:38-195)
and the annotation hook (:826-851).

DPEngine drives every backend through these operations; each takes a
collection and a stage name and returns a new collection.  The MI355X
implementation is pipelinedp_amd.columnar_backend.ColumnarBackend, a drop-in
for the reference's LocalBackend on the DPEngine.aggregate path.
"""
import abc
from typing import Callable, Iterable


class PipelineBackend(abc.ABC):
    """Operations the DP engine composes (same names and argument meaning as
    the reference; the reference's LocalBackend/Beam/Spark implement them
    row-wise)."""

    def to_collection(self, collection_or_iterable, col, stage_name: str):
        return collection_or_iterable

    def to_multi_transformable_collection(self, col):
        return col

    @abc.abstractmethod
    def map(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def map_with_side_inputs(self, col, fn, side_input_cols, stage_name: str):
        pass

    @abc.abstractmethod
    def flat_map(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def map_tuple(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def map_values(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def group_by_key(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def filter(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def filter_by_key(self, col, keys_to_keep, stage_name: str):
        """Keeps (key, data) elements whose key is in keys_to_keep."""

    @abc.abstractmethod
    def keys(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def values(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def sample_fixed_per_key(self, col, n: int, stage_name: str):
        """(key, value) -> (key, [<= n values sampled without replacement])."""

    @abc.abstractmethod
    def count_per_element(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def sum_per_key(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def combine_accumulators_per_key(self, col, combiner, stage_name: str):
        """(key, accumulator) -> (key, merged accumulator) per key."""

    @abc.abstractmethod
    def reduce_per_key(self, col, fn: Callable, stage_name: str):
        pass

    @abc.abstractmethod
    def flatten(self, cols: Iterable, stage_name: str):
        pass

    @abc.abstractmethod
    def distinct(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def to_list(self, col, stage_name: str):
        pass

    def annotate(self, col, stage_name: str, **kwargs):
        """Annotation hook, called once per aggregation (no-op by default)."""
        return col


class Annotator(abc.ABC):
    """Hook called once per DP aggregation with its params and budget."""

    @abc.abstractmethod
    def annotate(self, col, backend: PipelineBackend, stage_name: str, **kwargs):
        pass


_annotators = []


def register_annotator(annotator: Annotator):
    _annotators.append(annotator)
