"""pipelinedp_amd — MI355X-native DPEngine.aggregate hot path.

Mirrors the public API of PipelineDP (pipeline_dp 0.2.2rc2) for the aggregate
path — DPEngine, AggregateParams, DataExtractors, NaiveBudgetAccountant,
Metrics, NoiseKind, PartitionSelectionStrategy, ... — and adds
ColumnarBackend, a PipelineBackend that executes DPEngine.aggregate on the GPU
through hand-written HIP kernels (pipelinedp_amd/csrc, C ABI in
include/pipelinedp_amd.h).  ColumnarBackend also plugs into the reference's
own pipeline_dp.DPEngine.
"""
from pipelinedp_amd.aggregate_params import (AddDPNoiseParams, AggregateParams, MechanismType, Metric,
                                             Metrics, NoiseKind, NormKind, PartitionSelectionStrategy,
                                             SelectPartitionsParams)
from pipelinedp_amd.budget_accounting import (BudgetAccountant, MechanismSpec, NaiveBudgetAccountant,
                                              PLDBudgetAccountant)
from pipelinedp_amd.columnar import ColumnTable, DictColumn
from pipelinedp_amd.columnar_backend import ColumnarBackend
from pipelinedp_amd.combiners import Combiner, CustomCombiner
from pipelinedp_amd.data_extractors import ColumnExtractor, DataExtractors, PreAggregateExtractors
from pipelinedp_amd.dp_engine import DPEngine
from pipelinedp_amd.pipeline_backend import Annotator, PipelineBackend, register_annotator
from pipelinedp_amd.report_generator import ExplainComputationReport

__version__ = "0.1.0"
