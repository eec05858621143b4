"""Explain-computation reports (mirror of pipeline_dp/report_generator.py).

A report lists the aggregation parameters and the computation stages; stage
descriptions may be callables resolved after compute_budgets() (budgets are
not known while the graph is built)."""
from typing import Callable, Optional, Union

from pipelinedp_amd import aggregate_params as agg


class ReportGenerator:

    def __init__(self, params, method_name: str, is_public_partition: Optional[bool] = None):
        self._params_str = (agg.parameters_to_readable_string(params, is_public_partition)
                            if params else None)
        self._method_name = method_name
        self._stages = []

    def add_stage(self, stage_description: Union[Callable, str]) -> None:
        self._stages.append(stage_description)

    def report(self) -> str:
        if not self._params_str:
            return ""
        lines = [f"DPEngine method: {self._method_name}", self._params_str, "Computation graph:"]
        for i, stage in enumerate(self._stages, start=1):
            lines.append(f" {i}. {stage() if callable(stage) else stage}")
        return "\n".join(lines)


class ExplainComputationReport:
    """Holds the report of one aggregation; text() after compute_budgets()."""

    def __init__(self):
        self._report_generator = None

    def _set_report_generator(self, report_generator: ReportGenerator):
        self._report_generator = report_generator

    def text(self) -> str:
        if self._report_generator is None:
            raise ValueError("The report_generator is not set.\nWas this object passed as an "
                             "argument to DP aggregation method?")
        try:
            return self._report_generator.report()
        except Exception as e:
            raise ValueError("Explain computation report failed to be generated.\nWas "
                             "BudgetAccountant.compute_budget() called?") from e
