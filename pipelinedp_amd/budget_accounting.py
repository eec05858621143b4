"""Privacy budget accounting (mirror of pipeline_dp/budget_accounting.py).

MechanismSpec (:40-111) is a lazy handle: eps/delta raise until
compute_budgets() has run, which is why the GPU path reads budgets at
execution (iteration) time, never while the graph is built.
NaiveBudgetAccountant (:301-408) splits (epsilon, delta) proportionally to
mechanism weights after scope normalisation (BudgetAccountantScope :273-298);
delta goes only to mechanisms that use it (everything but LAPLACE).
PLDBudgetAccountant (:411-619) needs dp-accounting and is out of scope.
"""
import abc
import collections
import dataclasses
import logging
from typing import Optional

from pipelinedp_amd import aggregate_params as agg


@dataclasses.dataclass
class MechanismSpec:
    mechanism_type: agg.MechanismType
    _noise_standard_deviation: float = None
    _eps: float = None
    _delta: float = None
    _count: int = 1

    @property
    def noise_standard_deviation(self):
        if self._noise_standard_deviation is None:
            raise AssertionError("Noise standard deviation is not calculated yet.")
        return self._noise_standard_deviation

    @property
    def eps(self):
        if self._eps is None:
            raise AssertionError("Privacy budget is not calculated yet.")
        return self._eps

    @property
    def delta(self):
        if self._delta is None:
            raise AssertionError("Privacy budget is not calculated yet.")
        return self._delta

    @property
    def count(self):
        return self._count

    def set_eps_delta(self, eps: float, delta: Optional[float]) -> None:
        if eps is None:
            raise AssertionError("eps must not be None.")
        self._eps = eps
        self._delta = delta

    def set_noise_standard_deviation(self, stddev: float):
        self._noise_standard_deviation = stddev

    def use_delta(self) -> bool:
        return self.mechanism_type != agg.MechanismType.LAPLACE

    @property
    def standard_deviation_is_set(self) -> bool:
        return self._noise_standard_deviation is not None


@dataclasses.dataclass
class MechanismSpecInternal:
    sensitivity: float
    weight: float
    mechanism_spec: MechanismSpec


Budget = collections.namedtuple("Budget", ["epsilon", "delta"])


class BudgetAccountantScope:
    """Normalises the weights of the mechanisms requested inside it so that
    they sum to the scope weight."""

    def __init__(self, accountant, weight):
        self.weight = weight
        self.accountant = accountant
        self.mechanisms = []

    def __enter__(self):
        self.accountant._enter_scope(self)
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        self.accountant._exit_scope()
        if self.mechanisms:
            factor = self.weight / sum(m.weight for m in self.mechanisms)
            for m in self.mechanisms:
                m.weight *= factor


class BudgetAccountant(abc.ABC):

    def __init__(self, total_epsilon: float, total_delta: float, num_aggregations: Optional[int],
                 aggregation_weights: Optional[list]):
        agg.validate_epsilon_delta(total_epsilon, total_delta, "BudgetAccountant")
        self._total_epsilon = total_epsilon
        self._total_delta = total_delta
        self._scopes_stack = []
        self._mechanisms = []
        self._finalized = False
        if num_aggregations is not None and aggregation_weights is not None:
            raise ValueError("'num_aggregations' and 'aggregation_weights' can not be set "
                             "simultaneously.")
        if num_aggregations is not None and num_aggregations <= 0:
            raise ValueError(f"'num_aggregations'={num_aggregations}, but it has to be positive.")
        self._expected_num_aggregations = num_aggregations
        self._expected_aggregation_weights = aggregation_weights
        self._actual_aggregation_weights = []

    @abc.abstractmethod
    def request_budget(self, mechanism_type: agg.MechanismType, sensitivity: float = 1,
                       weight: float = 1, count: int = 1,
                       noise_standard_deviation: Optional[float] = None) -> MechanismSpec:
        pass

    @abc.abstractmethod
    def compute_budgets(self):
        pass

    def scope(self, weight: float) -> BudgetAccountantScope:
        return BudgetAccountantScope(self, weight)

    def _compute_budget_for_aggregation(self, weight: float) -> Optional[Budget]:
        self._actual_aggregation_weights.append(weight)
        if self._expected_num_aggregations:
            n = self._expected_num_aggregations
            return Budget(self._total_epsilon / n, self._total_delta / n)
        if self._expected_aggregation_weights:
            ratio = weight / sum(self._expected_aggregation_weights)
            return Budget(self._total_epsilon * ratio, self._total_delta * ratio)
        return None

    def _check_aggregation_restrictions(self):
        actual = self._actual_aggregation_weights
        if self._expected_num_aggregations:
            if len(actual) != self._expected_num_aggregations:
                raise ValueError(f"'num_aggregations'({self._expected_num_aggregations}) in the "
                                 f"constructor of BudgetAccountant is different from the actual "
                                 f"number of aggregations in the pipeline({len(actual)}).")
            if not all(w == 1 for w in actual):
                raise ValueError(f"Aggregation weights = {actual}. If 'num_aggregations' is set "
                                 f"in the constructor of BudgetAccountant, all aggregation weights "
                                 f"have to be 1.")
        if self._expected_aggregation_weights:
            expected = self._expected_aggregation_weights
            if len(actual) != len(expected):
                raise ValueError(f"Length of 'aggregation_weights' in the constructor of "
                                 f"BudgetAccountant is {len(expected)} != {len(actual)} the actual "
                                 f"number of aggregations.")
            if any(a != e for a, e in zip(actual, expected)):
                raise ValueError(f"'aggregation_weights' ({expected}) is different from actual "
                                 f"aggregation weights ({actual}).")

    def _register_mechanism(self, mechanism: MechanismSpecInternal):
        self._mechanisms.append(mechanism)
        for scope in self._scopes_stack:
            scope.mechanisms.append(mechanism)
        return mechanism

    def _enter_scope(self, scope):
        self._scopes_stack.append(scope)

    def _exit_scope(self):
        self._scopes_stack.pop()

    def _finalize(self):
        if self._finalized:
            raise Exception("compute_budgets can not be called twice.")
        self._finalized = True


class NaiveBudgetAccountant(BudgetAccountant):
    """Naive composition: eps_i = eps * w_i / sum(w), delta likewise over the
    mechanisms that use delta."""

    def __init__(self, total_epsilon: float, total_delta: float,
                 num_aggregations: Optional[int] = None, aggregation_weights: Optional[list] = None):
        super().__init__(total_epsilon, total_delta, num_aggregations, aggregation_weights)

    def request_budget(self, mechanism_type: agg.MechanismType, sensitivity: float = 1,
                       weight: float = 1, count: int = 1,
                       noise_standard_deviation: Optional[float] = None) -> MechanismSpec:
        if self._finalized:
            raise Exception("request_budget() is called after compute_budgets(). Please ensure "
                            "that compute_budgets() is called after DP aggregations.")
        if noise_standard_deviation is not None:
            raise NotImplementedError("Count and noise standard deviation have not been "
                                      "implemented yet.")
        if mechanism_type == agg.MechanismType.GAUSSIAN and self._total_delta == 0:
            raise ValueError("The Gaussian mechanism requires that the pipeline delta is greater "
                             "than 0")
        spec = MechanismSpec(mechanism_type=mechanism_type, _count=count)
        self._register_mechanism(
            MechanismSpecInternal(mechanism_spec=spec, sensitivity=sensitivity, weight=weight))
        return spec

    def compute_budgets(self):
        self._check_aggregation_restrictions()
        self._finalize()
        if not self._mechanisms:
            logging.warning("No budgets were requested.")
            return
        if self._scopes_stack:
            raise Exception("Cannot call compute_budgets from within a budget scope.")
        w_eps = sum(m.weight * m.mechanism_spec.count for m in self._mechanisms)
        w_delta = sum(m.weight * m.mechanism_spec.count for m in self._mechanisms
                      if m.mechanism_spec.use_delta())
        for m in self._mechanisms:
            eps = self._total_epsilon * m.weight / w_eps if w_eps else 0
            delta = 0
            if m.mechanism_spec.use_delta() and w_delta:
                delta = self._total_delta * m.weight / w_delta
            m.mechanism_spec.set_eps_delta(eps, delta)


class PLDBudgetAccountant(BudgetAccountant):
    """Out of scope: needs the dp-accounting library (not available)."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError("PLDBudgetAccountant is not supported by pipelinedp_amd "
                                  "(needs dp_accounting); use NaiveBudgetAccountant")

    def request_budget(self, *args, **kwargs):
        raise NotImplementedError

    def compute_budgets(self):
        raise NotImplementedError
