"""Histogram containers (mirror of pipeline_dp/dataset_histograms/
histograms.py): FrequencyBin (:21-57), HistogramType (:60-76), Histogram
(:79-162), compute_ratio_dropped (:165-204), DatasetHistograms (:207-216).
Same fields, equality and helper semantics, so code written against the
reference's objects reads these unchanged."""
import dataclasses
import enum
from typing import List, Optional, Sequence, Tuple, Union

Number = Union[int, float]


@dataclasses.dataclass
class FrequencyBin:
    """Bin [lower, upper) of a histogram (upper included only for the last
    bin of a float histogram) with the element count, sum and maximum."""
    lower: Number
    upper: Number
    count: int
    sum: Number
    max: Number

    def __add__(self, other: "FrequencyBin") -> "FrequencyBin":
        if self.lower != other.lower or self.upper != other.upper:
            raise AssertionError("bins with different bounds cannot be merged")
        return FrequencyBin(self.lower, self.upper, self.count + other.count, self.sum + other.sum,
                            max(self.max, other.max))

    def __eq__(self, other):
        # the reference compares lower, count, sum and max (histograms.py:51-53)
        return (self.lower, self.count, self.sum, self.max) == (other.lower, other.count, other.sum, other.max)


class HistogramType(enum.Enum):
    L0_CONTRIBUTIONS = "l0_contributions"
    L1_CONTRIBUTIONS = "l1_contributions"
    LINF_CONTRIBUTIONS = "linf_contributions"
    LINF_SUM_CONTRIBUTIONS = "linf_sum_contributions"
    COUNT_PER_PARTITION = "count_per_partition"
    COUNT_PRIVACY_ID_PER_PARTITION = "privacy_id_per_partition_count"
    SUM_PER_PARTITION = "sum_per_partition"


_FLOAT_TYPES = (HistogramType.LINF_SUM_CONTRIBUTIONS, HistogramType.SUM_PER_PARTITION)


@dataclasses.dataclass
class Histogram:
    """A histogram: its type and bins sorted by lower.  `lower` is 1 for
    integer histograms (None if empty); `upper` is the last bin's upper for
    float histograms, None for integer ones (no upper bound)."""
    name: HistogramType
    bins: List[FrequencyBin]
    lower: Optional[Number] = dataclasses.field(init=False)
    upper: Optional[Number] = dataclasses.field(init=False)

    def __post_init__(self):
        if not self.bins:
            self.lower = self.upper = None
        elif self.is_integer:
            self.lower, self.upper = 1, None
        else:
            self.lower, self.upper = self.bins[0].lower, self.bins[-1].upper

    @property
    def is_integer(self) -> bool:
        return self.name not in _FLOAT_TYPES

    def total_count(self):
        return sum(b.count for b in self.bins)

    def total_sum(self):
        return sum(b.sum for b in self.bins)

    def max_value(self):
        return self.bins[-1].max

    def quantiles(self, q: List[float]) -> List[Number]:
        """For each q, the lower of the first bin (scanning from the top)
        whose left part holds at most a q share of the elements
        (histograms.py:130-162)."""
        if sorted(q) != list(q):
            raise AssertionError("Quantiles to compute must be sorted.")
        total = self.total_count()
        if total == 0:
            raise ValueError("Cannot compute quantiles of an empty histogram")
        out = []
        smaller = total
        i = len(q) - 1
        for b in reversed(self.bins):
            smaller -= b.count
            ratio = smaller / total
            while i >= 0 and q[i] >= ratio:
                out.append(b.lower)
                i -= 1
        while i >= 0:  # unreachable: the first bin has ratio 0
            out.append(self.bins[0].lower)
            i -= 1
        return out[::-1]


def compute_ratio_dropped(contribution_histogram: Histogram) -> Sequence[Tuple[Number, float]]:
    """(threshold, share of the data dropped by bounding at threshold) for
    every bin lower plus the maximum, sorted, starting with (0, 1)
    (histograms.py:165-204)."""
    bins = contribution_histogram.bins
    if not bins:
        return []
    total = contribution_histogram.total_sum()
    out = []
    prev = bins[-1].lower
    if contribution_histogram.max_value() != prev:
        out.append((contribution_histogram.max_value(), 0.0))
    dropped = larger = 0
    for b in reversed(bins):
        dropped += larger * (prev - b.lower) + (b.sum - b.count * b.lower)
        out.append((b.lower, dropped / total))
        prev = b.lower
        larger += b.count
    out.append((0, 1))
    return out[::-1]


@dataclasses.dataclass
class DatasetHistograms:
    """The seven histograms of compute_dataset_histograms."""
    l0_contributions_histogram: Histogram
    l1_contributions_histogram: Histogram
    linf_contributions_histogram: Histogram
    linf_sum_contributions_histogram: Histogram
    count_per_partition_histogram: Histogram
    count_privacy_id_per_partition: Histogram
    sum_per_partition_histogram: Histogram
